# round 4: transcript forms on large launches (C5: 131072 proofs per launch), quad vs lane vs pair
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m
mkdir -p $O
for form in quad lane pair quad; do
  P2V_TRANSCRIPT=$form timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$form.json 2> $O/b_$form.err || { tail -3 $O/b_$form.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$form.json'));print('$form', d['value'], 'c5', d['c5']['value'], d['c5']['verified_all'], 'c3', d['c3']['value'])" | tee -a $O/bench.txt
done
