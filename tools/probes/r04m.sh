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
# VALU / SALU instruction counts of the transcript forms (k_leaf from the split run separates the leaf part)
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES"
P2V_PHASE1=split timeout -s KILL 90 rocprofv3 --pmc $C -T --output-format csv -d $O/pmc_split -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_split.err || exit 1
for form in pair lane; do
  P2V_TRANSCRIPT=$form timeout -s KILL 90 rocprofv3 --pmc $C -T --output-format csv -d $O/pmc_$form -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_$form.err || exit 1
done
echo pmc done
