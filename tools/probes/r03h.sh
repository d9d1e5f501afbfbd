# one-proof latency (serial steps of small batches), the K = 3 / 2 Merkle sharing variants, then the round's
# profile collection on the current code and the full default line
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
for b in 1 64 256 1024; do
  timeout -k 10 200 python3 bench.py --quick --batch $b --inflight 1 --steps 200 --warmup 10 > $O/lat_b$b.json 2> $O/lat_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/lat_b$b.json'));print('batch $b: serial ms/step', d['serial']['ms_per_step'], 'kernel_ms', d['kernel_ms'])"
done
for k in 3 2 0; do
  P2V_MTOP_K=$k timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/bench_k$k.json 2> $O/bench_k$k.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_k$k.json'));print('K=$k', d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
done
bash tools/profile_round.sh r03h || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'],d['serial']['value'],d['c5']['value'],d['verified_all'])"
