# latency mode (one-wave groups for k_merkle / k_fri, k_fri on its own stream below 2048 proofs):
# small-batch serial latency; then K = 2 Merkle sharing against off, alternated; GPU tests touched
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "matches_oracle_status or real_circuits or merkle_shared or multi_device or async" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for b in 1 64 1024; do
  timeout -k 10 200 python3 bench.py --quick --batch $b --inflight 1 --steps 200 --warmup 10 > $O/lat_b$b.json 2> $O/lat_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/lat_b$b.json'));print('batch $b: serial ms/step', d['serial']['ms_per_step'], 'kernel_ms', d['kernel_ms'])"
done
for k in 2 0 2 0 2 0; do
  P2V_MTOP_K=$k timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/bench_k$k.json 2> $O/bench_k$k.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_k$k.json'));print('K=$k', d['value'],d['serial']['value'],d['verified_all'])"
done
