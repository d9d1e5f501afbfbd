# Merkle top-level sharing, parallel checks: targeted GPU tests, quick line on/off alternated, serial trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "merkle_shared or real_circuits or random_number or matches_oracle_status" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for k in 5 0 5 0; do
  P2V_MTOP_K=$k timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/bench_k$k.json 2> $O/bench_k$k.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_k$k.json'));print('K=$k', d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_serial -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 > $O/bench_under_trace_serial.json 2> $O/trace_serial.err
cat $O/trace_serial/run_kernel_stats.csv
