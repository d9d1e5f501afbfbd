# Merkle top-level sharing: quick line with and without it (P2V_MTOP_K), alternated, then a serial kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f
mkdir -p $O
for k in 5 0 5 0 4; do
  P2V_MTOP_K=$k timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/bench_k$k.json 2> $O/bench_k$k.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_k$k.json'));print('K=$k', d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_serial -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 > $O/bench_under_trace_serial.json 2> $O/trace_serial.err
cat $O/trace_serial/run_kernel_stats.csv
