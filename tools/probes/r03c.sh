set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03c
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03c/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03c/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03c/gpu_tests.log
timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > gpurun_out/r03c/bench_quick.json 2> gpurun_out/r03c/bench_quick.err
python3 -c "import json;d=json.load(open('gpurun_out/r03c/bench_quick.json'));print(d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r03c/trace_serial -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 > gpurun_out/r03c/bench_under_trace_serial.json 2> gpurun_out/r03c/trace_serial.err
cat gpurun_out/r03c/trace_serial/run_kernel_stats.csv
