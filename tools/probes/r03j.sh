# row-form Merkle paths in latency mode: full GPU suite, small-batch latency, quick line
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for b in 1 64 256 1024; do
  timeout -k 10 200 python3 bench.py --quick --batch $b --inflight 1 --steps 200 --warmup 10 > $O/lat_b$b.json 2> $O/lat_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/lat_b$b.json'));print('batch $b: serial ms/step', d['serial']['ms_per_step'], 'kernel_ms', d['kernel_ms'])"
done
timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/bench_quick.json 2> $O/bench_quick.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_quick.json'));print('quick', d['value'],d['serial']['value'],d['verified_all'])"
