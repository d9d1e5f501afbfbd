# latency mode with the coset / misc vanishing kernels on a third stream: GPU suite, then batch 1 / 8 / 64 latency
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for b in 1 1 8 64; do
  timeout -k 10 200 python3 bench.py --quick --batch $b --inflight 1 --steps 200 --warmup 10 > $O/lat_b$b.json 2> $O/lat_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/lat_b$b.json'));print('batch $b: serial ms/step', d['serial']['ms_per_step'], d['serial'].get('kernel_ms'))"
done
