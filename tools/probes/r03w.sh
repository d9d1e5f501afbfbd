# the interleaved latency / batch mode test, the ragged and lookup cases beside it
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "interleaved or ragged or lookup_circuits" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
