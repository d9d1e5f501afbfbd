# the whole GPU suite on the final tree, as the driver runs it at round end
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
