#!/bin/bash
# final-code evidence of the session: full GPU suite, smoke, full default bench line, profiles (r02h)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe32
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python3 bench.py > $O/bench_default.json 2> $O/bench.err

echo done
