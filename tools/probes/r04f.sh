# round 4: ADVICE r3 fixes (lookahead in latency mode with traces, batch shapes past the limit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "lookahead or shape or latency" > $O/tests.log 2>&1; rc=$?
tail -12 $O/tests.log
exit $rc
