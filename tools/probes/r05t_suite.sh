#!/bin/bash
# the whole GPU suite on the final round-5 tree, as the driver runs it at round end
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
