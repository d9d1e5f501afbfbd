#!/bin/bash
# round 5, re-entry: the tree rebuilt in a fresh container — GPU suite, smoke and the driver's bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05za
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));print(d['value'],d['ms_per_step'],d.get('verified_steps'))"
echo done
