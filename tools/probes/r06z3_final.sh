#!/bin/bash
# round 6, the final tree as committed (library rebuilt from the same sources, src 41f01fe3f29df2f9):
# the whole GPU suite, smoke, the driver's command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06z3
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_1.json 2> $O/driver_cmd_1.err || { tail -20 $O/driver_cmd_1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd_1.json'));print('driver', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['build']['src_hash_built'], d['build']['match'])"
echo done
