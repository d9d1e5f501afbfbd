#!/bin/bash
# round 5, final tree after the re-entry experiments (sources as r05za): GPU suite, smoke, the driver's bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zf
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));print(d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'])"
echo done
