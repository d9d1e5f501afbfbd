#!/bin/bash
# round 6: the library with the split uniform S-box (P2V_ROW_SBOX2=1) and the Makefile header dependencies: the whole
# GPU suite, smoke, the driver's command, the default line (drop-in latency legs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_1.json 2> $O/driver_cmd_1.err || { tail -20 $O/driver_cmd_1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd_1.json'));print('driver', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['build']['src_hash_built'], d['build']['match'])"
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['c5']['value'], d['c3']['value'], json.dumps(d['dropin']))"
echo done
