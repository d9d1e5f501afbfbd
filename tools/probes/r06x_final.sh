#!/bin/bash
# round 6, final library (row form: chain rows on idle lanes, split S-boxes; quad form: split chain
# S-boxes): the whole GPU suite, smoke, the driver's command twice, tools/profile_round.sh r06x
# (the tag the bench line reads), the default line with every leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_$i.json 2> $O/driver_cmd_$i.err || { tail -20 $O/driver_cmd_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print('driver', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['build']['src_hash_built'], d['build']['match'])"
done
timeout -k 10 700 bash tools/profile_round.sh r06x > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -1 $O/profile.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['c5']['value'], d['c3']['value'], d['dropin']['n1']['warm'], d['dropin']['n64']['warm'], d['cpu_baseline']['value'])"
echo done
