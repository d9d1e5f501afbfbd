#!/bin/bash
# round 6 final build: tools/profile_round.sh r06n (kernel stats, FETCH / WRITE / VALU PMC passes, the C3
# passes: the tag bench.py reads), then the default bench line with every leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 bash tools/profile_round.sh r06n > gpurun_out/r06n_profile.log 2>&1 || { tail -20 gpurun_out/r06n_profile.log; exit 1; }
tail -1 gpurun_out/r06n_profile.log
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['c5']['value'], d['c3']['value'], d['dropin']['n1']['warm'], d['cpu_baseline']['value'], d['roofline']['kernels']['step_ratio'], d['roofline']['traffic_source'])"
echo done
