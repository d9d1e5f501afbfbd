#!/bin/bash
# round 6 final build: tools/profile_round.sh r06n (kernel stats, FETCH / WRITE / VALU PMC passes, the C3
# passes: the tag bench.py reads), then the default bench line with every leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 bash tools/profile_round.sh r06n > gpurun_out/r06n_profile.log 2>&1 || { tail -20 gpurun_out/r06n_profile.log; exit 1; }
tail -1 gpurun_out/r06n_profile.log
# the vanishing kernels' traffic with no chain kernel beside them (one stream): is their 2.4x the
# L2 turnover of the concurrent k_merkle_cse, or their own re-reads?
P2V_SINGLE_STREAM=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_r06n/pmc_fetch_single -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> gpurun_out/prof_r06n/pmc_fetch_single.err || { tail -5 gpurun_out/prof_r06n/pmc_fetch_single.err; exit 1; }
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['c5']['value'], d['c3']['value'], d['dropin']['n1']['warm'], d['cpu_baseline']['value'], d['roofline']['kernels']['step_ratio'], d['roofline']['traffic_source'])"
echo done
