#!/bin/bash
# round 6: the C3 leg as the first bench process on a fresh box, with 4 untimed passes (C3_WARM)
# (r06t: with 2, the first reading was ~0.97 M against ~1.20 M for every later one)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06z2
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-c5 --no-cpu-baseline --no-host-legs --steps 20 > $O/run_$r.json 2> $O/run_$r.err || { tail -20 $O/run_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/run_$r.json'));c=d['c3'];print('run', $r, d['value'], d['clock']['run_clock']['clock_ghz'], c['value'], c['seconds'], c['verified_all'])" | tee -a $O/c3_first.txt
done
echo done
