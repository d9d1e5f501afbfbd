#!/bin/bash
# k_status at priority 3 (this build) with side-stream order / queue priority variants, alternated
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe21
mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --quick --steps 60 > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'])" >> $O/summary.txt
}
for i in 1 2 3; do
  run base$i P2V_X=0
  run frifirst$i P2V_FRI_FIRST=1
  run sideprio$i P2V_SIDE_PRIO=1
  run both$i P2V_FRI_FIRST=1 P2V_SIDE_PRIO=1
done
echo done
