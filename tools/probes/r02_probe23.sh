#!/bin/bash
# transcript form x batches in flight (lane form: fewest issue slots, longest chain)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe23
mkdir -p $O
run() {
  local name=$1 inf=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --quick --steps 60 --inflight $inf > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'])" >> $O/summary.txt
}
for i in 1 2; do
  run quad2_$i 2 P2V_TRANSCRIPT=quad
  run lane3_$i 3 P2V_TRANSCRIPT=lane
  run lane4_$i 4 P2V_TRANSCRIPT=lane
  run quad3_$i 3 P2V_TRANSCRIPT=quad
done
echo done
