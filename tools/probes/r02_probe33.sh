#!/bin/bash
# fused k_phase1 vs split (k_transcript on the side stream + k_leaf at its own occupancy), final code
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe33
mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --quick --steps 60 > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'], d['kernel_ms'])" >> $O/summary.txt
}
for i in 1 2 3; do
  run fused$i P2V_X=0
  run split$i P2V_PHASE1=split
done
echo done
