#!/bin/bash
# upper bound of the vanishing kernels' tail: a measurement-only variant build that can skip them
# (statuses still check: the workspace keeps the warm-up's vanishing results)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe24
mkdir -p $O
export P2V_LIB=$GRAFT_REPO_ROOT/plonky2-verifier_amd/variants/libp2v_novan.so
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --quick --steps 60 > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'], d['kernel_ms'])" >> $O/summary.txt
}
for i in 1 2; do
  run base$i P2V_X=0
  run novan$i P2V_MEASURE_NO_VANISH=1
done
echo done
