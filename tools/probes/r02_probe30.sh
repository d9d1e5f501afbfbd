#!/bin/bash
# k_merkle at 6 waves per SIMD (variant build) vs the default 5, alternated
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe30
mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --quick --steps 60 > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'], d['kernel_ms']['k_merkle'])" >> $O/summary.txt
}
for i in 1 2 3; do
  run base$i P2V_X=0
  run m6_$i P2V_LIB=$GRAFT_REPO_ROOT/plonky2-verifier_amd/variants/libp2v_m6.so
done
echo done
