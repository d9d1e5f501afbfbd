#!/bin/bash
# staggered workspaces (p2v_verifier_chain) vs lockstep, 2 and 3 in flight
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe26
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --quick --steps 60 "$@" > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'])" >> $O/summary.txt
}
timeout -k 10 200 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "chained or transcript_forms" > $O/gpu_tests.log 2>&1
for i in 1 2; do
  run lock2_$i --stagger 0
  run stag2_$i --stagger 1
  run stag3_$i --stagger 1 --inflight 3
done
echo done
