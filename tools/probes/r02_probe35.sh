#!/bin/bash
# final code: batches in flight 2 vs 3, alternated (information for the next round)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe35
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --quick --steps 100 "$@" > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'])" >> $O/summary.txt
}
for i in 1 2; do
  run inf2_$i --inflight 2
  run inf3_$i --inflight 3
done
echo done
