#!/bin/bash
# scheduling of the two in-flight batches: side-stream priority, 3 in flight
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe20
mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --quick --steps 60 > $O/$name.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['serial']['value'])" >> $O/summary.txt
}
run base P2V_X=0
run sideprio P2V_SIDE_PRIO=1
run base2 P2V_X=0
run sideprio2 P2V_SIDE_PRIO=1
P2V_X=0 timeout -k 10 300 python3 bench.py --quick --steps 60 --inflight 3 > $O/inflight3.json 2>> $O/bench.err
python3 -c "import json; d=json.load(open('$O/inflight3.json')); print('inflight3', d['value'])" >> $O/summary.txt
P2V_SIDE_PRIO=1 timeout -k 10 300 python3 bench.py --quick --steps 60 --inflight 3 > $O/inflight3_sp.json 2>> $O/bench.err
python3 -c "import json; d=json.load(open('$O/inflight3_sp.json')); print('inflight3_sideprio', d['value'])" >> $O/summary.txt
echo done
