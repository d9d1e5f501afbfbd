#!/bin/bash
# Batches in flight x hardware queues per process on the shared-node Merkle code (quad transcript):
# 2 (default) vs 3 / 4 with GPU_MAX_HW_QUEUES=8 (each workspace holds a main and a side stream),
# alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05r
mkdir -p $O
run() {  # name, args
  timeout -k 10 300 python3 bench.py --quick --no-c3 $2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
for r in 1 2; do
  run def_$r "$Q" || exit 1
  run if3_$r "$Q --inflight 3 --hw-queues 8" || exit 1
  run if4_$r "$Q --inflight 4 --hw-queues 8" || exit 1
  run def8_$r "$Q --hw-queues 8" || exit 1
done
echo done
