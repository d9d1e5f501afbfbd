#!/bin/bash
# transcript forms against batches in flight on the final round-5 code (shared-node Merkle paths):
# the default (quad at 4096 proofs, two in flight) against the lane / pair forms at two and three
# in flight (8 hardware queues for three), quick line, 100 steps, two rounds alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zc
mkdir -p $O
run() {  # name, args
  timeout -k 10 300 python3 bench.py --quick --no-c3 $2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
for r in 1 2; do
  run def_$r "$Q" || exit 1
  run lane2_$r "$Q --transcript lane" || exit 1
  run lane3_$r "$Q --transcript lane --inflight 3 --hw-queues 8" || exit 1
  run pair2_$r "$Q --transcript pair" || exit 1
  run pair3_$r "$Q --transcript pair --inflight 3 --hw-queues 8" || exit 1
done
echo done
