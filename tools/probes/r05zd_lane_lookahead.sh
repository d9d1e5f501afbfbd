#!/bin/bash
# the lane and pair transcripts on the lookahead stream (its chain off the batch's critical path) at three and
# four batches in flight, against the default, on the final round-5 code; quick line, 100 steps,
# two rounds alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zd
mkdir -p $O
run() {  # name, args
  timeout -k 10 300 python3 bench.py --quick --no-c3 $2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
for r in 1 2; do
  run def_$r "$Q" || exit 1
  run la3_$r "$Q --transcript lane --lookahead 1 --inflight 3 --hw-queues 12" || exit 1
  run la4_$r "$Q --transcript lane --lookahead 1 --inflight 4 --hw-queues 12" || exit 1
  run pla2_$r "$Q --transcript pair --lookahead 1 --hw-queues 12" || exit 1
  run pla3_$r "$Q --transcript pair --lookahead 1 --inflight 3 --hw-queues 12" || exit 1
done
echo done
