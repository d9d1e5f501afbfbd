#!/bin/bash
# round 6: the lane-form transcript on the lookahead stream (half the quad's VALU instructions, a ~6 ms
# chain that must run ahead of its batch) at several in-flight depths and hardware-queue counts,
# against the default; quick lines, one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06k
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['clock']['step_ms']['mean'])"
}
run default
run lane_la_if2 --lookahead 1 --transcript lane --inflight 2
run lane_la_if3_q4 --lookahead 1 --transcript lane --inflight 3
run lane_la_if3_q16 --lookahead 1 --transcript lane --inflight 3 --hw-queues 16
run lane_la_if4_q16 --lookahead 1 --transcript lane --inflight 4 --hw-queues 16
run quad_la_if2 --lookahead 1 --inflight 2
run default2
echo done
