#!/bin/bash
# round 6: on the final kernels, the transcript forms and in-flight depths against the default
# (quad transcript fused in k_phase1, two batches in flight), and the exclusive-SIMD transcript
# (P2V_PHASE1=excl); quick lines, one box, default first and last
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06f
mkdir -p $O
run() {   # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['kernel_ms'].get('k_phase1'), d['kernel_ms'].get('k_transcript'))"
}
run default X=0
run lane_la_if3 X=0 --lookahead 1 --transcript lane --inflight 3 --hw-queues 8
run lane_la_if4 X=0 --lookahead 1 --transcript lane --inflight 4 --hw-queues 8
run pair X=0 --transcript pair
run if3_hwq8 X=0 --inflight 3 --hw-queues 8
run excl P2V_PHASE1=excl
run default2 X=0
echo done
