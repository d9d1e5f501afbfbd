# round 4: lane-form transcript with the lookahead stream (the chain runs ahead across steps), 8 hardware queues
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n
mkdir -p $O
run() {  # name, args
  timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 $2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['kernel_ms'])" | tee -a $O/bench.txt
}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "lookahead" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run quad "" || exit 1
run quad_la_q8 "--lookahead 1 --hw-queues 8" || exit 1
run lane_la_q8 "--transcript lane --lookahead 1 --hw-queues 8" || exit 1
run lane_la_q8_i3 "--transcript lane --lookahead 1 --hw-queues 8 --inflight 3" || exit 1
run lane_la_q12_i4 "--transcript lane --lookahead 1 --hw-queues 12 --inflight 4" || exit 1
run quad_b "" || exit 1
