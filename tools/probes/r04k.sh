# round 4: lane-form transcript (1 lane per proof, a third of the quad's instructions, longer chain) with more batches in flight
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "transcript_forms" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, args
  timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 $2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['kernel_ms'].get('k_phase1'))" | tee -a $O/bench.txt
}
run quad_i2 "" || exit 1
run lane_i2 "--transcript lane" || exit 1
run lane_i3 "--transcript lane --inflight 3" || exit 1
run lane_i4 "--transcript lane --inflight 4" || exit 1
run lane_i4_ss "--transcript lane --inflight 4 --single-stream" || exit 1
run lane_i3_q8 "--transcript lane --inflight 3 --hw-queues 8" || exit 1
run lane_i4_q8 "--transcript lane --inflight 4 --hw-queues 8" || exit 1
run quad_i3_q8 "--inflight 3 --hw-queues 8" || exit 1
run quad_i2_b2 "" || exit 1
