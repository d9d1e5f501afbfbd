#!/bin/bash
# round 6: the Merkle slot's small launches beside the other batch: k_merkle_fix on 256 blocks (default,
# lane form for long lists) against 1024 (variants/libp2v_fix1024.so), and k_merkle_plan in 256-thread
# work-groups (variants/libp2v_plan4.so) against 1024; the garbage-batch / Merkle tests; quick lines
# alternated; a pipelined kernel trace of the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "garbage or merkle_shared or top_level" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/plonky2-verifier_amd/variants
for i in 1 2; do
  for v in default fix1024 plan4; do
    if [ $v = default ]; then L="X=0"; else L="P2V_LIB=$V/libp2v_$v.so"; fi
    env $L timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 > $O/quick_${v}_$i.json 2> $O/quick_${v}_$i.err || { tail -5 $O/quick_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/quick_${v}_$i.json'));print('$v', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'].get('k_merkle'), d['verified_steps'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick > $O/bench_under_trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
grep -E "merkle|phase1|status" $O/trace/run_kernel_stats.csv | cut -d, -f1-4
echo done
