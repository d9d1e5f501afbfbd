#!/bin/bash
# round 2 of the shared-node Merkle path (work-group-aggregated bucket counts, per-follower flags,
# k_merkle_fix): a serial kernel trace, the full GPU suite, the quick line alternated against
# P2V_MERKLE_CSE=0 and against the variant that re-runs (A)/(C)-failing followers inline (variants/libp2v_inl.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick --no-c3 --inflight 1 > $O/bench_trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
cut -d, -f1-4 $O/trace/run_kernel_stats.csv | head -14
P2V_LIB=plonky2-verifier_amd/variants/libp2v_inl.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_inl -o run -- python3 bench.py --steps 10 --warmup 2 --quick --no-c3 --inflight 1 > $O/bench_trace_inl.json 2> $O/trace_inl.err || { tail -5 $O/trace_inl.err; exit 1; }
cut -d, -f1-4 $O/trace_inl/run_kernel_stats.csv | head -14
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cse, args, lib
  P2V_LIB=$4 P2V_MERKLE_CSE=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_all'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
L0=plonky2-verifier_amd/libp2v.so
LI=plonky2-verifier_amd/variants/libp2v_inl.so
run c1_1 1 "$Q" $L0 && run ci_1 1 "$Q" $LI && run c0_1 0 "$Q" $L0 && run c1_2 1 "$Q" $L0 && run ci_2 1 "$Q" $LI && run c0_2 0 "$Q" $L0 || exit 1

echo done
