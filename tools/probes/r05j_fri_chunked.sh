#!/bin/bash
# combineInitial in chunks of 8 with unreduced product sums (P2V_FRI_CHUNKED=1, default) against the
# round-4 per-word F^2 Horner (variant fri0): the parity tests that compare every query's
# combineInitial value with the oracle, then the quick line alternated (k_fri's serial time)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05j
mkdir -p $O
L0=plonky2-verifier_amd/libp2v.so
L1=plonky2-verifier_amd/variants/libp2v_fri0.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "oracle or golden or ext_conventions or shape_variants" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
run c1_1 $L0 "$Q" && run c0_1 $L1 "$Q" && run c1_2 $L0 "$Q" && run c0_2 $L1 "$Q" && run c1_3 $L0 "$Q" && run c0_3 $L1 "$Q" || exit 1
echo done
