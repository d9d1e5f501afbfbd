#!/bin/bash
# The quad (and pair) transcript's S-box as the asm-block multiply of lposeidon.h (one statement per
# multiply: P2V_QUAD_SBOX=1, now the default) against p2::sbox_lat (variant quad0): quad chain
# latency, the transcript-forms parity tests, and the quick 4096-proof line alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g
mkdir -p $O
L0=plonky2-verifier_amd/libp2v.so
L1=plonky2-verifier_amd/variants/libp2v_quad0.so
for r in 1 2; do
  for b in q1 q0; do
    echo "perm_bench_$b" >> $O/quad_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_$b 1 1000 9 >> $O/quad_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_$b 4096 100 9 >> $O/quad_chain.txt
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "transcript or latency or golden or permutation" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['serial'].get('ms_per_step'), d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
run q1_1 $L0 "$Q" && run q0_1 $L1 "$Q" && run q1_2 $L0 "$Q" && run q0_2 $L1 "$Q" && run q1_3 $L0 "$Q" && run q0_3 $L1 "$Q" || exit 1
run pair1 $L0 "$Q --transcript pair" && run pair0 $L1 "$Q --transcript pair" || exit 1
echo done
