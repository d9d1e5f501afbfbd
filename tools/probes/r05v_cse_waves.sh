#!/bin/bash
# k_merkle_cse occupancy: 6 waves per SIMD (default, 80 VGPRs, 40 B of spills outside the chain
# loop) against 5 (variants/libp2v_cse5.so: 83 VGPRs, no spills), alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v
mkdir -p $O
run() {  # name, lib
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 --steps 100 --warmup 5 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_all'], d['kernel_ms'])" | tee -a $O/bench.txt
}
L6=plonky2-verifier_amd/libp2v.so
L5=plonky2-verifier_amd/variants/libp2v_cse5.so
for r in 1 2 3; do run w6_$r $L6 && run w5_$r $L5 || exit 1; done
echo done
