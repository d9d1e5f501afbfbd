#!/bin/bash
# MDS MADs in plain C (P2V_MADK_C=1: no s_nop padding after them) against the inline-asm MADs
# (variant madk0): isolated permutation rate (generic / compression form), then the quick bench
# line alternated, then the permutation parity tests on the default build
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c
mkdir -p $O
for r in 1 2; do
  for b in c1 c0; do
    for v in 0 3; do echo "perm_bench_$b variant $v" >> $O/perm_bench.txt; timeout -k 10 60 tools/microbench/perm_bench_$b 1048576 32 $v >> $O/perm_bench.txt; done
  done
done
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --quick --steps 100 --warmup 5 > $O/quick_c1_$r.json 2>> $O/bench.err
  P2V_LIB=plonky2-verifier_amd/variants/libp2v_madk0.so timeout -k 10 200 python bench.py --quick --steps 100 --warmup 5 > $O/quick_c0_$r.json 2>> $O/bench.err
done
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "permutation or sbox or golden or real_circuits_vs_oracle or mds" > $O/tests.log 2>&1
echo done
