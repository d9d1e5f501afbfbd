#!/bin/bash
# Latency row form (lposeidon.h: LDS exchange, merged partial blocks, asm-block multiply) against
# the DPP row form (rposeidon.h, current S-box and the asm-block S-box), dependent-chain latency
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e
mkdir -p $O
for r in 1 2; do
  for b in "l 10" "r0 8" "r2 8"; do
    set -- $b
    echo "perm_bench_$1 mode $2" >> $O/row_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_$1 1 2000 $2 >> $O/row_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_$1 64 500 $2 >> $O/row_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_$1 1024 200 $2 >> $O/row_chain.txt
  done
done
echo done
