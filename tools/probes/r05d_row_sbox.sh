#!/bin/bash
# Row-form (16-lane) permutation chain latency per S-box form (P2V_ROW_SBOX 0..3: branch-per-stage
# asm multiply, plain C multiply, asm-block multiply, branch-free asm multiply), alternated; then
# the two-rank launcher rehearsal on the one GPU (bench.py --gpus 2 --dist-backend gloo) for the
# per-rank figures
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d
mkdir -p $O
for r in 1 2; do
  for v in 0 1 2 3; do
    echo "P2V_ROW_SBOX=$v" >> $O/row_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_r$v 1 2000 8 >> $O/row_chain.txt
    timeout -k 10 60 tools/microbench/perm_bench_r$v 64 500 8 >> $O/row_chain.txt
  done
done
timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-c3 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
echo done
