#!/bin/bash
# Phase-1 forms A/B (GPU box): fused k_phase1 vs P2V_PHASE1=excl (k_transcript_x alone on its
# SIMDs + k_leaf beside it), alternated, bench.py --quick (serial + two in flight).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_excl
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --quick --steps 100 --warmup 5 > $O/fused$i.json 2> $O/fused$i.err
  P2V_PHASE1=excl timeout -k 10 150 python3 bench.py --quick --steps 100 --warmup 5 > $O/excl$i.json 2> $O/excl$i.err
  echo "round $i done"
done
