#!/bin/bash
# quad transcript with the chunk's loads issued before the permutation: GPU parity subset, then
# bench.py --quick fused vs P2V_PHASE1=excl, alternated
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_prefetch
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "oracle or real or quad or row" > $O/gpu_tests.log 2>&1
echo tests-done
for i in 1 2; do
  timeout -k 10 150 python3 bench.py --quick --steps 100 --warmup 5 > $O/fused$i.json 2> $O/fused$i.err
  P2V_PHASE1=excl timeout -k 10 150 python3 bench.py --quick --steps 100 --warmup 5 > $O/excl$i.json 2> $O/excl$i.err
  echo "round $i done"
done
