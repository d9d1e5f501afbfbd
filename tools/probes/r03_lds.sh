#!/bin/bash
# transcript permutation tables in LDS: quad / row chain latency, GPU parity subset, bench --quick x2
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_lds
mkdir -p $O
timeout -k 10 60 tools/microbench/bin/perm_bench 4096 200 9 > $O/perm.txt 2>&1
timeout -k 10 60 tools/microbench/bin/perm_bench 4096 200 8 >> $O/perm.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "oracle or real or quad or row" > $O/gpu_tests.log 2>&1
echo tests-done
for i in 1 2; do
  timeout -k 10 150 python3 bench.py --quick --steps 100 --warmup 5 > $O/fused$i.json 2> $O/fused$i.err
done
echo bench-done
