#!/bin/bash
# merged partial rounds: isolated permutation rate per schedule, then GPU suite + quick bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe17
mkdir -p $O
for v in 0 2 3 4; do
  timeout -k 10 60 tools/microbench/bin/perm_bench_m$v 1048576 32 0 >> $O/perm.txt 2>&1
  timeout -k 10 60 tools/microbench/bin/perm_bench_m$v 1048576 32 3 >> $O/perm.txt 2>&1
done
timeout -k 10 120 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "poseidon or perm or selftest or mds" > $O/gpu_perm_tests.log 2>&1
timeout -k 10 300 python3 bench.py --quick --steps 50 > $O/bench_quick.json 2> $O/bench.err
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
echo done
