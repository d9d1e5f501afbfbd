#!/bin/bash
# zh-folded round 0: permutation rate, parity subset, quick bench; then the round's profiles (r02g)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe19
mkdir -p $O
timeout -k 10 60 tools/microbench/bin/perm_bench_m4 1048576 32 3 >> $O/perm.txt 2>&1
timeout -k 10 60 tools/microbench/bin/perm_bench_m4z 1048576 32 3 >> $O/perm.txt 2>&1
timeout -k 10 60 tools/microbench/bin/perm_bench_m4z 1048576 32 0 >> $O/perm.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "poseidon or mds or real_circuits or golden or n12" > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py --quick --steps 50 > $O/bench_quick.json 2> $O/bench.err
bash tools/profile_round.sh r02g > $O/prof.log 2>&1
echo done
