#!/bin/bash
# GPU suite (incl. the P2V_EXT_* parity tests), two bench lines, one FETCH_SIZE pass
# (leaf hashing loads two sponge blocks per trip)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe5
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --quick --steps 30 > $O/bench_$i.json 2> $O/bench_$i.err
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_fetch.err
echo done
