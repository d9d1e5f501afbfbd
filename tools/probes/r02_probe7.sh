#!/bin/bash
# k_merkle: two levels of siblings per load trip, the odd half parked in LDS (variant mlds) vs default
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe7
mkdir -p $O
V=plonky2-verifier_amd/variants/libp2v_mlds.so
P2V_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "golden or real or shape_sweep or ext or n12" > $O/mlds_tests.log 2>&1
for v in default mlds default mlds; do
  if [ $v = default ]; then L=plonky2-verifier_amd/libp2v.so; else L=$V; fi
  P2V_LIB=$L timeout -k 10 200 python3 bench.py --quick --steps 30 > $O/bench_${v}_$RANDOM.json 2>> $O/bench.err
done
P2V_LIB=$V timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch_mlds -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_fetch_mlds.err
echo done
