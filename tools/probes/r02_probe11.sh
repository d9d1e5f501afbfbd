#!/bin/bash
# binary-proof ingest on the GPU (k_bytes_pack): its tests, then the full default bench line
# (now with the bytes_end_to_end leg); stdout of a 2-rank gloo run must be one JSON line
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe11
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "bytes or json_ingest or intermediates" > $O/gpu_tests.log 2>&1
timeout -k 10 500 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python3 bench.py --gpus 2 --quick --steps 10 --dist-backend gloo > $O/bench_gpus2.json 2> $O/bench_gpus2.err
echo done
