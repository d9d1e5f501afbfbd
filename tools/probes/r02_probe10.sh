#!/bin/bash
# new GPU tests (random number mutations vs the oracle), then the driver's multi-GPU launch shape
# (torchrun, 2 ranks, full line incl. the C5 leg) rehearsed on the one GPU with gloo
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe10
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "random_number or tiled or intermediates" > $O/gpu_tests.log 2>&1
timeout -k 10 600 python3 bench.py --gpus 2 --steps 20 --dist-backend gloo > $O/bench_gpus2.json 2> $O/bench_gpus2.err
echo done
