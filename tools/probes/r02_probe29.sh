#!/bin/bash
# the driver's N>1 launcher path on the final code: bench.py --gpus 2 spawns torchrun itself
# (2 ranks on the one GPU of this box, gloo for the host-side collectives)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe29
mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 30 > $O/bench_gpus2_gloo.json 2> $O/bench.err
echo done
