#!/bin/bash
# full GPU suite, the default bench line (with the C5 leg), the --gpus launcher rehearsal (2
# gloo ranks on the one GPU), then the round's profile set
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe3
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python3 bench.py --gpus 2 --quick --steps 10 --dist-backend gloo > $O/bench_gpus2.json 2> $O/bench_gpus2.err
bash tools/profile_round.sh r02c
echo done
