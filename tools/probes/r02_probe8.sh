#!/bin/bash
# tiled input layout (P2V_FLAG_INPUT_TILED, now the bench default): GPU suite, bench tiled vs
# proof-major, then the round's profile set (kernel stats, FETCH / WRITE / VALU PMC passes)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe8
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for l in tiled proof-major tiled proof-major; do
  timeout -k 10 200 python3 bench.py --quick --steps 30 --layout $l > $O/bench_${l}_$RANDOM.json 2>> $O/bench.err
done
bash tools/profile_round.sh r02e
echo done
