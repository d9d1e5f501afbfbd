#!/bin/bash
# batches in flight (1..4) at the C2 shape, and single-batch latency at 1 / 256 / 1024 proofs
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe6
mkdir -p $O
for k in 2 3 4 2 3; do
  timeout -k 10 200 python3 bench.py --quick --steps 40 --inflight $k > $O/inflight_${k}_$RANDOM.json 2>> $O/bench.err
done
for b in 1 256 1024; do
  timeout -k 10 200 python3 bench.py --quick --steps 20 --inflight 1 --batch $b --distinct 16 > $O/latency_$b.json 2>> $O/bench.err
done
echo done
