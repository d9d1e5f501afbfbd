#!/bin/bash
# degree_bits sweep (the same verifier on deeper trees / more FRI steps; degenerate circuit, whose
# verifier work has the same shape) and C3 (lookup tables)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe13
mkdir -p $O
for nb in 8 10 14 16; do
  timeout -k 10 400 python3 bench.py --quick --steps 20 --circuit degenerate --degree-bits $nb --distinct 16 --witnesses 4 > $O/sweep_n$nb.json 2>> $O/sweep.err
done
timeout -k 10 400 python3 bench.py --quick --steps 20 --lookups 2 > $O/c3.json 2> $O/c3.err
echo done
