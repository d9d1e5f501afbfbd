#!/bin/bash
# throughput of circuits under the opt-in plonky2 conventions (P2V_EXT_*), against the default
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe15
mkdir -p $O
timeout -k 10 300 python3 bench.py --quick --steps 30 > $O/default.json 2> $O/err.log
timeout -k 10 300 python3 bench.py --quick --steps 30 --ext 2 > $O/ext2_hiding.json 2>> $O/err.log
timeout -k 10 300 python3 bench.py --quick --steps 30 --ext 7 --arities 3,3,2 > $O/ext7_minsize332.json 2>> $O/err.log
timeout -k 10 300 python3 bench.py --quick --steps 30 --ext 5 --arities 2,2,2,2 > $O/ext5_arity4x4.json 2>> $O/err.log
echo done
