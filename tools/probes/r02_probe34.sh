#!/bin/bash
# the default bench command as the driver runs it (300 timed steps by default now)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe34
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench_default.json 2> $O/bench.err
echo done
