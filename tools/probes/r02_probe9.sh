#!/bin/bash
# the default bench line (tiled layout, C5 leg, CPU baseline, ingest / PCIe legs) and smoke()
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe9
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
echo done
