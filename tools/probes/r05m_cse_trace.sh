#!/bin/bash
# kernel trace of the shared-node Merkle path (serial pass): per-kernel durations of
# k_merkle_plan / k_merkle_cse / k_merkle_resolve
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick --no-c3 --inflight 1 > $O/bench.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
cat $O/trace/run_kernel_stats.csv | cut -d, -f1-8 | head -30
echo done
