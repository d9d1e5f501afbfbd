#!/bin/bash
# the isolated permutation rate of the current code (generic and compression form), for the
# verifier-vs-isolated comparison of the VALU roofline
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe14
mkdir -p $O
B=tools/microbench/perm_bench
for v in 0 3 0 3; do timeout -k 10 60 $B 1048576 32 $v >> $O/perm_bench.txt; done
echo done
