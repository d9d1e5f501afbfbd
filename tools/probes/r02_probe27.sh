#!/bin/bash
# VALU issue cost of the VOP2 (vcc) encodings of the carry-chain ops, and of a VOP3/VOP2 mix
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe27
mkdir -p $O
timeout -k 10 200 tools/microbench/bin/valu_rates2 > $O/valu_rates2.txt 2>&1
echo done
