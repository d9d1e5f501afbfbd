#!/bin/bash
# round 6: which PMC counters the box offers for instruction fetch / issue stalls (rocprofv3 -L)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -5 $O/counters.txt; exit 1; }
grep -iE "ICACHE|IFETCH|SQC_|WAIT_INST|INST_LEVEL|SQ_WAVE_CYCLES|ACTIVE_INST_ANY|SQ_WAIT_ANY" $O/counters.txt | sort -u | head -60
echo done
