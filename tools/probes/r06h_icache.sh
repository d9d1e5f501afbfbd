#!/bin/bash
# round 6: instruction-cache misses and issue stalls per kernel (serial bench pass): are the ~250 KB
# k_phase1 and ~82 KB k_merkle_cse code bodies fetched from L2 while they run?
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06h
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -T --output-format csv -d $O/icache -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/icache.err || { tail -5 $O/icache.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_BUSY_CYCLES -T --output-format csv -d $O/stall -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/stall.err || { tail -5 $O/stall.err; exit 1; }
python3 - <<PY
import csv, statistics
for d in ("icache", "stall"):
    vals = {}
    for row in csv.DictReader(open("$O/%s/run_counter_collection.csv" % d)):
        if row["Kernel_Name"].startswith("k_"):
            vals.setdefault((row["Kernel_Name"], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
    med = {k: statistics.median(x) for k, x in vals.items()}
    for k in sorted({k for k, _ in med}):
        print(d, k, {c: "%.4g" % v for (kk, c), v in med.items() if kk == k})
PY
echo done
