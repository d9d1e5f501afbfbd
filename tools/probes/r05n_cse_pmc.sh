#!/bin/bash
# VALU instruction counts of the shared-node Merkle kernels against the plain k_merkle
# (P2V_MERKLE_CSE=0), one PMC pass each (serial launches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05n
mkdir -p $O
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for m in 1 0; do
  P2V_MERKLE_CSE=$m timeout -k 10 120 rocprofv3 --pmc $C -T --output-format csv -d $O/pmc_$m -o run -- python3 bench.py --steps 3 --warmup 1 --quick --no-c3 --inflight 1 > /dev/null 2> $O/pmc_$m.err || { tail -5 $O/pmc_$m.err; exit 1; }
done
python3 - <<'PY'
import csv, statistics, glob
for m in (1, 0):
    f = glob.glob(f"gpurun_out/r05n/pmc_{m}/**/run_counter_collection.csv", recursive=True)[0]
    v = {}
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_merkle"):
            v.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for k in sorted(v):
        print(m, k[0], k[1], statistics.median(v[k]))
PY
echo done
