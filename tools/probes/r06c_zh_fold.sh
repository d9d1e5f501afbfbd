#!/bin/bash
# round 6: the peeled zh round 0 with its constant MDS columns folded (P2V_ZH_FOLD)
# and the round-6 fixes: the full GPU suite, then quick lines alternated against -DP2V_ZH_FOLD=0
# (variants/libp2v_nofold.so) and one VALU PMC pass of each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in fold nofold; do
    if [ $v = fold ]; then L=""; else L="P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_nofold.so"; fi
    env $L timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 > $O/quick_${v}_$i.json 2> $O/quick_${v}_$i.err || { tail -5 $O/quick_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/quick_${v}_$i.json'));print('$v', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'].get('k_merkle'), d['kernel_ms'].get('k_phase1'), d['verified_steps'])"
  done
done
for v in fold nofold; do
  if [ $v = fold ]; then L=""; else L="P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_nofold.so"; fi
  env $L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 -T --output-format csv -d $O/pmc_valu_$v -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_valu_$v.err || { tail -5 $O/pmc_valu_$v.err; exit 1; }
done
python3 - <<PY
import csv, statistics
for v in ("fold", "nofold"):
    vals = {}
    for row in csv.DictReader(open("$O/pmc_valu_%s/run_counter_collection.csv" % v)):
        if row["Kernel_Name"].startswith("k_"):
            vals.setdefault((row["Kernel_Name"], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
    med = {k: statistics.median(x) for k, x in vals.items()}
    ks = sorted({k for k, _ in med})
    cyc = {k: 4 * (med.get((k, "SQ_INSTS_VALU"), 0) - med.get((k, "SQ_ACTIVE_INST_VALU2"), 0)) for k in ks}
    print(v, "issue cycles G per launch:", {k: round(c / 1e9, 4) for k, c in cyc.items() if c > 1e7}, "step", round(sum(cyc.values()) / 1e9, 4))
PY
echo done
