#!/bin/bash
# round 6: the fix-list dedup + lane-form fix and k_merkle_cse's merged tile order
# per XCD: Merkle / mutation / garbage / pool GPU tests, smoke, FETCH_SIZE of the
# Merkle kernels for the new order against the round-5 order (variants/libp2v_cse0.so,
# -DP2V_CSE_ORDER=0), quick pipelined + serial lines alternated, the driver's bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "merkle or mutation or ragged or garbage or pool" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for v in new cse0; do
  if [ $v = new ]; then L=""; else L="P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_cse0.so"; fi
  env $L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch_$v -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_fetch_$v.err || { tail -5 $O/pmc_fetch_$v.err; exit 1; }
done
python3 - <<PY
import csv, statistics
for v in ("new", "cse0"):
    vals = {}
    for row in csv.DictReader(open("$O/pmc_fetch_%s/run_counter_collection.csv" % v)):
        if row["Counter_Name"] == "FETCH_SIZE" and row["Kernel_Name"].startswith("k_merkle"):
            vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    print(v, {k: round(statistics.median(x) * 2 * 1024 / 1e6, 1) for k, x in vals.items()}, "MB (2 x FETCH_SIZE KiB)")
PY
for i in 1 2; do
  for v in new cse0; do
    if [ $v = new ]; then L=""; else L="P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_cse0.so"; fi
    env $L timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 > $O/quick_${v}_$i.json 2> $O/quick_${v}_$i.err || { tail -5 $O/quick_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/quick_${v}_$i.json'));print('$v', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'].get('k_merkle'), d['verified_steps'])"
  done
done
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));print('driver', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['build']['version'], d['build']['match'])"
echo done
