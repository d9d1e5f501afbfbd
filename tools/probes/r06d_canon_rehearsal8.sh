#!/bin/bash
# round 6: canonical outputs only for the groups a caller reads + the folded round 0 on the leaf
# sponges' first block: permutation / Merkle / oracle GPU tests, a quick line and a VALU PMC pass;
# then the driver's 8-GPU command rehearsed on the one GPU: 8 torchrun ranks,
# gloo default group, C5 sharded 8 ways, wall time recorded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "poseidon or permutation or sbox or merkle or garbage or matches_oracle or real_circuits" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 > $O/quick.json 2> $O/quick.err || { tail -5 $O/quick.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/quick.json'));print('quick', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'].get('k_merkle'), d['kernel_ms'].get('k_phase1'), d['verified_steps'])"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 -T --output-format csv -d $O/pmc_valu -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_valu.err || { tail -5 $O/pmc_valu.err; exit 1; }
python3 - <<PY
import csv, statistics
vals = {}
for row in csv.DictReader(open("$O/pmc_valu/run_counter_collection.csv")):
    if row["Kernel_Name"].startswith("k_"):
        vals.setdefault((row["Kernel_Name"], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
med = {k: statistics.median(x) for k, x in vals.items()}
ks = sorted({k for k, _ in med})
cyc = {k: 4 * (med.get((k, "SQ_INSTS_VALU"), 0) - med.get((k, "SQ_ACTIVE_INST_VALU2"), 0)) for k in ks}
print("issue cycles G per launch:", {k: round(c / 1e9, 4) for k, c in cyc.items() if c > 1e7}, "step", round(sum(cyc.values()) / 1e9, 4))
PY
date +%s > $O/rehearsal8.start
timeout -k 10 700 python3 bench.py --gpus 8 --dist-backend gloo --steps 20 --warmup 5 > $O/bench_gpus8.json 2> $O/bench_gpus8.err || { tail -30 $O/bench_gpus8.err; exit 1; }
date +%s > $O/rehearsal8.end
python3 - <<PY
import json
d = json.load(open("$O/bench_gpus8.json"))
w = int(open("$O/rehearsal8.end").read()) - int(open("$O/rehearsal8.start").read())
print("gpus8", d["n_gpus"], d["value"], "per_rank", len(d["per_rank"]["proofs_per_s"]), d["verified_all"], d["verified_steps"],
      "c5", d["c5"]["value"], d["c5"]["verified_all"], d["c5"]["shard_per_gpu"], "wall_s", w, "threads", d["build"]["host_threads_per_rank"])
PY
echo done
