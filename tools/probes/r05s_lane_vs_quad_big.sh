#!/bin/bash
# Transcript form at large launches on the shared-node Merkle code: the lane form (default from
# 16384 proofs) against the quad (P2V_LANE_MIN past the batch), 16384 and 131072 proofs per step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s
mkdir -p $O
run() {  # name, lane_min, batch, steps
  P2V_LANE_MIN=$2 timeout -k 10 400 python3 bench.py --quick --no-c3 --batch $3 --steps $4 --warmup 2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_all'], d['kernel_ms'])" | tee -a $O/bench.txt
}
for r in 1 2; do
  run lane16k_$r 16384 16384 40 && run quad16k_$r 100000000 16384 40 || exit 1
  run lane128k_$r 16384 131072 6 && run quad128k_$r 100000000 131072 6 || exit 1
done
echo done
