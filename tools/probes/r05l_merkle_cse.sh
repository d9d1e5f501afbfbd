#!/bin/bash
# Shared-node Merkle paths (k_merkle_plan / k_merkle_cse / k_merkle_resolve, default) against the
# plain one-path-per-lane k_merkle (P2V_MERKLE_CSE=0): the full GPU suite on the default build,
# then the quick line alternated (the serial pass's k_merkle slot covers all three kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cse, args
  P2V_MERKLE_CSE=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_all'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
run c1_1 1 "$Q" && run c0_1 0 "$Q" && run c1_2 1 "$Q" && run c0_2 0 "$Q" && run c1_3 1 "$Q" && run c0_3 0 "$Q" || exit 1
echo done
