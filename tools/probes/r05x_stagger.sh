#!/bin/bash
# staggered workspaces (p2v_verifier_chain: a workspace's phase 1 after the other's) on the final
# round-5 code, against the default, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05x
mkdir -p $O
run() {  # name, args
  timeout -k 10 300 python3 bench.py --quick --no-c3 --steps 100 --warmup 5 $2 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_all'], d['kernel_ms'])" | tee -a $O/bench.txt
}
for r in 1 2 3; do run def_$r "" && run stag_$r "--stagger 1" || exit 1; done
echo done
