#!/bin/bash
# round 0 of a zh permutation (compression, first sponge block) with the constant words' MDS
# columns folded into round 1's constants (P2V_ZH_FOLD=1, libp2v.so) against the round-5 form
# (variant zf0): the whole GPU suite on the new build, SQ VALU passes of both, quick line alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ze
mkdir -p $O
L1=plonky2-verifier_amd/libp2v.so
L0=plonky2-verifier_amd/variants/libp2v_zf0.so
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in 1 0; do
  L=$L1; [ $v = 0 ] && L=$L0
  P2V_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES -T --output-format csv -d $O/pmc_valu_$v -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --no-c3 > /dev/null 2> $O/pmc_valu_$v.err || { tail -5 $O/pmc_valu_$v.err; exit 1; }
done
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
run f1_1 $L1 "$Q" && run f0_1 $L0 "$Q" && run f1_2 $L1 "$Q" && run f0_2 $L0 "$Q" && run f1_3 $L1 "$Q" && run f0_3 $L0 "$Q" || exit 1
echo done
