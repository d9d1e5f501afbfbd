#!/bin/bash
# round 6: loads one permutation ahead -- the chain kernel's next-level siblings (P2V_CSE_PREFETCH) and
# the leaf sponges' next block (P2V_LEAF_PREFETCH, one block per trip) -- against neither
# (variants/libp2v_nopf.so) and the chain prefetch alone (libp2v_csepf.so): the whole GPU suite on
# the default, then quick lines alternated and serial kernel times
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/plonky2-verifier_amd/variants
for i in 1 2; do
  for v in default nopf csepf; do
    if [ $v = default ]; then L="X=0"; else L="P2V_LIB=$V/libp2v_$v.so"; fi
    env $L timeout -k 10 200 python3 bench.py --quick --steps 200 --warmup 5 > $O/quick_${v}_$i.json 2> $O/quick_${v}_$i.err || { tail -5 $O/quick_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/quick_${v}_$i.json'));k=d['kernel_ms'];print('$v', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], k.get('k_phase1'), k.get('k_merkle'), d['verified_steps'])"
  done
done
echo done
