#!/bin/bash
# round 6: the quad transcript's chain S-boxes split over lane pairs (qposeidon.h sbox_qu,
# P2V_QUAD_SBOX2=1, the library) against =0 (variants/libp2v_qs0.so): quad chain latency (KAT,
# mismatches), the transcript / permutation-form GPU tests, then quick lines alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06w
mkdir -p $O
for v in 0 1 0 1; do
  echo "QUAD_SBOX2=$v" >> $O/quad_chain.txt
  timeout -k 10 60 tools/microbench/bin/perm_bench_qs$v 4096 200 9 >> $O/quad_chain.txt || { cat $O/quad_chain.txt; exit 1; }
done
cat $O/quad_chain.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "transcript or forms or selftest or reference_intermediates or real_circuits" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in qs1 qs0; do
    if [ $v = qs0 ]; then export P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_qs0.so; else unset P2V_LIB; fi
    timeout -k 10 200 python3 bench.py --quick --steps 300 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -20 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v', $r, d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['serial']['clock']['run_clock']['clock_ghz'], d['verified_steps'], d.get('kernel_ms',{}).get('k_phase1'))" | tee -a $O/ab.txt
  done
done
echo done
