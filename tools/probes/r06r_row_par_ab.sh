#!/bin/bash
# round 6: P2V_ROW_PAR=1 (the library) against =0 (variants/libp2v_rp0.so), alternated: the default
# line without C5 / CPU legs (main step pipelined + serial, C3 leg, drop-in latency, host legs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06r
mkdir -p $O
for r in 1 2; do
  for v in par rp0; do
    if [ $v = rp0 ]; then export P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_rp0.so; else unset P2V_LIB; fi
    timeout -k 10 300 python3 bench.py --no-c5 --no-cpu-baseline --steps 200 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -20 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v', $r, d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['c3']['value'], d['dropin']['n1']['warm'], d['dropin']['n64']['warm'])" | tee -a $O/ab.txt
  done
done
echo done
