#!/bin/bash
# round 6: the C3 leg, P2V_ROW_PAR=1 (the library) against =0 (variants/libp2v_rp0.so), alternated, the old library first (is the first reading on a fresh box low whichever library runs?)
# three times (r06r saw one low C3 reading on the new library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
for r in 1 2 3; do
  for v in rp0 par; do
    if [ $v = rp0 ]; then export P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_rp0.so; else unset P2V_LIB; fi
    timeout -k 10 200 python3 bench.py --no-c5 --no-cpu-baseline --no-host-legs --steps 20 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -20 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));c=d['c3'];print('$v', $r, d['value'], d['clock']['run_clock']['clock_ghz'], c['value'], c['seconds'], c['verified_all'], c['kernel_ms_serial_4096'])" | tee -a $O/ab.txt
  done
done
echo done
