#!/bin/bash
# round 6: the large-launch legs (C5: 131072-proof launches, C3: 16384, both with the lane-form
# transcript) on the final tree against the round-5 library (variants/libp2v_r5.so, built from the
# round-5 commit's sources), the leaf sponges without the fold (libp2v_leafnofold.so) and no fold at
# all (libp2v_nofold.so); alternated, device-resident legs only
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06j
mkdir -p $O
V=$PWD/plonky2-verifier_amd/variants
for i in 1 2; do
  for v in default r5 leafnofold nofold; do
    if [ $v = default ]; then L="X=0"; else L="P2V_LIB=$V/libp2v_$v.so"; fi
    env $L timeout -k 10 240 python3 bench.py --steps 100 --warmup 5 --no-host-legs > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], 'c5', d['c5']['value'], d['c5']['verified_all'], 'c3', d['c3']['value'], d['c3']['verified_all'])"
  done
done
echo done
