#!/bin/bash
# With the faster row permutation (lposeidon.h): which form wins at which batch size.  Serial
# latency (one batch at a time) and two-in-flight throughput per batch size: the Merkle paths in
# the row form (latency mode, P2V_LAT_MAX) beyond 64 proofs, and the row vs quad transcript
# around the 2048-proof switch (P2V_TRANSCRIPT)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
run() {  # name, env, args
  env $2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['serial'].get('ms_per_step'), d['kernel_ms'])" | tee -a $O/bench.txt
}
for n in 128 256; do
  run lat${n}_def "P2V_LAT_MAX=64" "--batch $n --steps 100 --warmup 10" || exit 1
  run lat${n}_row "P2V_LAT_MAX=$n" "--batch $n --steps 100 --warmup 10" || exit 1
done
for n in 512 1024 2048 4096; do
  run tr${n}_row "P2V_QUAD_MIN=100000" "--batch $n --steps 60 --warmup 5" || exit 1
  run tr${n}_quad "P2V_QUAD_MIN=1" "--batch $n --steps 60 --warmup 5" || exit 1
done
echo done
