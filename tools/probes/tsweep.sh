#!/bin/bash
# Transcript-form sweep on the GPU box: quad vs row (P2V_TRANSCRIPT) across batch sizes.
# An A/B library can be swept too by exporting P2V_LIB=<path to an alternative libp2v.so>.
set -e
mkdir -p gpurun_out/ts
for B in 1024 4096 16384; do
  for M in quad row; do
    P2V_TRANSCRIPT=$M timeout -k 10 200 python3 bench.py --quick --batch $B > gpurun_out/ts/${M}_${B}.json 2>/dev/null
    python3 -c "import json;d=json.load(open('gpurun_out/ts/${M}_${B}.json'));print('$M',$B,d['value'],d['serial']['value'],d['kernel_ms']['k_phase1'],d['kernel_ms']['k_merkle'])"
  done
done
