#!/bin/bash
# lane-form transcript: parity of the three transcript forms, then quick bench per form
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe18
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "transcript_forms" > $O/gpu_forms_tests.log 2>&1
for f in quad lane quad lane; do
  P2V_TRANSCRIPT=$f timeout -k 10 300 python3 bench.py --quick --steps 50 > $O/bench_$f.json 2>> $O/bench.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_$f.json')); print('$f', d['value'], d['serial']['value'], d['kernel_ms'])" >> $O/summary.txt
done
echo done
