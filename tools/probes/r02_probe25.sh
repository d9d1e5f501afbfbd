#!/bin/bash
# merged partial rounds in the quad transcript: chain latency, parity, bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe25
mkdir -p $O
for v in q0 q4; do
  timeout -k 10 60 tools/microbench/bin/perm_bench_$v 4096 200 9 >> $O/perm.txt 2>&1
  timeout -k 10 60 tools/microbench/bin/perm_bench_$v 4096 200 8 >> $O/perm.txt 2>&1
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "transcript_forms or golden or real_circuits or n12" > $O/gpu_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --quick --steps 60 > $O/bench_$i.json 2>> $O/bench.err
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('qmerge', d['value'], d['serial']['value'], d['kernel_ms'])" >> $O/summary.txt
done
echo done
