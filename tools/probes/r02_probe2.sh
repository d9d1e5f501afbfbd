#!/bin/bash
# A/B: proof-major in-place reads (no k_transpose) and the branch-form general multiply,
# against the default build; the proof-major build's GPU parity suite first.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe2
mkdir -p $O
P2V_LIB=plonky2-verifier_amd/variants/libp2v_pm.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pm_tests.log 2>&1
for v in default pm mul2 default pm; do
  if [ $v = default ]; then L=plonky2-verifier_amd/libp2v.so; else L=plonky2-verifier_amd/variants/libp2v_$v.so; fi
  P2V_LIB=$L timeout -k 10 200 python3 bench.py --quick --steps 30 > $O/bench_$v.json 2>> $O/bench.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['serial']['value'], d['kernel_ms'])" >> $O/summary.txt
done
P2V_LIB=plonky2-verifier_amd/variants/libp2v_pm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_pm_serial -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 > $O/bench_pm_trace.json 2> $O/trace_pm.err
echo done
