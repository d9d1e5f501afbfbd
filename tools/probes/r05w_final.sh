#!/bin/bash
# round-5 evidence on the final tree (k_merkle_cse at 5 waves per SIMD): Merkle / mutation / ragged GPU
# tests, a serial kernel trace, smoke, the driver's bench command twice, the
# default bench line (C5, C3, drop-in, from-host legs, CPU baseline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "merkle or mutation or ragged or full_size or c5 or golden or n12" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick --no-c3 --inflight 1 > $O/bench_trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
cut -d, -f1-4 $O/trace/run_kernel_stats.csv | head -12
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_$i.json 2> $O/driver_cmd_$i.err || { tail -5 $O/driver_cmd_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print('driver', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['valu']['issue']['at_run_clock'])"
done
timeout -k 10 900 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d.get('dropin'), (d.get('c5') or {}).get('value'), (d.get('c3') or {}).get('value'))"
echo done
