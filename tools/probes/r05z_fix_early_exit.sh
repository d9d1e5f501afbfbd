#!/bin/bash
# k_merkle_fix blocks without entries return before their LDS table fill: the Merkle / mutation /
# ragged GPU tests, a serial kernel trace, the driver's bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "merkle or mutation or ragged" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick --no-c3 --inflight 1 > $O/bench_trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
cut -d, -f1-4 $O/trace/run_kernel_stats.csv | head -12
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err || { tail -5 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));print('driver', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'])"
echo done
