#!/bin/bash
# round 6: the fix list deduplicated, the lane form of k_merkle_fix for long lists,
# lazily allocated host-input buffer, source hash in p2v_version: the Merkle / mutation / ragged GPU
# tests (+ the garbage-batch test), smoke, the driver's bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "merkle or mutation or ragged or garbage or pool" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));print(d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['verified_steps'], d['build']['version'], d['build']['match'])"
echo done
