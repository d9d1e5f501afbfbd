# round 4: after removing the opt-in shared Merkle levels and reordering the bench (warm-up right before the headline pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "merkle or real_circuits or golden or c5" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_$i.json 2> $O/driver_cmd_$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print('driver cmd', d['value'], d['ms_per_step'], json.dumps(d['clock']), 'serial', d['serial']['value'], json.dumps(d['serial']['clock']['step_ms']), json.dumps(d['cpu_baseline']), d['roofline'])"
done
