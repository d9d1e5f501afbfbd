# round 4, final code: full GPU suite, smoke, the default bench line and the driver's command twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d.get('c5',{}).get('value'), d.get('c3',{}).get('value'))"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -5 $O/driver_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/driver_$i.json'));print('driver', d['value'], d['serial']['value'], d['clock']['device_over_host'])"
done
