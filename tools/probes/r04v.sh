# round 4: the row-form S-box with the branch multiply (p2::sbox_lat_br), quad unchanged: full GPU suite,
# quick bench, batch-1 latency, smoke, and the driver's command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python3 bench.py --quick --no-c3 --steps 100 --warmup 5 > $O/b_quick.json 2> $O/b_quick.err || { tail -3 $O/b_quick.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_quick.json'));print('quick', d['value'], d['serial']['value'], d['kernel_ms'])"
timeout -k 10 300 python3 bench.py --quick --no-c3 --batch 1 --inflight 1 --steps 200 --warmup 10 > $O/b_lat.json 2> $O/b_lat.err || { tail -3 $O/b_lat.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_lat.json'));print('lat', d['serial'].get('ms_per_step'), d['kernel_ms'])"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_1.json 2> $O/driver_1.err || { tail -5 $O/driver_1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_1.json'));print('driver', d['value'], d['serial']['value'], d.get('c5',{}).get('value'), d.get('c3',{}).get('value'))"
