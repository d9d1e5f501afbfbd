# round 4, final tree: smoke, then the driver's command twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -5 $O/driver_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/driver_$i.json'));print('driver', d['value'], d['serial']['value'], d.get('c5',{}).get('value'), d.get('c3',{}).get('value'), d['clock']['device_over_host'])"
done
