# round-end rehearsal on the final tree: smoke, the default bench line, one-proof latency
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'],d['serial']['value'],d['c5']['value'],d['verified_all'],d['roofline']['traffic_source'],d['valu']['issue']['step_frac'])"
timeout -k 10 200 python3 bench.py --quick --batch 1 --inflight 1 --steps 200 --warmup 10 > $O/lat_b1.json 2> $O/lat_b1.err || exit 1
python3 -c "import json;d=json.load(open('$O/lat_b1.json'));print('batch 1: serial ms/step', d['serial']['ms_per_step'])"
