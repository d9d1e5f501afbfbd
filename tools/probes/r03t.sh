# final evidence of the round-3 code (k_merkle split): GPU suite, smoke, profile collection (kernel stats + VALU / FETCH / WRITE
# PMC passes), the full default line, latency; k_fri-first variant alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh r03t || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'],d['serial']['value'],d['c5']['value'],d['verified_all'])"
timeout -k 10 200 python3 bench.py --quick --batch 1 --inflight 1 --steps 200 --warmup 10 > $O/lat_b1.json 2> $O/lat_b1.err || exit 1
python3 -c "import json;d=json.load(open('$O/lat_b1.json'));print('batch 1: serial ms/step', d['serial']['ms_per_step'])"
