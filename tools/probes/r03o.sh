# transcript lookahead (P2V_FLAG_LOOKAHEAD): GPU test, then quick lines with and without it, alternated, and a pipelined trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "lookahead or chained" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for la in 1 0 1 0 1 0; do
  timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 --lookahead $la > $O/b_la$la.json 2> $O/b_la$la.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_la$la.json'));print('lookahead $la', d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick --lookahead 1 > $O/bench_under_trace.json 2> $O/trace.err
