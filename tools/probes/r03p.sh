# transcript lookahead against hardware queues per process (GPU_MAX_HW_QUEUES 4 = HIP's default, 8), alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "lookahead or chained" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in "4 0" "4 1" "8 0" "8 1" "4 0" "4 1" "8 0" "8 1"; do
  set -- $v
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 --lookahead $2 > $O/b_q$1_la$2.json 2> $O/b_q$1_la$2.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_q$1_la$2.json'));print('hwq $1 lookahead $2', d['value'],d['serial']['value'],d['verified_all'])"
done
