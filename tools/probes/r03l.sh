# side-stream work-groups (k_fri, k_vanish_final: one wave vs 256 threads) and k_fri first, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "matches_oracle_status or real_circuits_vs_oracle or c5_shard" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in "64 0" "256 0" "64 1" "64 0" "256 0" "64 1" "64 0"; do
  set -- $v
  P2V_SIDE_WG=$1 P2V_FRI_FIRST=$2 timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_$1_$2.json'));print('side_wg $1 fri_first $2', d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick > $O/bench_under_trace.json 2> $O/trace.err
