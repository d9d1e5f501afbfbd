#!/bin/bash
# split phase 1 (k_transcript on the side stream beside k_leaf) vs the fused k_phase1; the
# FETCH_SIZE calibration of the proof-major read pattern (tools/microbench/stream_pm.hip)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --quick --steps 30 > $O/bench_split_$i.json 2> $O/bench_split_$i.err
  P2V_PHASE1=fused timeout -k 10 200 python3 bench.py --quick --steps 30 > $O/bench_fused_$i.json 2> $O/bench_fused_$i.err
done
B=tools/microbench/stream_pm
for m in 0 1 2; do
  for s in 0 300; do
    timeout -k 10 60 $B $m $s > $O/stream_${m}_${s}.json
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_stream_${m}_${s} -o run -- $B $m $s > /dev/null 2> $O/pmc_stream_${m}_${s}.err
  done
done
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -T --output-format csv -d $O/pmc_rq_0 -o run -- $B 0 300 > /dev/null 2> $O/pmc_rq_0.err
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -T --output-format csv -d $O/pmc_rq_2 -o run -- $B 2 300 > /dev/null 2> $O/pmc_rq_2.err
echo done
