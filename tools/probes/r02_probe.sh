#!/bin/bash
# Round-2 measurement probe (GPU box): VALU issue costs, side-stream priority A/B, isolated
# kernel durations, VALU class counters; then the fault-isolation run of the branch-form
# general multiply, last.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_probe
mkdir -p $O
timeout -k 10 120 ./tools/microbench/valu_rates 400 40 > $O/valu_rates.txt 2>&1
timeout -k 10 200 python3 bench.py --quick --steps 20 > $O/bench_prio1.json 2> $O/bench_prio1.err
P2V_SIDE_PRIO=0 timeout -k 10 200 python3 bench.py --quick --steps 20 > $O/bench_prio0.json 2> $O/bench_prio0.err
P2V_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_single -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 > $O/bench_single.json 2> $O/trace_single.err
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv -d $O/pmc_rates -o run -- ./tools/microbench/valu_rates 100 10 > /dev/null 2> $O/pmc_rates.err
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv -d $O/pmc_bench -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_bench.err
echo probe-done
# fault isolation: branch-form general multiply, every launch named and synchronised
P2V_LIB=plonky2-verifier_amd/variants/libp2v_mul2.so P2V_DEBUG_SYNC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/mul2_tests.log 2>&1
echo mul2-done
