#!/bin/bash
# Collect the round's profiles on the GPU box (then run tools/pmc_summary.py <tag> locally):
#  1) kernel trace + stats of the default bench command (serial pass + two-in-flight pass)
#  2) kernel trace + stats with --inflight 1: per-launch averages = bench's kernel_ms
#  3) two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic per kernel
#  4) one PMC pass of SQ instruction counters (VALU instructions and dual-issued quads per kernel: the binding resource)
#  5) the same serial trace and PMC passes for the C3 circuit (bench.py --lookups 2: live lookup argument)
# usage: tools/profile_round.sh <tag>
set -e
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 2 --quick > $OUT/bench_under_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_serial -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 > $OUT/bench_under_trace_serial.json 2> $OUT/trace_serial.err
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $OUT/pmc_write.err
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/pmc_valu -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $OUT/pmc_valu.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c3_trace_serial -o run -- python3 bench.py --steps 10 --warmup 2 --quick --inflight 1 --lookups 2 > $OUT/c3_bench_under_trace_serial.json 2> $OUT/c3_trace_serial.err
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/c3_pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --lookups 2 > /dev/null 2> $OUT/c3_pmc_fetch.err
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/c3_pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --lookups 2 > /dev/null 2> $OUT/c3_pmc_write.err
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/c3_pmc_valu -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --lookups 2 > /dev/null 2> $OUT/c3_pmc_valu.err
echo done
