#!/bin/bash
# round 6: FETCH_SIZE calibration for sparse line reads (tools/microbench/sparse_fetch.hip: S lanes
# per 128-B line, every line of 2 GiB read once), the time of each, and the request-size counters
# (TCC_EA0_RDREQ, TCC_EA0_RDREQ_32B) of the bench's kernels: is k_merkle_cse's 6.4x (FETCH x 2)
# the bytes it moves?
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o
mkdir -p $O
B=tools/microbench/bin/sparse_fetch
for S in 16 8 4 2 1; do
  timeout -k 10 60 $B $S > $O/time_S$S.json || exit 1
  cat $O/time_S$S.json
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/fetch_S$S -o run -- $B $S > /dev/null 2> $O/fetch_S$S.err || { tail -5 $O/fetch_S$S.err; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -T --output-format csv -d $O/req_S$S -o run -- $B $S > /dev/null 2> $O/req_S$S.err || { tail -5 $O/req_S$S.err; exit 1; }
done
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -T --output-format csv -d $O/req_bench -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/req_bench.err || { tail -5 $O/req_bench.err; exit 1; }
echo done
