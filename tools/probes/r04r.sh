# round 4: where the vanishing kernels' fabric reads come from: L2 hits / misses / fabric read requests and
# L1 -> L2 read requests per kernel, final code
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04r
mkdir -p $O
for v in new:plonky2-verifier_amd/libp2v.so; do n=${v%%:*}; l=${v#*:}
  P2V_LIB=$l timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -T --output-format csv -d $O/pmc_${n}_tcc -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --no-c3 > /dev/null 2> $O/pmc_${n}_tcc.err || { tail -5 $O/pmc_${n}_tcc.err; exit 1; }
done
echo done
