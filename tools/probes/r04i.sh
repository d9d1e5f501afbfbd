# round 4: effective clock, wave stall and instruction-cache counters per kernel (serial 4096-proof runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*\|GRBM_GUI_ACTIVE\|SQ_WAVE_CYCLES\|SQ_WAIT_ANY\|SQ_BUSY_CU_CYCLES\|SQ_INSTS_SMEM\|SQ_ACTIVE_INST_ANY\|SQ_ACTIVE_INST_MISC\|SQ_ACTIVE_INST_SCA\|SQ_INST_CYCLES_VMEM\|SQ_WAIT_INST_LDS" $O/avail.txt | sort -u > $O/avail_sel.txt
cat $O/avail_sel.txt | tr '\n' ' '; echo
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -T --output-format csv -d $O/pmc_a -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_a.err || { tail -5 $O/pmc_a.err; exit 1; }
echo pass a
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -T --output-format csv -d $O/pmc_b -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 > /dev/null 2> $O/pmc_b.err || { tail -5 $O/pmc_b.err; exit 1; }
echo pass b
# S-box groups: perm_bench per P2V_SBOX_ILP, then the bench alternated over ilp0 / default (2) / ilp4
M=tools/microbench
for v in 0 1 2 4; do timeout -k 10 60 $M/perm_bench_s$v 1048576 32 0 | tail -1 | sed "s/^/ilp$v /" | tee -a $O/perm.txt || exit 1; timeout -k 10 60 $M/perm_bench_s$v 1048576 32 3 | tail -1 | sed "s/^/ilp$v /" | tee -a $O/perm.txt || exit 1; done
for i in 1 2; do
  for lib in ilp0 default ilp4; do
    if [ $lib = default ]; then unset P2V_LIB; else export P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_$lib.so; fi
    timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/b_${lib}_$i.json 2> $O/b_${lib}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b_${lib}_$i.json'));print('$lib', d['value'], d['serial']['value'], d['kernel_ms'])" | tee -a $O/bench.txt
  done
done
