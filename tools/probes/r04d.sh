# round 4: partial products chained through the MAD addends (P2V_MUL_PRODUCT=1) against the carry-add form (0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d
mkdir -p $O
M=tools/microbench
for v in 0 1; do
  for V in 0 3; do timeout -k 10 60 $M/perm_bench_m$v 1048576 32 $V | tee -a $O/perm.txt || exit 1; done
  timeout -k 10 60 $M/perm_bench_m$v 4096 200 9 | tee -a $O/perm.txt || exit 1
  timeout -k 10 60 $M/perm_bench_m$v 1024 200 8 | tee -a $O/perm.txt || exit 1
done
for i in 1 2; do
  for lib in mulold default; do
    if [ $lib = default ]; then unset P2V_LIB; else export P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_$lib.so; fi
    timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/b_${lib}_$i.json 2> $O/b_${lib}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b_${lib}_$i.json'));print('$lib', d['value'], d['serial']['value'], d['kernel_ms'])" | tee -a $O/bench.txt
  done
done
unset P2V_LIB
