# round 4: k_fri arity-16 fold in two halves (no scratch): FRI-touching GPU tests, A/B bench against the
# 16-value fold (variants/libp2v_fold0.so: also the item-major vanishing order) and against the item-major
# vanishing order alone (variants/libp2v_vx0.so); FETCH/WRITE PMC passes of all three
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "oracle or golden or c5 or c3 or full_size" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, lib
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 --steps 100 --warmup 5 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['kernel_ms'])" | tee -a $O/bench.txt
}
L0=plonky2-verifier_amd/variants/libp2v_fold0.so
L1=plonky2-verifier_amd/libp2v.so
L2=plonky2-verifier_amd/variants/libp2v_vx0.so
run new_1 $L1 && run fold0_1 $L0 && run vx0_1 $L2 && run new_2 $L1 && run fold0_2 $L0 && run vx0_2 $L2 || exit 1
for v in new:$L1 fold0:$L0 vx0:$L2; do n=${v%%:*}; l=${v#*:}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    P2V_LIB=$l timeout -s KILL 120 rocprofv3 --pmc $ctr -T --output-format csv -d $O/pmc_${n}_$ctr -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --no-c3 > /dev/null 2> $O/pmc_${n}_$ctr.err || exit 1
  done
done
echo done
