# round 4: PoseidonGate parts as 3 items and both partial-product rounds in one item (vanishing
# re-reads): full GPU suite, A/B bench and batch-1 latency against variants/libp2v_old8.so (8 parts,
# one pp item per round), FETCH/WRITE PMC passes of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['serial'].get('ms_per_step'), d['kernel_ms'])" | tee -a $O/bench.txt
}
L0=plonky2-verifier_amd/variants/libp2v_old8.so
L1=plonky2-verifier_amd/libp2v.so
S="--steps 100 --warmup 5"
LAT="--batch 1 --inflight 1 --steps 200 --warmup 10"
run new_1 $L1 "$S" && run old8_1 $L0 "$S" && run new_2 $L1 "$S" && run old8_2 $L0 "$S" || exit 1
run lat_new_1 $L1 "$LAT" && run lat_old8_1 $L0 "$LAT" && run lat_new_2 $L1 "$LAT" && run lat_old8_2 $L0 "$LAT" || exit 1
for v in new:$L1 old8:$L0; do n=${v%%:*}; l=${v#*:}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    P2V_LIB=$l timeout -s KILL 120 rocprofv3 --pmc $ctr -T --output-format csv -d $O/pmc_${n}_$ctr -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --no-c3 > /dev/null 2> $O/pmc_${n}_$ctr.err || exit 1
  done
done
echo done
# C3 leg (65536 live-lookup proofs, launches of 16384) with the lookup items capped (default) and uncapped
L2=plonky2-verifier_amd/variants/libp2v_lk0.so
c3() {  # name, lib
  P2V_LIB=$2 timeout -k 10 400 python3 bench.py --no-c5 --no-cpu-baseline --steps 20 --warmup 5 > $O/c3_$1.json 2> $O/c3_$1.err || { tail -3 $O/c3_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$1.json'))['c3'];print('c3 $1', d['value'], d['kernel_ms_serial_4096'])" | tee -a $O/bench.txt
}
c3 cap_1 $L1 && c3 nocap_1 $L2 && c3 cap_2 $L1 && c3 nocap_2 $L2 || exit 1
echo done_c3
