# round 4: the transcript chains' S-box with the 11-VALU multiply and one uniform fix-up branch per stage
# (P2V_SBOX_LAT_BRANCH=1, libp2v.so) against the 14-VALU branch-free multiply (variants/libp2v_lat0.so):
# transcript / oracle GPU tests, A/B bench (pipelined, serial), batch-1 latency, C5 unaffected (lane form)
# (after this probe: the branch form kept for the row form only, p2::sbox_lat_br; the quad keeps sbox_lat)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "transcript or oracle or golden or latency or poseidon or field_mul" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['serial'].get('ms_per_step'), d['kernel_ms'])" | tee -a $O/bench.txt
}
L0=plonky2-verifier_amd/variants/libp2v_lat0.so
L1=plonky2-verifier_amd/libp2v.so
S="--steps 100 --warmup 5"
LAT="--batch 1 --inflight 1 --steps 200 --warmup 10"
run new_1 $L1 "$S" && run lat0_1 $L0 "$S" && run new_2 $L1 "$S" && run lat0_2 $L0 "$S" || exit 1
run lat_new_1 $L1 "$LAT" && run lat_lat0_1 $L0 "$LAT" && run lat_new_2 $L1 "$LAT" && run lat_lat0_2 $L0 "$LAT" || exit 1
echo done
