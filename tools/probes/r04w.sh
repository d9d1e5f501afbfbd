# round 4: a row-only k_phase1_row for latency-mode batches (tools/probes/r04w_phase1_row.patch, built as
# variants/libp2v_row.so) against the tree's k_phase1 (row and quad in one kernel): latency-mode GPU tests
# through the variant, batch-1 latency A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w
mkdir -p $O
L0=plonky2-verifier_amd/libp2v.so
L1=plonky2-verifier_amd/variants/libp2v_row.so
P2V_LIB=$L1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "latency or ragged or lookahead or transcript_forms or empty or golden" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['serial'].get('ms_per_step'), d['kernel_ms'])" | tee -a $O/bench.txt
}
LAT="--batch 1 --inflight 1 --steps 200 --warmup 10"
run lat_row_1 $L1 "$LAT" && run lat_tree_1 $L0 "$LAT" && run lat_row_2 $L1 "$LAT" && run lat_tree_2 $L0 "$LAT" || exit 1
echo done
