#!/bin/bash
# The latency row form (lposeidon.h) in the product: the whole GPU suite on the default build, then
# batch-1 / batch-64 latency against the DPP row form (variant rowdpp: -DP2V_ROW_LAT=0), alternated,
# and the quick 4096-proof line of both (the quad path must not move)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f
mkdir -p $O
L0=plonky2-verifier_amd/libp2v.so
L1=plonky2-verifier_amd/variants/libp2v_rowdpp.so
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['serial'].get('ms_per_step'), d['kernel_ms'])" | tee -a $O/bench.txt
}
LAT1="--batch 1 --inflight 1 --steps 200 --warmup 10"
LAT64="--batch 64 --inflight 1 --steps 200 --warmup 10"
run lat1_lp_1 $L0 "$LAT1" && run lat1_dpp_1 $L1 "$LAT1" && run lat1_lp_2 $L0 "$LAT1" && run lat1_dpp_2 $L1 "$LAT1" || exit 1
run lat64_lp $L0 "$LAT64" && run lat64_dpp $L1 "$LAT64" || exit 1
run q_lp $L0 "--steps 100 --warmup 5" && run q_dpp $L1 "--steps 100 --warmup 5" || exit 1
echo done
