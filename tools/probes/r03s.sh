# k_merkle split (default kernel without the bottom-stage logic: 79 VGPRs, no scratch) and k_fri at the compiler's
# 122 VGPRs (variants/libp2v_fri0.so) against 96 VGPRs with 156 B of spills; GPU tests touched
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "merkle_shared or c5_shard or real_circuits_vs_oracle" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in def fri0 def fri0 def fri0; do
  if [ $v = def ]; then L=""; else L="$GRAFT_REPO_ROOT/plonky2-verifier_amd/variants/libp2v_fri0.so"; fi
  P2V_LIB=$L timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v', d['value'],d['serial']['value'],d['kernel_ms'],d['verified_all'])"
done
