#!/bin/bash
# vanishing items in tile-major order with each tile's items on one XCD (P2V_VANISH_XCD=1, libp2v.so)
# against the item-major order (variant vx0): the vanishing parity tests, FETCH/WRITE PMC passes of
# both builds (serial), then the quick line alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zb
mkdir -p $O
L1=plonky2-verifier_amd/libp2v.so
L0=plonky2-verifier_amd/variants/libp2v_vx0.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "oracle or golden or real or lookup or vanish or ragged" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  L=$L1; [ $v = 0 ] && L=$L0
  for c in FETCH_SIZE WRITE_SIZE; do
    P2V_LIB=$L timeout -k 10 300 rocprofv3 --pmc $c -T --output-format csv -d $O/pmc_${c}_$v -o run -- python3 bench.py --steps 3 --warmup 1 --quick --inflight 1 --no-c3 > /dev/null 2> $O/pmc_${c}_$v.err || { tail -5 $O/pmc_${c}_$v.err; exit 1; }
  done
done
run() {  # name, lib, args
  P2V_LIB=$2 timeout -k 10 300 python3 bench.py --quick --no-c3 $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -3 $O/b_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/b_$1.json'));print('$1', d['value'], d['serial']['value'], d['clock']['run_clock']['clock_ghz'], d['kernel_ms'])" | tee -a $O/bench.txt
}
Q="--steps 100 --warmup 5"
run x1_1 $L1 "$Q" && run x0_1 $L0 "$Q" && run x1_2 $L1 "$Q" && run x0_2 $L0 "$Q" && run x1_3 $L1 "$Q" && run x0_3 $L0 "$Q" || exit 1
echo done
