# round 4: C3 (live lookup circuit): tests, the default line with its c3 leg, lookup kernels capped vs not, kernel traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "lookup or c3" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['serial']['value'], d['c5']['value'], json.dumps(d['c3']), d['cpu_baseline'])"
for i in 1 2; do
  for lib in lknocap default; do
    if [ $lib = default ]; then unset P2V_LIB; else export P2V_LIB=$PWD/plonky2-verifier_amd/variants/libp2v_$lib.so; fi
    timeout -k 10 300 python3 bench.py --quick --lookups 2 --steps 50 --warmup 5 > $O/c3_${lib}_$i.json 2> $O/c3_${lib}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('$O/c3_${lib}_$i.json'));print('c3 $lib', d['value'], d['serial']['value'], d['kernel_ms'])"
  done
done
unset P2V_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_serial -o run -- python3 bench.py --quick --lookups 2 --steps 10 --warmup 2 --inflight 1 > $O/c3_trace_serial.json 2> $O/c3_trace_serial.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --quick --lookups 2 --steps 10 --warmup 2 > $O/c3_trace.json 2> $O/c3_trace.err || exit 1
echo traced
