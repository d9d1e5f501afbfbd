# round 4: kernel trace of a 20-step line (driver's shape) to see the pipeline fill at the start of the pipelined pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --quick > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], json.dumps(d['clock']['step_ms']))"
find $O/trace -name '*kernel_trace.csv' | head -3
