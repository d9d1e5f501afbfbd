# the N-rank launcher on the final code: two ranks on the one GPU over gloo (the driver's 8-GPU command
# with --dist-backend gloo), full line incl. C5
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 3 --no-cpu-baseline > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err || { tail -20 $O/bench_gpus2_gloo.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_gpus2_gloo.json'));print(d['n_gpus'], d['value'], d['serial']['value'], d['c5'], d['verified_all'])"
