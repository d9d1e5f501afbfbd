# round 4, final code: the multi-rank launcher rehearsed with two ranks sharing the one GPU (gloo
# data-path group), as the driver's N = 2 run shapes it; C5 leg sharded over both ranks (lane-form launches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 900 python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { tail -20 $O/bench_gpus2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_gpus2.json'));print(d['value'], d['n_gpus'], d.get('c5',{}).get('value'), d.get('verified_all'), d.get('config'))"
