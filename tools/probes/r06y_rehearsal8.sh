#!/bin/bash
# round 6, final library: the driver's 8-GPU command in the driver's own torchrun form, with all 8
# ranks on the one GPU (each rank verifies its statuses; C5 sharded over the 8 ranks), wall time
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
t0=$(date +%s)
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 > $O/bench_gpus8.json 2> $O/bench_gpus8.err || { tail -30 $O/bench_gpus8.err; exit 1; }
t1=$(date +%s)
echo "wall_s $((t1 - t0))" | tee $O/wall.txt
python3 -c "import json;d=json.load(open('$O/bench_gpus8.json'));print('gpus8', d['value'], d['n_gpus'], d.get('verified_all'), d['verified_steps'], len(d.get('per_rank',[])), d['c5']['value'], d['c5']['verified_all'], d['build']['match'])"
echo done
