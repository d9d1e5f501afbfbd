# batches in flight and staggering on the round-3 code (alternated), plus the small-batch latency after the n <= 128 cut
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k
mkdir -p $O
for b in 1 128 256; do
  timeout -k 10 200 python3 bench.py --quick --batch $b --inflight 1 --steps 200 --warmup 10 > $O/lat_b$b.json 2> $O/lat_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/lat_b$b.json'));print('batch $b: serial ms/step', d['serial']['ms_per_step'], 'kernel_ms', d['kernel_ms'])"
done
for v in "2 0" "3 0" "2 1" "3 1" "2 0" "3 0" "4 0"; do
  set -- $v
  timeout -k 10 300 python3 bench.py --quick --steps 100 --warmup 5 --inflight $1 --stagger $2 > $O/bench_i$1_s$2.json 2> $O/bench_i$1_s$2.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_i$1_s$2.json'));print('inflight $1 stagger $2', d['value'],d['serial']['value'],d['verified_all'])"
done
