# round 4: the driver's exact bench command, twice, with the device clock in the line; a 300-step quick line
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_$i.json 2> $O/driver_cmd_$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print('driver cmd', d['value'], d['ms_per_step'], json.dumps(d['clock']), 'serial', d['serial']['value'], json.dumps(d['serial']['clock']))"
done
timeout -k 10 300 python3 bench.py --quick --steps 300 --warmup 3 > $O/quick300.json 2> $O/quick300.err || exit 1
python3 -c "import json;d=json.load(open('$O/quick300.json'));print('quick300', d['value'], d['ms_per_step'], json.dumps(d['clock']), 'serial', d['serial']['value'])"
