set -e
mkdir -p gpurun_out
P2V_TRANSCRIPT=quad timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick6q.log 2>&1; tail -1 gpurun_out/quick6q.log
P2V_TRANSCRIPT=row timeout -k 10 300 python3 tools/gpu_quick.py > gpurun_out/quick6r.log 2>&1; tail -1 gpurun_out/quick6r.log
for B in 512 1024 2048 4096 8192; do
  for M in quad row; do
    P2V_TRANSCRIPT=$M timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch $B > gpurun_out/tb_${M}_${B}.json 2> /dev/null
    python3 -c "import json;d=json.load(open('gpurun_out/tb_${M}_${B}.json'));print('$M',$B,d['value'],d['ms_per_step'],d['kernel_ms']['k_phase1'],d['kernel_ms']['k_merkle'])"
  done
done
