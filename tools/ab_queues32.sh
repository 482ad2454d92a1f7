# A/B of 16 vs 32 HIP hardware queues per process on the full bench line (1 GPU).
set -e
mkdir -p gpurun_out
for q in 16 32 16 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_q$q.log 2>&1
  echo "q=$q $(grep '^{' gpurun_out/bench_q$q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['tiled_headline_1gpu']['ms_per_step'], d['tiled_frame']['ms_per_frame'], d['shipped_frame']['ms_per_frame'], d['readme_frame']['ms_per_frame'])")" | tee -a gpurun_out/ab_q32.log
done
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_q32_k20.log 2>&1
echo "q=32 K=20 $(grep '^{' gpurun_out/bench_q32_k20.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['tiled_headline_1gpu']['ms_per_step'], d['tiled_frame']['ms_per_frame'], d['shipped_frame']['ms_per_frame'], d['readme_frame']['ms_per_frame'])")" | tee -a gpurun_out/ab_q32.log
