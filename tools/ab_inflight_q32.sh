# A/B of frames in flight for plain C2 frames at 32 hardware queues (bench headline leg only).
set -e
mkdir -p gpurun_out
: > gpurun_out/ab_inflight_q32.log
for rep in 1 2; do
  for n in 4 6 8; do
    timeout -k 10 200 python bench.py --no-cpu --tiled-frames 0 --extra-frames 0 --inflight $n > gpurun_out/b_if$n.log 2>&1
    echo "inflight=$n $(grep '^{' gpurun_out/b_if$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['tiled_headline_1gpu']['ms_per_step'])")" >> gpurun_out/ab_inflight_q32.log
  done
done
cat gpurun_out/ab_inflight_q32.log
