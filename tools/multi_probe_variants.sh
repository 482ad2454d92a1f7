# A/B of tools/multi_probe.py conditions (bench.py's tiled leg at one rank vs the bare probe):
# which combination of a prior Renderer, a torch stream and a counting pass slows the
# pipelined multi-frame path, and whether more hardware queues remove it.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 120 python tools/multi_probe.py --frames 1024 --per-gather 64 "$@" 2>/dev/null | grep '^{' >> gpurun_out/mp.log; }
: > gpurun_out/mp.log
run
run --prior-renderer --torch-stream --count-pass
run --prior-renderer --torch-stream
run --prior-renderer --count-pass
run --torch-stream --count-pass
GPU_MAX_HW_QUEUES=32 run --prior-renderer --torch-stream --count-pass
GPU_MAX_HW_QUEUES=32 run
