#!/usr/bin/env bash
# Round-3 closing run, part 2: rocprofv3 kernel statistics of the C2 frame loop alone (20-frame
# launches as in the 20-step bench; one frame per launch at one in flight), of the 20-step bench
# command, and the PMC passes of tools/pmc_r03.sh.
source "$(dirname "$0")/gpu_lib.sh"
export TMPDIR=/tmp
R="$ROOT/gpurun_out"
cd /tmp && step rp_c2_b20 300 rocprofv3 --kernel-trace --stats -d "$R/rp_c2_b20" -o run -- python3 "$ROOT/tools/kbench.py" --config C2 --frames 640 --frame-batch 20 \
 && step rp_c2_1in 300 rocprofv3 --kernel-trace --stats -d "$R/rp_c2_1in" -o run -- python3 "$ROOT/tools/kbench.py" --config C2 --frames 600 --inflight 1 --frame-batch 1 \
 && step rp_c4 300 rocprofv3 --kernel-trace --stats -d "$R/rp_c4" -o run -- python3 "$ROOT/tools/kbench.py" --config C4 --frames 20 \
 && step rp_bench20 420 rocprofv3 --kernel-trace --stats -d "$R/rp_bench20" -o run -- python3 "$ROOT/bench.py" --steps 20 --no-cpu \
 && CFGS="${PMC_CFGS:-C2 C4 ref readme}" step pmc 700 "$ROOT/tools/pmc_r03.sh"
