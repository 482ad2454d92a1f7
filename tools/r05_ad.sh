#!/usr/bin/env bash
# Round 5: rocprofv3 kernel-trace summary of the driver's bench command (N = 1, 20 steps; the
# CPU leg and the live PMC child runs off, since they cannot nest under the tracer).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05ad}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu --traffic off > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
grep '^{' "$OUT/prof_bench.log" | tail -1 | cut -c1-400
cut -d, -f1-4 "$OUT/prof/run_kernel_stats.csv" | head -14
