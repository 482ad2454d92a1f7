#!/usr/bin/env bash
# Round 5: per-kernel time split of the deep frames (shipped frame, README scene) at 16 and 2
# frames in flight: pass A / pass B (defer_shadows) / pass C (defer_resolve) / fallback.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05ab}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=32
for v in "ref 16" "ref 2" "readme 16"; do
  set -- $v
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$1_$2" -o run -- python3 "$ROOT/tools/kbench.py" --config $1 --frames 64 --inflight $2 --settle-ms 0 > "$OUT/kt_$1_$2.log" 2>&1 || { tail -5 "$OUT/kt_$1_$2.log"; exit 1; }
  echo "== $1 in flight $2"
  cut -d, -f1-4 "$OUT/kt_$1_$2/run_kernel_stats.csv" | head -8
done
