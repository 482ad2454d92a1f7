#!/usr/bin/env bash
# Round 5: where a drawFrame-paced C2 frame (one launch per frame) loses against multi-frame
# launches: kernel traces of one launch per frame at 1 and 2 in flight and of 20-frame launches
# (per-kernel durations and the gaps between kernels).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05s}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=32
for v in "fb1_if1 --frame-batch 1 --inflight 1" "fb1_if2 --frame-batch 1 --inflight 2" "fb20 --frame-batch 20"; do
  set -- $v
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$name" -o run -- python "$ROOT/tools/kbench.py" --config C2 --frames 200 "$@" > "$OUT/kt_$name.log" 2>&1 || { tail -5 "$OUT/kt_$name.log"; exit 1; }
  grep '^{' "$OUT/kt_$name.log" | tail -1 | cut -c1-300
done
echo done
