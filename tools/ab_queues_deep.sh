#!/usr/bin/env bash
# Frames in flight 4 / 6 / 8 with 8 or 16 HIP hardware queues per process.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for cfg in ${CONFIGS:-C2 C3 ref readme}; do
  for q in 8 16; do
    for fl in 4 6 8; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/kbench.py --config $cfg --frames ${FRAMES:-80} --inflight $fl --tag "q$q"
    done
  done
done
