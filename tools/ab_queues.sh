#!/usr/bin/env bash
# Frames in flight x HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4) on C2.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for rep in 1 2; do
  for q in 4 8; do
    for fl in 2 3 4; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/kbench.py --config ${CFG:-C2} --frames 400 --inflight $fl --tag "q$q"
    done
  done
done
