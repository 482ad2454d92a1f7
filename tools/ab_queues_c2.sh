#!/usr/bin/env bash
# C2, same box, interleaved: (HW queues, frames in flight) pairs, 3 rounds.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for rep in 1 2 3; do
  for qf in 4:2 8:3 8:4 16:4 16:6 16:8; do
    q=${qf%%:*}; fl=${qf##*:}
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/kbench.py --config ${CFG:-C2} --frames 1000 --inflight $fl --tag "q$q"
  done
done
