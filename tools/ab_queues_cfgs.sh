#!/usr/bin/env bash
# GPU_MAX_HW_QUEUES=8 with 2 / 3 / 4 frames in flight vs the default (4 queues, 2 in flight).
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for cfg in ${CONFIGS:-C3 C4 ref readme}; do
  timeout -k 10 120 python tools/kbench.py --config $cfg --frames 40 --inflight 2 --tag q4
  for fl in 2 3 4; do
    GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/kbench.py --config $cfg --frames 40 --inflight $fl --tag q8
  done
done
