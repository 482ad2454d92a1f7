#!/usr/bin/env bash
# Deferred frames: unsplit pass A vs one depth per launch (TRT_DEFER_WAVEFRONT=1), 1 and 2 in flight.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for cfg in ${CONFIGS:-ref readme}; do
  for fl in 1 2; do
    timeout -k 10 120 python tools/kbench.py --config $cfg --frames 40 --inflight $fl --tag unsplit
    TRT_DEFER_WAVEFRONT=1 timeout -k 10 120 python tools/kbench.py --config $cfg --frames 40 --inflight $fl --tag wavefront
  done
done
