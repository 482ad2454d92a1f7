#!/usr/bin/env bash
# A/B of deferred shadows (trt_set_deferred_shadows) vs the per-pixel loop on the mesh configs,
# 1 and 2 frames in flight.  One JSON line per run (tools/kbench.py) into gpurun_out/ab_defer.log.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/ab_defer.log
: > "$OUT"
for cfg in ${CONFIGS:-ref readme C3 C4}; do
  for fl in 1 2; do
    for d in 1 2; do
      timeout -k 10 120 python tools/kbench.py --config "$cfg" --frames ${FRAMES:-40} --inflight $fl --defer $d --tag "defer$d" >> "$OUT"
    done
  done
done
cat "$OUT"
