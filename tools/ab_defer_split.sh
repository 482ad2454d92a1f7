#!/usr/bin/env bash
# Deferred shadows with a LINK-event subtree split: windows off / 2..5 on the deep mesh frames,
# 2 frames in flight.  JSON lines into gpurun_out/ab_defer_split.log.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/ab_defer_split.log
: > "$OUT"
for cfg in ${CONFIGS:-ref readme}; do
  for w in ${WINDOWS:-1 2 3 4 5}; do
    for fl in ${INFLIGHT:-2}; do
      timeout -k 10 120 python tools/kbench.py --config "$cfg" --frames ${FRAMES:-40} --inflight $fl --defer 2 --split $w --tag "defer_w$w" >> "$OUT"
    done
  done
done
cat "$OUT"
