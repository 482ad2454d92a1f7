#!/usr/bin/env bash
# Round 5: workgroup timeline of single-frame C2 launches (diagnostic clock build): span,
# workgroup durations, when the longest workgroups start, the tail.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05t}"
mkdir -p "$OUT"
cd "$ROOT"
for cf in C2 C3; do
  TRT_LIB="$ROOT/variants/libtrt_clock.so" timeout -k 10 120 python tools/waveclock.py --config $cf --frames 20 --out "$OUT/clock_$cf.npz" > "$OUT/clock_$cf.log" 2>&1 || { tail -5 "$OUT/clock_$cf.log"; exit 1; }
  tail -1 "$OUT/clock_$cf.log"
done
