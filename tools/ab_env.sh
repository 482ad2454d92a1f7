#!/usr/bin/env bash
# A/B: envmap pair rows (one 16-B footprint load) vs the row-major texels (two 8-B row loads),
# alternating, 2 frames in flight.  JSON lines into gpurun_out/ab_env.log.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/ab_env.log
: > "$OUT"
for rep in 1 2 3; do
  for cfg in ${CONFIGS:-C2 C3 ref}; do
    for m in 0 1; do
      TRT_ENV_PAIRROWS=$m timeout -k 10 120 python tools/kbench.py --config "$cfg" --frames ${FRAMES:-200} --tag "pairrows$m" >> "$OUT"
    done
  done
done
cat "$OUT"
