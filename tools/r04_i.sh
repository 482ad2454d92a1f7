#!/usr/bin/env bash
# Round 4: the default (1000-step) bench run of the product build, beside the driver's 20 steps.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04i}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python bench.py > "$OUT/bench1000.log" 2>&1 || { tail -30 "$OUT/bench1000.log"; exit 1; }
tail -c 300 "$OUT/bench1000.log"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu --traffic off > "$OUT/bench20b.log" 2>&1 || { tail -30 "$OUT/bench20b.log"; exit 1; }
