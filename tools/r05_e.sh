#!/usr/bin/env bash
# Round 5 validation: the whole GPU suite, the driver's bench command (N = 1, 20 steps: the line
# with its C3 / C5 / per-frame-launch legs and live PMC traffic) and smoke().
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05e}"
mkdir -p "$OUT"
cd "$ROOT"
export TRT_PARITY_LOG="$OUT/parity_log.jsonl"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=15 > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -20 "$OUT/pytest_gpu.log"
unset TRT_PARITY_LOG
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20.log" 2>&1 || { tail -20 "$OUT/bench20.log"; exit 1; }
tail -c 3000 "$OUT/bench20.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
