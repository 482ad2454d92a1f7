#!/usr/bin/env bash
# Round 4: the prepared frame-list call in the timed region: its GPU test, then the 20-step and
# 1000-step C2 lines (3 + 1 runs).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04r}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "prepared or frame_loop" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
B="--no-cpu --tiled-frames 0 --extra-frames 0 --traffic off"
for sw in 20 20 20 1000 20 1000; do
  timeout -k 10 300 python bench.py --steps $sw $B > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
  python - "$OUT/b.log" <<'PY' | tee -a "$OUT/bench.jsonl"
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(json.dumps({"steps": d["steps"], "value": d["value"], "us": d["roofline"]["us_per_frame"], "kernel_us": d["roofline"].get("kernel_us_per_frame"), "ok": d["config"]["last_frame_matches_trt_render"]}))
PY
done
