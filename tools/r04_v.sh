#!/usr/bin/env bash
# Round 4: the prepared multi-frame call: its GPU tests, the --force-dist bench test, and the
# 20-step line's tiled_1gpu leg.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04v}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_bench_dist.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "prepared or bench or frame_loop" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for k in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --no-cpu --extra-frames 0 --traffic off > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
python - "$OUT/b.log" <<'PY' | tee -a "$OUT/bench.jsonl"
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(json.dumps({"steps": d["steps"], "value": d["value"], "tiled_1gpu": d.get("tiled_1gpu", {}).get("value"), "tiled_c4_ms": d.get("tiled_frame", {}).get("ms_per_frame"), "us": d["roofline"]["us_per_frame"], "kernel_us": d["roofline"].get("kernel_us_per_frame"), "ok": d["config"]["last_frame_matches_trt_render"]}))
PY
done
