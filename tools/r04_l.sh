#!/usr/bin/env bash
# Round 4: the 20-step C2 loop after an untimed settle phase of S ms (GPU clocks at their
# sustained state?) against the 1000-step loop; kernel us per frame from the HIP-event pass.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04l}"
mkdir -p "$OUT"
cd "$ROOT"
B="--no-cpu --tiled-frames 0 --extra-frames 0 --traffic off"
row() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(json.dumps({"tag": sys.argv[2], "steps": d["steps"], "value": d["value"], "us": d["roofline"]["us_per_frame"], "kernel_us": d["roofline"].get("kernel_us_per_frame"), "launches": d["config"]["launches"], "ok": d["config"]["last_frame_matches_trt_render"]}), flush=True)
PY
}
for round in 1 2; do
  for sw in "20 0" "20 10" "20 30" "20 100" "20 300" "1000 0" "1000 100"; do
    set -- $sw
    timeout -k 10 300 python bench.py --steps $1 --settle-ms $2 $B > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
    row "$OUT/b.log" "s$1_settle$2" | tee -a "$OUT/bench.jsonl"
  done
done
timeout -k 10 60 rocm-smi --showclocks > "$OUT/clocks_idle.txt" 2>&1 || true
