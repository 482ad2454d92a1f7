#!/usr/bin/env bash
# Round 4: where the C2 20-frame launch loses to the 64-frame one.  bench.py's plain loop at
# 20 / 64 / 256 / 1000 steps and 20 steps after a long warmup; kbench at F frames per launch;
# workgroup timelines (clock build) of a 20- and a 64-frame launch.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04k}"
mkdir -p "$OUT"
cd "$ROOT"
B="--no-cpu --tiled-frames 0 --extra-frames 0 --traffic off"
row() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(json.dumps({"tag": sys.argv[2], "steps": d["steps"], "warmup": d["warmup"], "value": d["value"], "us": d["roofline"]["us_per_frame"], "kernel_us": d["roofline"].get("kernel_us_per_frame"), "launches": d["config"]["launches"], "ok": d["config"]["last_frame_matches_trt_render"]}), flush=True)
PY
}
for round in 1 2; do
  for sw in "20 5" "20 200" "20 1000" "64 5" "256 5" "1000 5"; do
    set -- $sw
    timeout -k 10 300 python bench.py --steps $1 --warmup $2 $B > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
    row "$OUT/b.log" "s$1_w$2" | tee -a "$OUT/bench.jsonl"
  done
done
FRAMES="1 4 16 20 32 64" ROUNDS=1 timeout -k 10 400 bash tools/launch_tail_probe.sh > "$OUT/tail_probe.log" 2>&1 || exit 1
cat "$OUT/tail_probe.log"
for F in 20 64; do
  TRT_LIB=variants/libtrt_clock.so timeout -k 10 200 python tools/waveclock_multi.py --config C2 --frames $F --reps 2 > "$OUT/clock_f$F.log" 2>&1 || { tail -5 "$OUT/clock_f$F.log"; exit 1; }
  grep '^{' "$OUT/clock_f$F.log" | cut -c1-400
done
