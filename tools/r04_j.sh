#!/usr/bin/env bash
# Round 4: waves per workgroup (TRT_WPB 1 / 2 / 4) for the C2 multi-frame launches: the bench's
# 20-step leg (value + last-frame check) and kbench at 20- and 64-frame launches.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04j}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2 3; do
  for v in ${VARIANTS:-base wpb2 wpb4}; do
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --tiled-frames 0 --extra-frames 0 --traffic off > "$OUT/bench_$v.log" 2>&1 || { tail -5 "$OUT/bench_$v.log"; exit 1; }
    python - "$OUT/bench_$v.log" "$v" >> "$OUT/bench.jsonl" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(json.dumps({"tag": sys.argv[2], "value": d["value"], "us": d["roofline"]["us_per_frame"], "kernel_us": d["roofline"].get("kernel_us_per_frame"), "ok": d["config"]["last_frame_matches_trt_render"]}))
PY
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C2 --frames 192 --frame-batch 64 --tag $v >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || exit 1
  done
done
cat "$OUT/bench.jsonl"
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append(r['med_us'])
for k, v in d.items(): print('kbench64', k, v, statistics.median(v))
PY
