#!/usr/bin/env bash
# Round 5: sanity timing of the product library against an older build (variants/late0) on one
# box: C2 20-frame launches and one launch per frame.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05w}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
rocm-smi --showclocks > "$OUT/smi.log" 2>&1 || true
for lib in old prod; do
  L=""; [ $lib = old ] && L="$ROOT/variants/libtrt_late0.so"
  for cf in "--frame-batch 20" "--frame-batch 1 --inflight 1"; do
    TRT_LIB=$L TRT_HOT_FIRST=0 timeout -k 10 120 python tools/kbench.py --config C2 --frames 200 $cf --tag "$lib:$cf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); print(r['tag'], r['wall_us_no_events'], r['med_us'])
PY
