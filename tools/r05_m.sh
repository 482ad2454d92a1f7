#!/usr/bin/env bash
# Round 5: multi-sample frames with one lane per sample (trace_samples) vs the per-pixel sample
# loop (TRT_SPP_LANES=0): the spp > 1 parity tests, then kbench C5 (3840x2160, 16 spp) and a
# 1920x1080 C5-scene frame at 4 spp, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05m}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_fullres.py tests/test_golden_renders.py tests/test_gpu_parity.py -k "spp or C5 or golden or xcd" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for round in 1 2; do
  for v in 1 0; do
    TRT_SPP_LANES=$v timeout -k 10 200 python tools/kbench.py --config C5 --frames 4 --tag "lanes$v:C5" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append((r['wall_us_no_events'], r['med_us']))
for k in sorted(d): print(k, 'wall us/frame', [x[0] for x in d[k]], 'span us', [x[1] for x in d[k]])
PY
