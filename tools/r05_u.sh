#!/usr/bin/env bash
# Round 5: hot-first dealing of single-frame launches (TRT_HOT_FIRST=1, product) vs plain
# dealing: the hot-first tests and the parity subset, then kbench C2 at one launch per frame
# (1 and 2 in flight: drawFrame pacing), C3 single frames, C2 20-frame launches (unaffected),
# interleaved rounds; the single-frame C2 timeline with hot-first on.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05u}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
[ "${SKIP_TESTS:-0}" = 1 ] || { timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_hot.py tests/test_gpu_parity.py tests/test_gpu_fullres.py tests/test_golden_renders.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -2 "$OUT/pytest.log"
for round in 1 2; do
  for h in 1 0; do
    for cf in "C2 300 --frame-batch 1 --inflight 1" "C2 300 --frame-batch 1 --inflight 2" "C3 100 --frame-batch 1 --inflight 1" "C3 100 --frame-batch 1 --inflight 2" "C2 200 --frame-batch 20"; do
      set -- $cf
      c=$1; n=$2; shift 2
      TRT_HOT_FIRST=$h timeout -k 10 200 python tools/kbench.py --config $c --frames $n "$@" --tag "hot$h:$c:$*" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
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
TRT_LIB="$ROOT/variants/libtrt_clock.so" TRT_HOT_FIRST=1 timeout -k 10 120 python tools/waveclock.py --config C2 --frames 20 > "$OUT/clock_C2_hot.log" 2>&1 || { tail -5 "$OUT/clock_C2_hot.log"; exit 1; }
tail -1 "$OUT/clock_C2_hot.log"
