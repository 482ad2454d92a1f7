#!/usr/bin/env bash
# Round 5: shadow walks of a wave split by origin (TRT_SHADOW_SUBSET = 8 / 16 / 32: the lanes
# near the first lane walk together when there are at least that many, the others alone) vs the
# all-or-nothing gate (product): parity of sub16 (mesh tests through TRT_LIB), then kbench C4 /
# C3 / C5 / deep frames, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05ac}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
TRT_LIB="$ROOT/variants/libtrt_sub16.so" timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_fullres.py tests/test_gpu_defer.py tests/test_golden_renders.py -k "not dropin" > "$OUT/pytest_sub16.log" 2>&1 || { tail -30 "$OUT/pytest_sub16.log"; exit 1; }
tail -1 "$OUT/pytest_sub16.log"
for round in 1 2; do
  for lib in prod sub8 sub16 sub32; do
    L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
    for cf in "C4 20" "C3 200" "C5 3" "ref 160 --inflight 16" "ref 160 --inflight 2" "readme 160 --inflight 16"; do
      set -- $cf
      c=$1; n=$2; shift 2
      TRT_LIB=$L timeout -k 10 200 python tools/kbench.py --config $c --frames $n "$@" --tag "$lib:$c:$*" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append(r['wall_us_no_events'])
for k in sorted(d): print(k, 'wall us/frame', d[k])
PY
