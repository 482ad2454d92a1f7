#!/usr/bin/env bash
# Round 5: (1) mesh kernels with a rolled light loop and no frame-pair copies (one shadow walk
# inlined instead of three, 29k -> 6k instructions) vs the old code size (variant oldsize), kbench
# on C3 / C4 / C5 / shipped / README; (2) the unrotated, permuted-class frame-interleaved dealing
# (TRT_XCD_INTER=2) vs the rotating one on the C2 headline with live PMC traffic.  Tests first.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05g}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullres.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for round in 1 2; do
  for lib in prod oldsize sh4 lds32; do
    L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
    for cf in "C4 20" "C3 200" "C5 4" "ref 160" "readme 160"; do
      set -- $cf
      TRT_LIB=$L timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --tag "$lib:$1" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
for round in 1 2; do
  for bv in "bvh_old 1 16 0" "bvh_axes3 3 32 0" "bvh_sbvh 3 32 1"; do
    set -- $bv
    for cf in "C4 20" "C3 200" "ref 160" "readme 160"; do
      set -- $bv $cf
      TRT_BVH_AXES=$2 TRT_BVH_BINS=$3 TRT_BVH_SPLITS=$4 timeout -k 10 200 python tools/kbench.py --config $5 --frames $6 --tag "$1:$5" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
for round in 1 2 3; do
  for v in "inter1 1" "inter2 2"; do
    set -- $v
    TRT_XCD_INTER=$2 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --legs '' --extra-frames 0 \
        --tiled-frames 0 --no-cpu > "$OUT/b_$1_$round.json" 2>> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python - "$OUT/b_$1_$round.json" "$1" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rl = r['roofline']; td = rl.get('traffic_detail') or {}
print(sys.argv[2], 'value', r['value'], 'kernel_us', rl.get('kernel_us_per_frame'), 'fetch_raw', td.get('fetch_bytes_raw'), 'write', td.get('write_bytes'))
PY
  done
done
