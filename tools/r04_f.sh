#!/usr/bin/env bash
# Round 4: waves per SIMD of pass A (TRT_DEFER_WAVES 4 = prod, 5, 6) on the deep frames.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04f}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2; do
  for v in ${VARIANTS:-prod dw5 dw6}; do
    lib=""; [ "$v" != prod ] && lib="variants/libtrt_$v.so"
    for cfg in ref readme; do
      for inf in 2 8; do
        TRT_LIB=$lib timeout -k 10 200 python tools/kbench.py --config $cfg --frames 40 --inflight $inf --tag "$v" >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
      done
    done
  done
done
python - "$OUT/ab.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[(r['tag'], r['config'], r['inflight'])].append(r['wall_us_no_events'])
for k in sorted(d): print(k, [round(x, 1) for x in d[k]], 'median', round(statistics.median(d[k]), 1))
PY
