#!/usr/bin/env bash
# Round 4: A/B of the work tree (base) against HEAD's kernel (prev) on C2 (20-frame launches),
# C4 and the deep frames, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04g}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2 3; do
  for v in ${VARIANTS:-prev base}; do
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --frame-batch 20 --tag $v >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C4 --frames 10 --frame-batch 10 --tag $v >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config ref --frames 40 --inflight 8 --tag $v >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
  done
done
python - "$OUT/ab.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[(r['config'], r['tag'])].append((r['med_us'], r['wall_us_no_events']))
for k in sorted(d): print(k, 'kernel med', round(statistics.median(x[0] for x in d[k]), 2), 'wall med', round(statistics.median(x[1] for x in d[k]), 2))
PY
