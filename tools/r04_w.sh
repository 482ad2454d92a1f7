#!/usr/bin/env bash
# Round 4: A/B of two builds on C2 (20- and 64-frame launches) and the mesh frames, kbench after
# a settle, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04w}"
mkdir -p "$OUT"
cd "$ROOT"
VS=${VARIANTS:-prod cur}
for round in $(seq 1 ${ROUNDS:-3}); do
  for v in $VS; do
    for cf in "C2 80 20 c2b20" "C2 192 64 c2b64" "C4 20 0 C4" "C3 60 0 C3" "ref 100 0 ref" "readme 100 0 readme"; do
      set -- $cf
      TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --frame-batch $3 --tag "$v:$4" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); v, c = r['tag'].split(':'); d[(c, v)].append((r['wall_us_no_events'], r['med_us']))
for k in sorted(d): print(k, 'wall', statistics.median(x[0] for x in d[k]), 'kernel', statistics.median(x[1] for x in d[k]), [x[0] for x in d[k]])
PY
