#!/usr/bin/env bash
# Round 4: GEOM 3 kernels with the quantized walk only (cur) vs the build before (base):
# C4 / C3 / shipped frame / README scene / C2, kbench after a 50 ms settle, 3 interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04m}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2 3; do
  for v in ${VARIANTS:-base cur}; do
    for cf in "C4 20" "C3 60" "ref 100" "readme 100" "C2 192"; do
      set -- $cf
      TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --tag "$v" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[(r['config'], r['tag'])].append(r['wall_us_no_events'])
for k in sorted(d): print(k, d[k], 'median', statistics.median(d[k]))
PY
