#!/usr/bin/env bash
# C2 stage pricing (diagnostic variants: notrig = no atan2/acos, noenvfetch = no texel gathers,
# nopow = no pow in Phong, noshadow = no shadow rays) against the work tree's build, interleaved
# rounds of tools/kbench.py at the bench's 20-frame launches; then the drop-in hashes recorded.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04c}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2 3; do
  for v in ${VARIANTS:-base notrig noenvfetch nopow noshadow}; do
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config ${CFG:-C2} --frames 200 --frame-batch 20 --tag $v >> "$OUT/ab_c2.jsonl" 2>> "$OUT/ab_c2.err" || { tail -5 "$OUT/ab_c2.err"; exit 1; }
  done
done
python - "$OUT/ab_c2.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append(r['med_us'])
for k, v in d.items(): print(k, [round(x, 2) for x in v], 'median', round(statistics.median(v), 2))
PY
TRT_DROPIN_RECORD="$OUT/dropin_hashes.json" timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 280 --timeout-method thread > "$OUT/dropin.log" 2>&1 || { tail -20 "$OUT/dropin.log"; exit 1; }
tail -2 "$OUT/dropin.log"
