#!/usr/bin/env bash
# Round 4 closing session: the deferred frames at 16 (auto) / 24 / 32 frames in flight
# (TRT_DEFER_IN_FLIGHT), then the closing validation (tools/r04_n.sh).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r04zz"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2; do
  for n in 16 24 32; do
    for cf in ref readme; do
      GPU_MAX_HW_QUEUES=32 TRT_DEFER_IN_FLIGHT=$n timeout -k 10 200 python tools/kbench.py --config $cf --frames 192 --tag "if$n:$cf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); v, c = r['tag'].split(':'); d[(c, v)].append(r['wall_us_no_events'])
for k in sorted(d): print(k, 'wall us/frame', statistics.median(d[k]), d[k])
PY
R04_TAG=r04final bash tools/r04_n.sh
