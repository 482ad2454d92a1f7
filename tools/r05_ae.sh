#!/usr/bin/env bash
# Round 5: deferred-shadow frames at 16 / 24 / 32 frames in flight (the shipped frame and the
# README scene, kbench loops of 160 frames), interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05ae}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for inf in 16 24 32; do
    for cf in ref readme; do
      timeout -k 10 200 python tools/kbench.py --config $cf --frames 192 --inflight $inf --tag "if$inf:$cf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
