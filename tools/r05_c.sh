#!/usr/bin/env bash
# Round 5: deferred frames at the reference's 2 frames in flight — the pool design with a subtree
# split window (trt_set_subtree_split 2..5: window-edge subtrees go to task queues traced by
# other waves) against no split, shipped and README frames.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05c}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for sp in 1 2 3 4 5; do
    for cf in ref readme; do
      for inf in 2 16; do
        timeout -k 10 150 python tools/kbench.py --config $cf --frames 160 --inflight $inf --split $sp --tag "split$sp:$cf:$inf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
      done
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
