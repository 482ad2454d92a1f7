#!/usr/bin/env bash
# Round 5: C4 with deferred shadows (pass A without shadow rays, then the shadow and resolve
# passes) vs the per-pixel kernel on today's build (verdict item 2, option 1), and C3 the same.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05p}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for dm in 1 2; do
    for cf in "C4 20" "C3 200"; do
      set -- $cf
      timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --defer $dm --tag "defer$dm:$1" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_defer" -o run -- python "$ROOT/tools/kbench.py" --config C4 --frames 8 --settle-ms 0 --defer 2 --inflight 1 > "$OUT/kt_defer.log" 2>&1 || { tail -5 "$OUT/kt_defer.log"; exit 1; }
echo done
