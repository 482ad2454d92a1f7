#!/usr/bin/env bash
# Round 5: the level design of deferred frames — GPU tests of both designs, then kbench A/B of
# levels vs pool on the shipped and README frames at 16 and 2 frames in flight (interleaved
# rounds), then a kernel trace of one level-mode frame loop.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05b}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_defer.py > "$OUT/pytest_defer.log" 2>&1 || { tail -40 "$OUT/pytest_defer.log"; exit 1; }
tail -3 "$OUT/pytest_defer.log"
for round in 1; do
  for mode in pool levels_b levels; do
    for cf in ref readme; do
      for inf in 16 2; do
        TRT_DEFER_MODE=$mode timeout -k 10 150 python tools/kbench.py --config $cf --frames 160 --inflight $inf --tag "$mode:$cf:$inf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
      done
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append((r['wall_us_no_events'], r['med_us'], r['host_enqueue_us']))
for k in sorted(d): print(k, 'wall us/frame', [x[0] for x in d[k]], 'launch-span med us', [x[1] for x in d[k]], 'host us', [x[2] for x in d[k]])
PY
cd /tmp && export TMPDIR=/tmp
TRT_DEFER_MODE=levels_b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python "$ROOT/tools/kbench.py" --config ref --frames 16 --inflight 1 --settle-ms 0 --tag prof > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
echo done
