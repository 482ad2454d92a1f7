#!/usr/bin/env bash
# Round 5: wave priority for deep segments (TRT_PRIO: s_setprio once a lane traces a child
# segment) on the drawFrame-paced C2 loop (one launch per frame, 1 / 2 in flight), the 20-frame
# headline loop and C3 single frames, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05z}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for lib in prod prio1 prio3; do
    L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
    for cf in "C2 300 --frame-batch 1 --inflight 1" "C2 300 --frame-batch 1 --inflight 2" "C2 200 --frame-batch 20" "C3 100 --frame-batch 1 --inflight 2"; do
      set -- $cf
      c=$1; n=$2; shift 2
      TRT_LIB=$L timeout -k 10 120 python tools/kbench.py --config $c --frames $n "$@" --tag "$lib:$c:$*" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
