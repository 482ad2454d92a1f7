#!/usr/bin/env bash
# Round 4: frames in flight for the deferred-shadow frames (shipped, README scene): the product
# (at most 8, auto 8) vs a build allowing 16 (TRT_MAX_FRAMES_IN_FLIGHT=16u) at 8 / 12 / 16,
# kbench after a settle, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04z}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for vi in "prod 8" "if16 8" "if16 12" "if16 16"; do
    set -- $vi
    for cf in ref readme; do
      TRT_LIB=variants/libtrt_$1.so timeout -k 10 200 python tools/kbench.py --config $cf --frames 192 --inflight $2 --tag "$1_if$2:$cf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
