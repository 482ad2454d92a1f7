#!/usr/bin/env bash
# Round 5: hot-first dealing, quick A/B (C2 one launch per frame at 1 / 2 in flight) plus the hot
# lists' state after a short loop (how many tiles each frame listed).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05x}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for v in "hot0 0 512" "hot8 1 8" "hot32 1 32" "hot128 1 128"; do
    set -- $v
    for cf in "--frame-batch 1 --inflight 1" "--frame-batch 1 --inflight 2"; do
      TRT_HOT_MAX=$3 TRT_HOT_FIRST=$2 timeout -k 10 120 python tools/kbench.py --config C2 --frames 300 $cf --tag "$1:C2:$cf" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
TRT_HOT_FIRST=1 TRT_HOT_MAX=32 timeout -k 10 120 python - <<'PY'
import ctypes, sys
sys.path.insert(0, '.')
import vkcomputeshader_tinyraytracer_amd as trt
from vkcomputeshader_tinyraytracer_amd import scene as S
from vkcomputeshader_tinyraytracer_amd._lib import lib
r = trt.Renderer(0)
sc = S.CONFIGS['C2']()
p = sc.params()
r.upload_scene(sc)
f = lib().trt_diag_hot
f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
for i in range(6):
    r.draw_frame(p)
    out = (ctypes.c_uint32 * 8)()
    f(r._h, 0, out)
    print('frame', i, 'lists (count, longest ticks):', [(out[2*k], out[2*k+1]) for k in range(3)], 'next', out[6], 'hot_max', out[7])
r.close()
PY
