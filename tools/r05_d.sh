#!/usr/bin/env bash
# Round 5: C2 envmap traffic vs the tile -> XCD dealing of multi-frame launches.  Primary-ray
# misses sample the same texels in every frame (the camera only translates), so a dealing that
# keeps a tile on one XCD across the frames of a launch can serve them from that XCD's L2.
# bench.py's headline loop (20 steps, 20-frame launch, camera walk) + its live PMC traffic, per
# dealing variant, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05d}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2; do
  for v in "inter 1 1" "rot0 1 0" "frame_major_rot 0 1" "frame_major_fixed 0 0"; do
    set -- $v
    TRT_XCD_INTER=$2 TRT_XCD_ROT=$3 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --legs '' --extra-frames 0 \
        --tiled-frames 0 --no-cpu > "$OUT/b_$1_$round.json" 2>> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python - "$OUT/b_$1_$round.json" "$1" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rl = r['roofline']; td = rl.get('traffic_detail') or {}
print(sys.argv[2], 'value', r['value'], 'kernel_us', rl.get('kernel_us_per_frame'), 'fetch_raw', td.get('fetch_bytes_raw'), 'write', td.get('write_bytes'), 'req', rl['request_bytes']['per_frame'])
PY
  done
done
