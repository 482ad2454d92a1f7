#!/usr/bin/env bash
# Round 5: envmap layout for the C2 gathers — pair rows (one 16-B load per footprint, every texel
# row stored twice) vs plain row-major texels (two 8-B loads per footprint): time and live PMC
# traffic of bench.py's headline loop, interleaved rounds.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05l}"
mkdir -p "$OUT"
cd "$ROOT"
for round in 1 2; do
  for v in "pairrows 1" "rowmajor 0"; do
    set -- $v
    TRT_ENV_PAIRROWS=$2 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --legs '' --extra-frames 0 \
        --tiled-frames 0 --no-cpu > "$OUT/b_$1_$round.json" 2>> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python - "$OUT/b_$1_$round.json" "$1" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rl = r['roofline']; td = rl.get('traffic_detail') or {}
print(json.dumps({"variant": sys.argv[2], "value": r['value'], "kernel_us": rl.get('kernel_us_per_frame'), "fetch_raw": td.get('fetch_bytes_raw'), "write": td.get('write_bytes'), "traffic": rl.get('traffic')}))
PY
  done
done
