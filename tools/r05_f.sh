#!/usr/bin/env bash
# Round 5: fixed (unrotated, permuted-class) frame-interleaved dealing (TRT_XCD_INTER=2) vs the
# rotating one (1): bench.py headline + live PMC traffic, interleaved rounds; the dealing tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05f}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k xcd_dealing > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for round in 1 2 3; do
  for v in "inter1 1" "inter2 2"; do
    set -- $v
    TRT_XCD_INTER=$2 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --legs '' --extra-frames 0 \
        --tiled-frames 0 --no-cpu > "$OUT/b_$1_$round.json" 2>> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python - "$OUT/b_$1_$round.json" "$1" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rl = r['roofline']; td = rl.get('traffic_detail') or {}
print(sys.argv[2], 'value', r['value'], 'kernel_us', rl.get('kernel_us_per_frame'), 'fetch_raw', td.get('fetch_bytes_raw'), 'write', td.get('write_bytes'), 'req', rl['request_bytes']['per_frame'])
PY
  done
done
for v in "inter1 1" "inter2 2"; do
  set -- $v
  TRT_XCD_INTER=$2 timeout -k 10 240 python bench.py --steps 1000 --warmup 20 --legs '' --extra-frames 0 \
      --tiled-frames 0 --no-cpu --traffic off > "$OUT/b1000_$1.json" 2>> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
  python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '1000 steps', r['value'], r['roofline'].get('kernel_us_per_frame'))" "$OUT/b1000_$1.json" "$1"
done
