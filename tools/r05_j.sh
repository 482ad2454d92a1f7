#!/usr/bin/env bash
# Round 5: mesh per-pixel kernel register pressure — the rolled light loop (product) vs the
# shading state parked in LDS around the walks (park1) and the unrolled light loop without the
# frame-pair copies (unroll): kbench C4 / C3 / C5 and PMC WRITE_SIZE on C4; the FETCH
# calibration with aligned regions.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05j}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do
  for lib in prod park1 unroll; do
    L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
    for cf in "C4 20" "C3 200" "C5 4"; do
      set -- $cf
      TRT_LIB=$L timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --tag "$lib:$1" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
for round in 1 2; do
  for ppw in 64 32 16; do
    for cf in ref readme; do
      for inf in 16 2; do
        TRT_DEFER_PPW=$ppw timeout -k 10 150 python tools/kbench.py --config $cf --frames 160 --inflight $inf --tag "ppw$ppw:$cf:$inf" >> "$OUT/kb_ppw.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
      done
    done
  done
done
python - "$OUT/kb_ppw.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append((r['wall_us_no_events'], r['med_us']))
for k in sorted(d): print(k, 'wall us/frame', [x[0] for x in d[k]], 'span us', [x[1] for x in d[k]])
PY
cd /tmp && export TMPDIR=/tmp
for lib in prod park1 unroll; do
  L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
  TRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_$lib" -o run -- python "$ROOT/tools/kbench.py" --config C4 --frames 4 --settle-ms 0 --inflight 1 > "$OUT/pmc_$lib.log" 2>&1 || { tail -5 "$OUT/pmc_$lib.log"; exit 1; }
  python "$ROOT/tools/pmc_fetch.py" "$OUT/pmc_$lib" 4 "$lib"
done
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/cal_fetch" -o run -- "$ROOT/tools/calib/fetch_calib" > "$OUT/cal_fetch.log" 2>&1 || { tail -5 "$OUT/cal_fetch.log"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d "$OUT/cal_req" -o run -- "$ROOT/tools/calib/fetch_calib" > "$OUT/cal_req.log" 2>&1 || { tail -5 "$OUT/cal_req.log"; exit 1; }
grep '^{' "$OUT/cal_fetch.log"
echo done
