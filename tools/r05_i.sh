#!/usr/bin/env bash
# Round 5: (1) FETCH_SIZE calibration for the tracer's access patterns (tools/calib); (2) the GPU
# suite on the current build (spatial-split BVH, rolled mesh light loop, packed sphere prologue);
# (3) packed sphere prologue vs scalar (variant pk0) on C2, kbench 20-frame launches.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05i}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/cal_fetch" -o run -- "$ROOT/tools/calib/fetch_calib" > "$OUT/cal_fetch.log" 2>&1 || { tail -5 "$OUT/cal_fetch.log"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d "$OUT/cal_req" -o run -- "$ROOT/tools/calib/fetch_calib" > "$OUT/cal_req.log" 2>&1 || { tail -5 "$OUT/cal_req.log"; echo "req pass failed (counters?)"; }
grep '^{' "$OUT/cal_fetch.log"
python3 - "$OUT" <<'PY'
import csv, sys
from pathlib import Path
for sub in ("cal_fetch", "cal_req"):
    for f in Path(sys.argv[1], sub).rglob("*counter_collection.csv"):
        rows = {}
        for r in csv.DictReader(open(f)):
            rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = rows.get(int(r["Dispatch_Id"]), {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k in sorted(rows): print(sub, k, rows[k])
PY
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for round in 1 2 3; do
  for lib in prod pk0; do
    L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
    TRT_LIB=$L timeout -k 10 200 python tools/kbench.py --config C2 --frames 20 --tag "$lib:C2" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    TRT_LIB=$L timeout -k 10 200 python tools/kbench.py --config C2 --frames 64 --tag "$lib:C2_64" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
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
cd /tmp
for cf in "C4 4" "C3 20" "ref 4"; do
  set -- $cf
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_$1_$ctr" -o run -- python "$ROOT/tools/kbench.py" --config $1 --frames $2 --settle-ms 0 --inflight 1 > "$OUT/pmc_$1_$ctr.log" 2>&1 || { tail -5 "$OUT/pmc_$1_$ctr.log"; exit 1; }
  done
done
echo pmc done
