#!/usr/bin/env bash
# Round 4: GEOM 3 per-pixel loop with its deferred children in a private array and the LDS given
# to the BVH stack (24 / 32 entries) vs the product (8 entries + children in LDS): kbench after a
# settle, 3 interleaved rounds, then one WRITE_SIZE PMC pass of C4 per build.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04o}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
VS=${VARIANTS:-cur g3p24 g3p32}
for round in $(seq 1 ${ROUNDS:-3}); do
  for v in $VS; do
    for cf in "C4 20" "C3 60" "ref 100" "readme 100"; do
      set -- $cf
      TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --tag "$v" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[(r['config'], r['tag'])].append(r['wall_us_no_events'])
for k in sorted(d): print(k, d[k], 'median', statistics.median(d[k]))
PY
for v in ${PMC_VARIANTS-$VS}; do
  (cd /tmp && TRT_LIB="$ROOT/variants/libtrt_$v.so" timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_$v" -o run -- python3 "$ROOT/tools/kbench.py" --config C4 --frames 4 --settle-ms 0 > "$OUT/pmc_$v.log" 2>&1) || { tail -5 "$OUT/pmc_$v.log"; exit 1; }
  python - "$OUT/pmc_$v" "$v" <<'PY'
import csv, sys, statistics, pathlib, re
per = {}
for f in pathlib.Path(sys.argv[1]).rglob("run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if re.search(r"trace_kernel<3, false, 3", r["Kernel_Name"]) and r["Counter_Name"] == "WRITE_SIZE":
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"]) * 1024
vals = list(per.values())
print(sys.argv[2], "C4 trace_kernel WRITE bytes per dispatch (median of", len(vals), "):", statistics.median(vals) if vals else None)
PY
done
