#!/usr/bin/env bash
# Round 5: active lanes per VALU instruction (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU) of the
# deep frame's passes (shipped frame, 1 and 2 in flight: pass A at one and two waves per tile)
# and of the C4 / C2 kernels, on the closing build.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05af}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=32
for v in "ref 1" "ref 2" "C4 1" "C2 1"; do
  set -- $v
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_$1_$2" -o run -- python3 "$ROOT/tools/kbench.py" --config $1 --frames 6 --inflight $2 --settle-ms 0 > "$OUT/pmc_$1_$2.log" 2>&1 || { tail -5 "$OUT/pmc_$1_$2.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, sys, collections, json
from pathlib import Path
out = Path(sys.argv[1])
for d in sorted(out.glob("pmc_*")):
    if not d.is_dir():
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if ", true," in name[:40]:
                continue  # counting passes
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        if v.get("SQ_ACTIVE_INST_VALU"):
            print(json.dumps({"run": d.name[4:], "kernel": k, "lanes_per_valu": round(v["SQ_THREAD_CYCLES_VALU"] / v["SQ_ACTIVE_INST_VALU"], 1),
                              "valu_per_wave": round(v["SQ_INSTS_VALU"] / max(v["SQ_WAVES"], 1), 1), "waves": v["SQ_WAVES"]}))
PY
