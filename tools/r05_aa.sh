#!/usr/bin/env bash
# Round 5 (verdict item 3): the C2 kernel's VALU instructions attributed to stages.  PMC
# SQ_INSTS_VALU / SQ_WAVES of the 20-frame C2 loop for the product and diagnostic builds that
# remove one stage each (they change the image: pricing only): no shadow rays, no pow (Phong and
# gamma), envmap u/v without atan2/acos, envmap u/v trig without the texel gathers, no envmap at
# all (runtime flag), launch + store only; plus their kernel times.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05aa}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=32
for v in "prod prod" "noshadow noshadow" "nopow nopow" "notrig notrig" "noenvfetch noenvfetch" "noenv prod --flags ${NOENV_FLAGS}" "trivial trivial"; do
  set -- $v
  name=$1; lib=$2; shift 2
  L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
  TRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS --kernel-trace --output-format csv -d "$OUT/pmc_$name" -o run -- python3 "$ROOT/tools/kbench.py" --config C2 --frames 40 --frame-batch 20 --settle-ms 0 "$@" > "$OUT/pmc_$name.log" 2>&1 || { tail -5 "$OUT/pmc_$name.log"; exit 1; }
  TRT_LIB=$L timeout -k 10 120 python3 "$ROOT/tools/kbench.py" --config C2 --frames 200 --frame-batch 20 "$@" --tag "$name" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, json, sys, collections
from pathlib import Path
out = Path(sys.argv[1])
times = {}
for l in open(out / "kb.jsonl"):
    if l.startswith("{"):
        r = json.loads(l); times[r["tag"]] = r["med_us"]
for d in sorted(out.glob("pmc_*")):
    if not d.is_dir():
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "trace_kernel<3, false" not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        continue
    last = [per[k] for k in sorted(per, key=int)][-1]
    waves = last["SQ_WAVES"]
    row = {"variant": d.name[4:], "waves": waves, "us_per_frame": times.get(d.name[4:])}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_INSTS_LDS"):
        row[k.lower() + "_per_wave"] = round(last[k] / waves, 1) if waves else None
    print(json.dumps(row))
PY
