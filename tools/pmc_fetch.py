#!/usr/bin/env python3
"""Median FETCH_SIZE / WRITE_SIZE (KiB -> bytes) per dispatch of the largest-grid non-counting
trace_kernel launches in a rocprofv3 --pmc CSV output directory, divided by the frames of a
launch.   python tools/pmc_fetch.py <dir> <frames_per_launch> [label]"""
import csv
import re
import statistics
import sys
from pathlib import Path

d, frames = Path(sys.argv[1]), int(sys.argv[2])
label = sys.argv[3] if len(sys.argv) > 3 else d.name
rows = {}
for f in d.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" not in r["Kernel_Name"] or re.search(r"trace_kernel<\d+, true", r["Kernel_Name"]):
            continue
        x = rows.setdefault(r["Dispatch_Id"], {"grid": int(r["Grid_Size"]), "v": {}})
        x["v"][r["Counter_Name"]] = x["v"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
g = max(x["grid"] for x in rows.values())
sel = [x["v"] for x in rows.values() if x["grid"] == g]
out = {"label": label, "launches": len(sel)}
for k in sorted({k for v in sel for k in v}):
    out[k + "_per_frame"] = round(statistics.median(v[k] for v in sel if k in v) * (1024 if k.endswith("SIZE") else 1) / frames)
print(out)
