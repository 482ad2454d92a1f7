#!/usr/bin/env python3
"""Recomputes a bench line's kernel roofline from a committed rocprofv3 kernel-stats CSV.

The bench's `roofline.kernel_us_per_frame` is the HIP-event span of its timed launches divided
by the frames they traced (one plain launch traces many frames).  A `rocprofv3 --kernel-trace
--stats` run of a loop with launches of the same size gives the same figure as
TotalDurationNs / frames traced by the matching kernels; with the bench line's counted
`flops_per_frame` that is the kernel fraction of the FP32 VALU peak.

  python tools/roofline_check.py --csv profiles/r03_rocprof_kernel_stats_c2_b20.csv \\
      --kernel 'trace_kernel<\\d+, false, 0,' --frames 1925 --bench profiles/r03_bench_20steps_final.log
"""
from __future__ import annotations

import argparse
import csv
import json
import re

PEAK_TF = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", required=True)
    ap.add_argument("--kernel", required=True, help="regex over kernel names (summed)")
    ap.add_argument("--frames", type=int, default=0, help="frames traced by the matching launches (total time / frames)")
    ap.add_argument("--frames-per-call", type=int, default=0,
                    help="instead: frames each matching launch traces; kernel time = the median launch / this "
                         "(the CSV's MedianNs, tools/rocpd_stats.py)")
    ap.add_argument("--bench", required=True, help="log holding the bench JSON line")
    ap.add_argument("--key", default="roofline", help="dotted path of the roofline object in the line")
    a = ap.parse_args()
    rx = re.compile(a.kernel)
    total_ns, calls, median_ns = 0.0, 0, None
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            if rx.search(row["Name"]):
                total_ns += float(row["TotalDurationNs"])
                calls += int(row["Calls"])
                median_ns = float(row["MedianNs"]) if row.get("MedianNs") else None
    line = None
    for s in open(a.bench):
        if s.startswith("{"):
            line = json.loads(s)
    rl = line
    for k in a.key.split("."):
        rl = rl[k]
    if a.frames_per_call:
        assert median_ns is not None, "the CSV has no MedianNs column (tools/rocpd_stats.py)"
        us = median_ns / a.frames_per_call / 1e3
    else:
        us = total_ns / a.frames / 1e3
    frac = rl["flops_per_frame"] / (us * 1e-6) / 1e12 / PEAK_TF
    out = {"calls": calls, "frames": a.frames, "kernel_us_per_frame_csv": round(us, 3),
           "kernel_frac_csv": round(frac, 4), "kernel_us_per_frame_line": rl.get("kernel_us_per_frame"),
           "kernel_frac_line": rl.get("kernel_frac"), "us_per_frame_wall_line": rl["us_per_frame"],
           "frac_line": rl["frac"]}
    if rl.get("kernel_frac"):
        out["ratio_csv_over_line"] = round(frac / rl["kernel_frac"], 4)
    out["kernel_le_wall"] = us <= rl["us_per_frame"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
