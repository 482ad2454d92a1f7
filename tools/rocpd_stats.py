#!/usr/bin/env python3
"""rocprofv3 --stats summary from its SQLite output (this rocprofv3 writes run_results.db by
default): one row per kernel name with the columns of rocprofv3's kernel_stats.csv, plus
`Workgroups` (the dispatches' grid size / workgroup size, summed) so a one-wave-per-tile
launch's frame count is Workgroups / tiles per frame.

  python tools/rocpd_stats.py gpurun_out/rp_c2_b20/run_results.db profiles/r03_rocprof_kernel_stats_c2_b20.csv
  --split-grid: one row per (kernel, workgroups per dispatch), e.g. to separate a bench run's
  20-frame launches of the C2 kernel from its single-frame ones.
"""
from __future__ import annotations

import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    split = "--split-grid" in sys.argv
    db, out = [a for a in sys.argv[1:] if not a.startswith("--")][:2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, workgroup_x from kernels").fetchall()
    by = defaultdict(list)
    wg = defaultdict(int)
    for name, dur, gx, wx in rows:
        if split:
            name = f"{name} [workgroups={int(gx) // max(int(wx), 1)}]"
        by[name].append(float(dur))
        wg[name] += int(gx) // max(int(wx), 1)
    total = sum(sum(v) for v in by.values()) or 1.0
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev",
                    "Workgroups", "MedianNs"])
        for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), int(sum(v)), sum(v) / len(v), round(100.0 * sum(v) / total, 2), int(min(v)),
                        int(max(v)), statistics.pstdev(v) if len(v) > 1 else 0.0, wg[name], statistics.median(v)])


if __name__ == "__main__":
    main()
