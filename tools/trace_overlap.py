#!/usr/bin/env python3
"""From a rocprofv3 kernel_trace.csv: for kernels whose name contains PATTERN, the busy time
(union of [start, end] intervals), the mean concurrency and the gaps of the last N launches.

  python tools/trace_overlap.py gpurun_out/prof_x/run_kernel_trace.csv trace_kernel 512
"""
import csv
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    if last:
        iv = iv[-last:]
    t0, t1 = iv[0][0], max(e for _, e in iv)
    busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = sum(e - s for s, e in iv)
    print({"launches": len(iv), "span_us": (t1 - t0) / 1e3, "busy_us": busy / 1e3,
           "busy_frac": round(busy / (t1 - t0), 3), "mean_concurrency_when_busy": round(tot / busy, 2),
           "per_launch_us": round(tot / len(iv) / 1e3, 2), "wall_per_launch_us": round((t1 - t0) / len(iv) / 1e3, 2)})


if __name__ == "__main__":
    main()
