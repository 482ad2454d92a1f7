#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 --pmc passes (tools/r06.sh stage `pmc`): every counter
summed over a kernel's dispatches, per wave, and the derived rates — VALU lanes per instruction
(SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU), the share of wave cycles waiting (SQ_WAIT_INST_ANY
/ SQ_WAVE_CYCLES) and issuing VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES), and TA / TD busy per
unit (the *_BUSY_sum counters over the 256 CUs and GRBM_GUI_ACTIVE / 8: that counter is summed over
the 8 XCDs, checked against the dispatch durations).  rocprofv3 serialises the
dispatches it counts, so these describe each kernel running alone.

  python tools/pmc_kernels.py gpurun_out/r06h/pmc [regex]   -> one JSON line per kernel
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

NCU = 256
NXCD = 8  # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (8 x the dispatch's cycles at the shader clock)


def main():
    root = Path(sys.argv[1])
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else re.compile(r"trace_|defer_")
    tot = defaultdict(lambda: defaultdict(float))
    grbm = defaultdict(lambda: defaultdict(float))  # GRBM_GUI_ACTIVE per pass (several passes may count it)
    busy_pass = defaultdict(dict)                    # the pass that counted each *_BUSY counter
    disp = defaultdict(set)
    for f in sorted(root.glob("*/**/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not pat.search(name):
                continue
            cn, v = r["Counter_Name"], float(r["Counter_Value"])
            if cn == "GRBM_GUI_ACTIVE":
                grbm[name][f.parent.name] += v
            else:
                tot[name][cn] += v
                if "BUSY" in cn:
                    busy_pass[name][cn] = f.parent.name
            disp[name].add((f.parent.name, r["Dispatch_Id"]))
    for name, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        waves = c.get("SQ_WAVES", 0) or float("nan")
        out = {"kernel": name, "dispatches_counted": len(disp[name])}
        if "SQ_WAVES" in c:
            out["waves"] = c["SQ_WAVES"]
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
                      "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if k in c:
                    out[k.lower() + "_per_wave"] = round(c[k] / waves, 1)
        if c.get("SQ_ACTIVE_INST_VALU"):
            if "SQ_THREAD_CYCLES_VALU" in c:
                out["valu_lanes"] = round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 1)
            if c.get("SQ_WAVE_CYCLES"):
                out["valu_issue_frac_of_wave_cycles"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 3)
        if c.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    out[k.lower() + "_frac"] = round(c[k] / c["SQ_WAVE_CYCLES"], 3)
        for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_BUSY_avr", "TD_BUSY_avr"):
            g = grbm[name].get(busy_pass[name].get(k, ""), 0.0)
            if k in c and g:
                div = g / NXCD * (NCU if k.endswith("_sum") else 1)
                out[k.lower() + "_frac"] = round(c[k] / div, 3)
        for k in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
            if k in c:
                out[k.lower()] = c[k]
        print(json.dumps(out))


if __name__ == "__main__":
    main()
