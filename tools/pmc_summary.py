#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per-dispatch averages of every counter for the timed trace
kernel (trace_kernel<*, false>), the HBM traffic per launch, and derived rates.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KiB) come from
separate passes; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a WIDE coalesced stream
(16 B/lane).  This kernel's reads are 4-B texel gathers and wave-uniform scalar loads, an
access width the guide lists as uncalibrated, so both the raw and the x2-corrected read
figures are written and `hbm_bytes_per_launch` uses the raw (uncorrected) value as the
conservative lower bound, stating so.

usage: python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_C2.json
"""
from __future__ import annotations

import csv
import re
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path


def load(pmc_dir: Path) -> dict:
    vals: dict = defaultdict(list)
    durs = []
    for f in sorted(pmc_dir.glob("*/run_counter_collection.csv")):
        per_dispatch: dict = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            # the timed frame kernel(s): trace_kernel<CAP, COUNT=false, GEOM, SPLIT>
            if "trace_kernel" not in name or re.search(r"trace_kernel<\d+, true", name):
                continue
            d = per_dispatch[r["Dispatch_Id"]]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["_dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d["_vgpr"] = int(r["VGPR_Count"])
            d["_sgpr"] = int(r["SGPR_Count"])
        for d in per_dispatch.values():
            for k, v in d.items():
                vals[k].append(v)
            durs.append(d["_dur"])
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    m = load(src)
    dur_ns = m.get("_dur", 0.0)
    out = {"kernel": "trace_kernel<CAP,false>", "median_dispatch_ns_under_pmc": dur_ns, "counters": {}}
    for k, v in sorted(m.items()):
        if not k.startswith("_"):
            out["counters"][k] = v
    out["vgpr"] = m.get("_vgpr")
    out["sgpr"] = m.get("_sgpr")
    c = out["counters"]
    if "FETCH_SIZE" in c:
        fetch = c["FETCH_SIZE"] * 1024.0
        write = c.get("WRITE_SIZE", 0.0) * 1024.0
        out["fetch_bytes_raw"] = fetch
        out["fetch_bytes_x2_corrected"] = 2 * fetch
        out["write_bytes"] = write
        out["hbm_bytes_per_launch"] = fetch + write
        out["hbm_bytes_note"] = ("FETCH_SIZE + WRITE_SIZE (KiB*1024), separate passes; reads are 4-B "
                                 "gathers + scalar loads (uncalibrated width): raw, not x2-corrected")
    if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
        out["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        out["salu_insts_per_wave"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"]
        out["smem_insts_per_wave"] = c.get("SQ_INSTS_SMEM", 0) / c["SQ_WAVES"]
        out["vmem_rd_insts_per_wave"] = c.get("SQ_INSTS_VMEM_RD", 0) / c["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in c and dur_ns:
        out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8.0 / dur_ns
    if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
        out["valu_active_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        out["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        out["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
