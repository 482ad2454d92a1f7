#!/usr/bin/env python3
"""Summarise tools/pmc_r03.sh: per configuration and kernel family, the median per dispatch
(one frame per dispatch) of every counter, plus derived figures:
  * HBM bytes per frame: FETCH_SIZE + WRITE_SIZE (KiB x 1024, separate passes).  On gfx950
    FETCH_SIZE reports 1/2 of the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM);
    these kernels read by 4/8/16-B per-lane gathers and scalar loads, an uncalibrated width, so
    both the raw and the x2 figure are given and `traffic_bytes` is the raw one (lower bound);
  * TA / TD busy per CU, VALU active lanes, wave-cycle fractions, L1 / L2 hit rates.
usage: python tools/pmc_summary_r03.py gpurun_out/pmc_r03 profiles/r03_pmc_summary.json
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys
from collections import defaultdict
from pathlib import Path

CUS = 256


def family(name: str) -> str | None:
    if re.search(r"trace_kernel<\d+, true", name):
        return None  # counting passes
    if "trace_kernel" in name:
        return "trace_kernel (pass A)" if re.search(r"trace_kernel<\d+, false, \d, (true|false), true", name) else "trace_kernel"
    for k in ("defer_shadows", "defer_resolve", "defer_fallback", "envp_kernel"):
        if k in name:
            return k
    return None


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    vals: dict = defaultdict(lambda: defaultdict(list))
    for f in sorted(src.glob("*/run_counter_collection.csv")):
        cfg = f.parent.name.split("_")[0]
        per: dict = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam is None:
                continue
            d = per[(fam, r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["_dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d["_vgpr"] = int(r.get("VGPR_Count", 0) or 0)
        for (fam, _), d in per.items():
            for k, v in d.items():
                vals[(cfg, fam)][k].append(v)
    out = {}
    for (cfg, fam), kv in sorted(vals.items()):
        c = {k: statistics.median(v) for k, v in kv.items()}
        e = {"dispatches_median_of": len(kv.get("_dur_ns", [])), "counters": {k: v for k, v in c.items() if not k.startswith("_")},
             "dur_ns_under_pmc": c.get("_dur_ns"), "vgpr": c.get("_vgpr")}
        cc = e["counters"]
        if "FETCH_SIZE" in cc:
            e["fetch_bytes_raw"] = cc["FETCH_SIZE"] * 1024
            e["fetch_bytes_x2"] = 2 * cc["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in cc:
            e["write_bytes"] = cc["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in cc and "WRITE_SIZE" in cc:
            e["traffic_bytes"] = e["fetch_bytes_raw"] + e["write_bytes"]
        if "GRBM_GUI_ACTIVE" in cc:
            gui = cc["GRBM_GUI_ACTIVE"] / 8.0  # sums 8 XCDs
            if "TA_TA_BUSY_sum" in cc:
                e["ta_busy_frac_per_cu"] = cc["TA_TA_BUSY_sum"] / CUS / gui
            if "TD_TD_BUSY_sum" in cc:
                e["td_busy_frac_per_cu"] = cc["TD_TD_BUSY_sum"] / CUS / gui
        if "SQ_THREAD_CYCLES_VALU" in cc and "SQ_ACTIVE_INST_VALU" in cc and cc["SQ_ACTIVE_INST_VALU"]:
            e["valu_active_lanes"] = cc["SQ_THREAD_CYCLES_VALU"] / cc["SQ_ACTIVE_INST_VALU"]
        if "SQ_WAVE_CYCLES" in cc:
            for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY"):
                if k in cc:
                    e[k.lower() + "_frac_of_wave_cycles"] = cc[k] / cc["SQ_WAVE_CYCLES"]
        if "SQ_WAVES" in cc and cc["SQ_WAVES"]:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD"):
                if k in cc:
                    e[k.lower() + "_per_wave"] = cc[k] / cc["SQ_WAVES"]
        if "TCC_HIT_sum" in cc:
            e["l2_hit_rate"] = cc["TCC_HIT_sum"] / max(1.0, cc["TCC_HIT_sum"] + cc["TCC_MISS_sum"])
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in cc and cc["TCP_TOTAL_CACHE_ACCESSES_sum"]:
            e["l1_hit_rate_approx"] = 1.0 - cc["TCP_TCC_READ_REQ_sum"] / cc["TCP_TOTAL_CACHE_ACCESSES_sum"]
        out.setdefault(cfg, {})[fam] = e
    out["note"] = ("tools/pmc_r03.sh: tools/kbench.py, one launch per frame (--frame-batch 1), 1 frame in flight; "
                   "medians per dispatch = per frame; GRBM_GUI_ACTIVE sums 8 XCDs; FETCH_SIZE raw (see docstring)")
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1)[:6000])


if __name__ == "__main__":
    main()
