#!/usr/bin/env python3
"""Workgroup timeline of one frame (diagnostic build: TRT_LIB=variants/libtrt_clock.so, built by
tools/build_variants.sh clock).  Each 64-lane workgroup (one 8x8 tile) records its tile, XCD
and start/end of the 100 MHz constant clock; this prints the frame span, workgroup duration
percentiles, the occupancy curve and the tail (time the last workgroups run alone).

  TRT_LIB=variants/libtrt_clock.so python tools/waveclock.py [--config C2] [--out f.npz]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--records", type=int, default=0,
                    help="workgroup records (default: one per tile; a deferred frame's pass A: tiles x defer_sub)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = S.config_reference_default() if a.config == "ref" else S.CONFIGS[a.config]()
    p = sc.params()
    r = trt.Renderer(0)
    r.upload_scene(sc)
    ntiles = a.records or ((p.width + 7) // 8) * ((p.height + 7) // 8)
    out8 = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    rec = torch.zeros((p.height, p.width, 4), dtype=torch.float32, device="cuda")
    res = []
    for _ in range(a.frames):
        r.draw_frame(p, out8=out8, out32=rec)
        torch.cuda.synchronize()
        raw = rec.view(torch.int32).flatten()[: 4 * ntiles].cpu().numpy().view(np.uint32).reshape(ntiles, 4)
        res.append(raw.copy())
    raw = res[-1]
    t0 = (raw[:, 3].astype(np.int64) << 32) | raw[:, 1].astype(np.int64)
    t1 = t0 + raw[:, 2].astype(np.int64)
    xcd = raw[:, 0] >> 28
    # each XCD has its own constant clock: align every XCD's first start to 0
    base = np.zeros_like(t0)
    for k in np.unique(xcd):
        base[xcd == k] = t0[xcd == k].min()
    s, e = (t0 - base) * 10, (t1 - base) * 10  # ns
    dur = e - s
    span = e.max()
    ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    peak = int(conc.max())
    # time during which fewer than half the peak workgroups are resident
    low = 0
    for i in range(len(ev) - 1):
        if conc[i] < peak / 2:
            low += ev[i + 1, 0] - ev[i, 0]
    tile = raw[:, 0] & 0x0FFFFFFF
    out = {
        "config": a.config, "workgroups": int(ntiles), "span_us": span / 1e3,
        "dur_us": {q: float(np.percentile(dur, q)) / 1e3 for q in (10, 50, 90, 99, 100)},
        "mean_dur_us": float(dur.mean()) / 1e3, "peak_resident": peak,
        "ideal_us": float(dur.sum() / peak) / 1e3,
        "time_below_half_peak_us": float(low) / 1e3,
        "last_start_us": float(s.max()) / 1e3,
        "per_xcd_busy_end_us": [float(e[xcd == k].max()) / 1e3 for k in range(8) if (xcd == k).any()],
    }
    print(json.dumps(out), flush=True)
    if a.out:
        np.savez_compressed(a.out, raw=raw, tile=tile, xcd=xcd, start_ns=s, end_ns=e, width=p.width)
    r.close()


if __name__ == "__main__":
    main()
