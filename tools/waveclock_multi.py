#!/usr/bin/env python3
"""Workgroup timeline of one multi-frame launch (diagnostic build: TRT_LIB=variants/libtrt_clock.so,
tools/build_variants.sh clock).  Every workgroup records (tile | frame << 20 | xcc << 28, start,
duration) of the 100 MHz constant clock into the diagnostic buffer; this prints the launch span,
the ramp (time until the resident count first reaches its peak), the tail (time from the moment
the resident count falls below half its peak for good to the end), per-frame end times and the
workgroup duration percentiles of the last frame.

  TRT_LIB=variants/libtrt_clock.so python tools/waveclock_multi.py [--config C2] [--frames 20]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) <= 4:
    os.environ["GPU_MAX_HW_QUEUES"] = "32"


def analyse(raw, F):
    import numpy as np

    t0 = (raw[:, 3].astype(np.int64) << 32) | raw[:, 1].astype(np.int64)
    t1 = t0 + raw[:, 2].astype(np.int64)
    xcd = raw[:, 0] >> 28
    frame = (raw[:, 0] >> 20) & 0xFF
    base = np.zeros_like(t0)
    for k in np.unique(xcd):  # each XCD has its own constant clock
        base[xcd == k] = t0[xcd == k].min()
    s, e = (t0 - base) * 10, (t1 - base) * 10  # ns
    ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
    ev = ev[np.lexsort((-ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    peak = int(conc.max())
    span = float(e.max())
    ramp = float(ev[int(np.argmax(conc >= 0.95 * peak)), 0])
    above = np.nonzero(conc >= peak / 2)[0]
    tail_start = float(ev[above[-1] + 1, 0]) if len(above) and above[-1] + 1 < len(ev) else span
    dur = e - s
    last = frame == frame.max()
    return {
        "frames": F, "workgroups": int(len(raw)), "span_us": span / 1e3, "peak_resident": peak,
        "ideal_us": float(dur.sum() / peak) / 1e3, "ramp_to_95pct_peak_us": ramp / 1e3,
        "tail_below_half_peak_us": (span - tail_start) / 1e3,
        "last_start_us": float(s.max()) / 1e3,
        # frame pairs record their first frame only (the block traces frames 2p and 2p + 1)
        "frame_end_us": [round(float(e[frame == f].max()) / 1e3, 2) for f in range(F) if (frame == f).any()],
        "dur_us_all": {q: round(float(np.percentile(dur, q)) / 1e3, 2) for q in (50, 90, 99, 100)},
        "dur_us_last_frame": {q: round(float(np.percentile(dur[last], q)) / 1e3, 2) for q in (50, 90, 99, 100)},
        "last_frame_longest_start_us": round(float(s[last][np.argmax(dur[last])]) / 1e3, 2),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = S.config_reference_default() if a.config == "ref" else S.CONFIGS[a.config]()
    p = sc.params()
    r = trt.Renderer(0)
    r.upload_scene(sc)
    L = r._L
    L.trt_diag_set_buffer.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ntiles = ((p.width + 7) // 8) * ((p.height + 7) // 8)
    F = a.frames
    buf = torch.zeros((F * ntiles, 4), dtype=torch.int32, device="cuda")
    out = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    r.set_stream(stream)
    r.set_frames_in_flight(1)
    r.set_frame_batch(F)
    r.render_frames(p, out, F)
    torch.cuda.synchronize()
    L.trt_diag_set_buffer(r._h, buf.data_ptr())
    res = []
    for _ in range(a.reps):
        r.render_frames(p, out, F)
        torch.cuda.synchronize()
        raw = buf.cpu().numpy().view(np.uint32).copy()
        res.append(analyse(raw, F))
    L.trt_diag_set_buffer(r._h, None)
    for x in res:
        print(json.dumps(x), flush=True)
    if a.out:
        np.savez_compressed(a.out, raw=raw, width=p.width)
    r.close()


if __name__ == "__main__":
    main()
