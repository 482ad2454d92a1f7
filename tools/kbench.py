#!/usr/bin/env python3
"""Quick kernel-time probe: median / min per-frame device time of the trace kernel for one
configuration (HIP events around each launch), no CPU baseline.

  python tools/kbench.py [--config C2] [--frames 100] [--width W --height H] [--depth D]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) <= 4:  # as the library (frames in flight = streams)
    os.environ["GPU_MAX_HW_QUEUES"] = "32"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--depth", type=int, default=0)
    ap.add_argument("--tag", default="")
    ap.add_argument("--inflight", type=int, default=0, help="frames in flight (0 = the library's auto)")
    ap.add_argument("--split", type=int, default=0, help="subtree split window (0 auto, 1 off, 2..5)")
    ap.add_argument("--defer", type=int, default=0, help="deferred shadows (0 auto, 1 off, 2 on)")
    ap.add_argument("--flags", type=lambda v: int(v, 0), default=None, help="override trt_params.flags")
    ap.add_argument("--frame-batch", type=int, default=0, help="frames per launch (0 auto, 1 = one per frame)")
    ap.add_argument("--settle-ms", type=float, default=50.0, help="untimed frames first for this long (clock ramp)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    kw = {}
    if a.width:
        kw = dict(width=a.width, height=a.height)
    if a.config == "ref":  # the shipped glass+water+ice frame
        sc = S.config_reference_default(**kw)
    elif a.config == "readme":  # the README-era scene (config.hpp:96)
        sc = S.config_readme(**kw)
    else:
        sc = S.CONFIGS[a.config](**kw)
    if a.depth:
        sc.max_depth = a.depth
    if a.flags is not None:
        sc.flags = a.flags
    p = sc.params()
    r = trt.Renderer(0)
    r.upload_scene(sc)
    _, _, st = r.draw_frame(p, count=True)
    out = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    r.set_stream(stream)
    r.set_frames_in_flight(a.inflight)
    r.set_subtree_split(a.split)
    r.set_deferred_shadows(a.defer)
    r.set_frame_batch(a.frame_batch)
    r.render_frames(p, out, 5)
    import time
    t_end = time.perf_counter() + a.settle_ms / 1e3
    while time.perf_counter() < t_end:
        r.render_frames(p, out, a.frames)
        torch.cuda.synchronize()
    nt = r.render_frames(p, out, a.frames, timing=True)
    ms = r.frame_times(nt)  # per frame of each launch
    torch.cuda.synchronize()
    # wall per frame of a back-to-back batch without per-frame events (one event pair)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    import time
    torch.cuda.synchronize()
    e0.record(stream)
    t0 = time.perf_counter()
    r.render_frames(p, out, a.frames)
    t1 = time.perf_counter()
    e1.record(stream)
    torch.cuda.synchronize()
    wall_noev = e0.elapsed_time(e1) / a.frames
    host_us = (t1 - t0) / a.frames * 1e6
    e0.record(stream)
    r.render_frames(p, out, a.frames, timing=True, time_every=16)
    e1.record(stream)
    torch.cuda.synchronize()
    wall_ev = e0.elapsed_time(e1) / a.frames
    rays = st["primary_rays"] + st["secondary_rays"]
    res = {"tag": a.tag, "inflight": a.inflight, "split": a.split, "defer": a.defer, "config": a.config,
           "size": [p.width, p.height], "depth": p.max_depth, "rays": rays,
           "med_us": round(float(np.median(ms)) * 1e3, 2), "min_us": round(float(ms.min()) * 1e3, 2),
           "Mray_s_kernel": round(rays / (float(np.median(ms)) * 1e-3) / 1e6, 1),
           "wall_us_no_events": round(wall_noev * 1e3, 2), "host_enqueue_us": round(host_us, 2), "wall_us_events_every16": round(wall_ev * 1e3, 2)}
    if a.defer != 1:
        res["defer_stats"] = r.defer_stats(0)
    print(json.dumps(res), flush=True)
    r.close()


if __name__ == "__main__":
    main()
