#!/usr/bin/env python3
"""Deferred-frame scratch use along the bench's camera walk: per frame of a frames-in-flight
loop, the event chunks and shadow queries its slot took against the capacities, and the pixels
re-traced in place (trt_defer_stats).  A pixel whose event chunk or query does not fit goes to
the per-pixel fallback after pass C, which lengthens the frame.

  python tools/defer_probe.py [--config ref|readme] [--inflight 2] [--frames 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) <= 4:
    os.environ["GPU_MAX_HW_QUEUES"] = "32"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ref")
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--frames", type=int, default=64)
    a = ap.parse_args()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = S.config_reference_default() if a.config == "ref" else S.config_readme()
    p = sc.params()
    ubos = S.camera_path(sc.ubo, a.frames)
    fb, chunks, queries = [], [], []
    with trt.Renderer(0) as r:
        r.upload_scene(sc)
        r.set_frames_in_flight(a.inflight)
        out = torch.zeros((a.inflight, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        for i in range(0, a.frames, a.inflight):
            n = min(a.inflight, a.frames - i)
            r.render_frames(p, out, n, ubos=np.stack(ubos[i:i + n]), frame_stride=p.height * p.width * 4)
            torch.cuda.synchronize()
            for s in range(n):
                st = r.defer_stats(s)
                fb.append(st["fallback_pixels"])
                chunks.append(st["chunks"] / max(st["chunk_cap"], 1))
                queries.append(st["queries"] / max(st["query_cap"], 1))
    print(json.dumps({
        "config": a.config, "in_flight": a.inflight, "frames": len(fb),
        "frames_with_fallback": int(sum(1 for x in fb if x)), "fallback_pixels_max": int(max(fb)),
        "fallback_pixels_mean": round(float(np.mean(fb)), 1),
        "chunk_use_max": round(float(max(chunks)), 3), "query_use_max": round(float(max(queries)), 3),
    }), flush=True)


if __name__ == "__main__":
    main()
