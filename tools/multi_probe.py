#!/usr/bin/env python3
"""trt_render_multi_frames on this process's GPUs (default: device 0 only) for one config:
wall time per frame, and with a rocprofv3 kernel trace (tools/multi_probe.sh) the GPU busy
fraction of the timed loop.

  python tools/multi_probe.py --config C2 --frames 400 --per-gather 8
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--per-gather", type=int, default=8)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=0, help="frames in flight of each device context")
    ap.add_argument("--prior-renderer", action="store_true",
                    help="first run and close a plain Renderer frame loop (as bench.py does)")
    ap.add_argument("--torch-stream", action="store_true", help="join the multi context into a torch stream")
    ap.add_argument("--count-pass", action="store_true", help="a counting draw_frame before the loop")
    a = ap.parse_args()
    import torch

    from vkcomputeshader_tinyraytracer_amd import scene as S
    from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, MultiRenderer

    sc = S.CONFIGS[a.config]()
    p = sc.params()
    if a.prior_renderer:
        from vkcomputeshader_tinyraytracer_amd import Renderer

        r = Renderer(0)
        r.upload_scene(sc)
        o8 = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        r.set_stream(torch.cuda.Stream())
        r.render_frames(p, o8, 100)
        torch.cuda.synchronize()
        r.close()
    m = MultiRenderer(devices=(0,))
    if a.inflight:
        L = m._L
        L.trt_set_frames_in_flight(L.trt_multi_context(m._h, 0), a.inflight)
    m.upload_scene(sc)
    if a.count_pass:
        m.draw_frame(p, band_rows=a.band_rows, root=0, count=True)
    if a.torch_stream:
        m.set_stream(0, torch.cuda.Stream())
    out = torch.zeros((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    m.render_frames(p, 16, a.band_rows, ROOT_ROTATE, a.per_gather, outs=[out])
    m.synchronize()
    t0 = time.perf_counter()
    m.render_frames(p, a.frames, a.band_rows, ROOT_ROTATE, a.per_gather, outs=[out])
    t1 = time.perf_counter()
    m.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"config": a.config, "frames": a.frames, "per_gather": a.per_gather, "inflight": a.inflight,
                      "prior_renderer": a.prior_renderer, "torch_stream": a.torch_stream, "count_pass": a.count_pass,
                      "host_enqueue_us_per_frame": round((t1 - t0) / a.frames * 1e6, 2),
                      "wall_us_per_frame": round((t2 - t0) / a.frames * 1e6, 2)}), flush=True)
    m.close()


if __name__ == "__main__":
    main()
