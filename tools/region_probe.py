"""Where the time of a short timed region goes with multi-frame launches (the driver runs
bench.py --steps 20).  For K frames of C2 (camera walk) through trt_render_frames:
  wall     synchronize -> perf_counter -> render_frames -> synchronize (bench.timed)
  enqueue  host time of the render_frames call alone
  gpu      torch events on the caller's stream around the call (GPU span incl. queue gaps)
  empty    the same region with nothing enqueued (synchronize round trip)
Usage: python tools/region_probe.py [--inflight N] [--batch B] [--reps R]
"""
from __future__ import annotations

import argparse
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=0)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--tiled", action="store_true", help="the multi-GPU path at one rank (trt_render_multi_frames)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt

    sc = trt.config_c2()
    p = sc.params()
    wk = trt.camera_path(sc.ubo, 16)
    r = trt.Renderer(0)
    r.upload_scene(sc)
    fb = p.height * p.width * 4
    out = torch.empty((64, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    r.set_stream(s)
    r.set_frames_in_flight(a.inflight)
    r.set_frame_batch(a.batch)
    ubos = np.stack([wk[i % 16] for i in range(64)])
    r.render_frames(p, out, 64, ubos=ubos, frame_stride=fb)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    m = None
    if a.tiled:
        from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, MultiRenderer

        m = MultiRenderer([0])
        m.upload_scene(sc)
        m.set_stream(0, s)
        m.render_frames(p, 64, 8, ROOT_ROTATE, 64, outs=[out], frame_stride=fb, ubos=ubos)
        m.render_frames(p, 64, 8, ROOT_ROTATE, 32, outs=[out], frame_stride=fb, ubos=ubos)
        torch.cuda.synchronize()
    uk = {k: np.ascontiguousarray(ubos[:k]) for k in (1, 5, 20, 64)}

    def region(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if k:
            e0.record(s)
            t1 = time.perf_counter()
            if m is not None:
                m.render_frames(p, k, 8, ROOT_ROTATE, 64, outs=[out], frame_stride=fb, ubos=uk[k])
            else:
                r.render_frames(p, out, k, ubos=uk[k], frame_stride=fb)
            t2 = time.perf_counter()
            e1.record(s)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if not k:
            return (t3 - t0) * 1e6, 0.0, 0.0
        return (t3 - t0) * 1e6, (t2 - t1) * 1e6, e0.elapsed_time(e1) * 1e3

    for k in (0, 1, 5, 20, 64):
        rs = [region(k) for _ in range(a.reps)]
        wall = statistics.median(x[0] for x in rs)
        enq = statistics.median(x[1] for x in rs)
        gpu = statistics.median(x[2] for x in rs)
        print(f"K={k:3d} wall {wall:8.1f} us ({wall / max(k, 1):6.2f}/frame)  enqueue {enq:7.1f} us  "
              f"gpu span {gpu:8.1f} us ({gpu / max(k, 1):6.2f}/frame)", flush=True)
    if m is not None:
        m.close()
    r.close()


if __name__ == "__main__":
    main()
