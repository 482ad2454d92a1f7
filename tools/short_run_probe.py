"""Where the fixed cost of a short timed region goes (the driver runs bench.py --steps 20).

For K in (1, 5, 20, 100, 1000) frames of C2 through the native frame loop, times the region
the way bench.timed does (synchronize, perf_counter, enqueue, synchronize) in three variants:
  plain     no events
  events    time_every=16 (the bench), event pool created inside the timed call
  prewarm   same, but the warmup call ran with timing so the pool already exists
and prints us per region and us per frame; fixed cost = intercept of the K -> time line.
Usage: python tools/short_run_probe.py [--inflight N] [--reps R]
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
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt

    sc = trt.config_c2()
    p = sc.params()
    r = trt.Renderer(0)
    r.upload_scene(sc)
    out = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    r.set_stream(s)
    r.set_frames_in_flight(a.inflight)
    r.render_frames(p, out, 50)
    torch.cuda.synchronize()

    def region(k, timing, prewarm):
        if prewarm:
            r.render_frames(p, out, 5, timing=True, time_every=1)  # pool of >= 10 events
        else:
            r.render_frames(p, out, 5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.render_frames(p, out, k, timing=timing, time_every=16)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    for variant in ("plain", "events", "prewarm"):
        for k in (1, 5, 20, 100, 1000):
            ts = [region(k, variant != "plain", variant == "prewarm") for _ in range(a.reps)]
            med = statistics.median(ts)
            print(f"{variant:8s} K={k:5d} region {med:9.1f} us  per frame {med / k:7.2f} us  "
                  f"min {min(ts):9.1f}", flush=True)
    r.close()


if __name__ == "__main__":
    main()
