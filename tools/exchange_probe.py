#!/usr/bin/env python3
"""Cost of the tiled path's exchange, measured on one GPU.

trt_render_multi_frames at one rank with G band groups per rank renders every group of every
frame; with trt_multi_set_self_gather the groups then travel the way a peer's would: compact
buffers, one grouped ncclSend/ncclRecv per batch (to itself), the gather-buffer layout and the
re-interleave kernel.  The difference between the two is the per-frame cost of the exchange's
GPU work on the root of an N = G run (minus the xGMI transfer time itself, which a self-send
does not pay): DESIGN.md §6 projects the N-GPU loop from it.

  python tools/exchange_probe.py [--config C2] [--frames 256] [--per-gather 32] [--groups 1 2 4 8]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--per-gather", type=int, nargs="+", default=[8, 32, 64])
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    from vkcomputeshader_tinyraytracer_amd import camera_path, scene as S
    from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, MultiRenderer

    sc = S.CONFIGS[a.config]()
    p = sc.params()
    ubos = np.stack([u for u in camera_path(sc.ubo, 16)] * (a.frames // 16 + 1))[: a.frames]
    fb = p.width * p.height * 4
    out = torch.zeros((a.frames, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    m = MultiRenderer([0])
    m.upload_scene(sc)
    s = torch.cuda.Stream()
    m.set_stream(0, s)
    rows = []
    for G in a.groups:
        m.set_band_groups(G)
        for F in a.per_gather:
            res = {"groups": G, "per_gather": F}
            for sg in (False, True):
                m.set_self_gather(sg)
                m.render_frames(p, min(a.frames, 2 * F), 8, ROOT_ROTATE, F, outs=[out], frame_stride=fb, ubos=ubos)
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    m.render_frames(p, a.frames, 8, ROOT_ROTATE, F, outs=[out], frame_stride=fb, ubos=ubos)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                res["self_gather_us_per_frame" if sg else "in_place_us_per_frame"] = round(
                    statistics.median(ts) / a.frames * 1e6, 2)
            res["exchange_us_per_frame"] = round(res["self_gather_us_per_frame"] - res["in_place_us_per_frame"], 2)
            rows.append(res)
            print(json.dumps(res), flush=True)
    m.close()


if __name__ == "__main__":
    main()
