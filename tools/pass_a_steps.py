#!/usr/bin/env python3
"""Pass A of the deferred deep frames, step by step (diagnostic build TRT_DIAG_PASSA_STEPS,
tools/build_variants.sh passa): per wave of pass A, the steps of its segment pool and the lanes
holding a segment at each step, weighted by the step's duration.  Separates idle lanes (no
segment to trace: the pool is empty) from the divergence inside a step's walks, which the PMC
lane count (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU) mixes.

  TRT_LIB=variants/libtrt_passa.so python tools/pass_a_steps.py [--config ref|readme] [--inflight 16]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ref")
    ap.add_argument("--inflight", type=int, default=16)
    ap.add_argument("--frames", type=int, default=32)
    a = ap.parse_args()
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S
    from vkcomputeshader_tinyraytracer_amd._lib import lib

    L = lib()
    L.trt_diag_counter.restype = ctypes.c_ulonglong
    L.trt_diag_counter.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    sc = S.config_reference_default() if a.config == "ref" else S.config_readme()
    p = sc.params()
    with trt.Renderer(0) as r:
        r.upload_scene(sc)
        out = torch.zeros((a.frames, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        ubos = S.camera_path(sc.ubo, a.frames)
        r.set_frames_in_flight(a.inflight)
        r.render_frames(p, out, a.frames, ubos=ubos, frame_stride=p.height * p.width * 4)  # warm
        torch.cuda.synchronize()
        r.draw_frame(p, count=True)  # a counting frame zeroes the counters (it runs no pass A)
        r.render_frames(p, out, a.frames, ubos=ubos, frame_stride=p.height * p.width * 4)
        torch.cuda.synchronize()
        c = [L.trt_diag_counter(r._h, k) for k in range(24, 29)]
    dt, adt, steps, act, waves = c
    print(json.dumps({
        "config": a.config, "in_flight": a.inflight, "frames": a.frames, "waves": waves,
        "steps_per_wave": round(steps / max(waves, 1), 2),
        "lanes_with_segment_per_step": round(act / max(steps, 1), 2),
        "lanes_with_segment_time_weighted": round(adt / max(dt, 1), 2),
        "wave_time_us_per_frame": round(dt * 0.01 / a.frames, 1),
        "note": "lanes out of 64 holding a segment at a pass-A step (the rest idle: pool empty); "
                "time-weighted by the step's duration",
    }))


if __name__ == "__main__":
    main()
