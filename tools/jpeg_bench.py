#!/usr/bin/env python3
"""Envmap JPEG path timing: host entropy decode vs GPU reconstruction of a
reference-sized (7616x3808) progressive 4:2:0 JPEG made with Pillow, plus Pillow's own
decode of the same bytes as a CPU yardstick.

  python tools/jpeg_bench.py [--reps 3]
"""
from __future__ import annotations

import argparse
import io
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    from PIL import Image

    import vkcomputeshader_tinyraytracer_amd as trt
    from tests.test_jpeg import _big_progressive_jpeg
    from vkcomputeshader_tinyraytracer_amd.jpeg import JpegFile

    data = _big_progressive_jpeg()
    r = trt.Renderer(0)
    out = torch.empty((3808, 7616, 4), dtype=torch.uint8, device="cuda")
    parse, recon, pil = [], [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        jf = JpegFile(data)
        t1 = time.perf_counter()
        r.decode_jpeg(jf, out=out)  # synchronous (uploads coefficients, kernels, waits)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        Image.open(io.BytesIO(data)).convert("RGBA").tobytes()
        t3 = time.perf_counter()
        parse.append(t1 - t0)
        recon.append(t2 - t1)
        pil.append(t3 - t2)
        jf.close()
    print(json.dumps({"bytes": len(data), "pixels": 7616 * 3808,
                      "host_entropy_ms": round(1e3 * float(np.median(parse)), 1),
                      "gpu_reconstruct_ms_incl_h2d": round(1e3 * float(np.median(recon)), 1),
                      "pillow_decode_ms": round(1e3 * float(np.median(pil)), 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
