#!/usr/bin/env python3
"""GPU JPEG decode vs the oracle for every committed fixture: per-file mismatch summary."""
import glob
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np

import vkcomputeshader_tinyraytracer_amd as trt
from oracle import jpeg_ref
from vkcomputeshader_tinyraytracer_amd.jpeg import JpegFile

r = trt.Renderer(0)
for f in sorted(glob.glob(str(Path(__file__).resolve().parents[1] / "tests/golden/jpeg/*.jpg"))):
    jf = JpegFile(f)
    g = r.decode_jpeg(jf)
    o = jpeg_ref.reconstruct(jf)
    d = np.abs(g.astype(int) - o.astype(int))
    bad = np.argwhere(d.max(-1) > 0)
    print(Path(f).name, "ok" if not len(bad) else
          f"{len(bad)}/{d.shape[0]*d.shape[1]} px differ, max {d.max()}, first {bad[:4].tolist()}, rows {np.unique(bad[:,0])[:12].tolist()}")
