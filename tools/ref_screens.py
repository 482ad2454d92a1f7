"""Register oracle renders against the reference's own Vulkan screenshots (build container only).

The reference ships lossless PNG screenshots of its compute shader's output (new_feature.md,
README.md).  This script renders the matching scene with the CPU oracle as displayed (sRGB
swapchain), checks the registration offset against its neighbours, classifies every pixel off
by more than 1 LSB (chaotic under a few-ulp primary-ray change / edge / shadow acne of the
older shader) and writes the record to --json.  It reads the screenshots and background.jpg in
place; nothing is copied into the repo.

    python tools/ref_screens.py [--search R] [--json profiles/r04_reference_screens.json] [name ...]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402

from tests import ref_screens as R  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", type=int, default=2)
    ap.add_argument("--json", default="")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    recs = []
    for shot in R.SHOTS:
        if a.names and shot.name not in a.names:
            continue
        t0 = time.time()
        frame = R.oracle_frame(shot)
        t1 = time.time()
        scr = R.load_screen(shot)
        best = None
        for dy in range(-a.search, a.search + 1):
            for dx in range(-a.search, a.search + 1):
                off = (shot.offset[0] + dy, shot.offset[1] + dx)
                rep = R.register(frame, scr, off, shot)
                if rep is not None and (best is None or rep["within1"] > best["within1"]):
                    best = dict(rep, offset=off)
        at = R.register(frame, scr, shot.offset, shot)
        d, m = R.pixel_diff(frame, scr, shot.offset, shot)
        cls = {"chaotic": 0, "edge": 0, "acne": 0, "unexplained": []}
        for yy, xx in zip(*np.nonzero((d > 1) & m)):
            fy, fx = shot.offset[0] + int(yy), shot.offset[1] + int(xx)
            if shot.direct_only and R.edge_match(frame, fy, fx, scr[yy, xx]):
                cls["edge"] += 1
            elif shot.direct_only and R.sphere_acne(shot, fy, fx, scr[yy, xx]):
                cls["acne"] += 1
            elif R.instability(shot, fy, fx, scr[yy, xx], radius3=6 if not shot.direct_only else 2)["unstable"]:
                cls["chaotic"] += 1
            else:
                cls["unexplained"].append([fy, fx, int(d[yy, xx])])
        rec = {"shot": shot.name, "png": shot.png, "source": shot.source, "models": list(shot.models),
               "offset": list(shot.offset), "screen_crop": list(shot.screen_crop), "max_depth": shot.max_depth,
               "mask": {"rows_below": shot.rows_below, "direct_only": shot.direct_only},
               "at_offset": at, "best_in_search": best, "outliers_gt1": cls, "oracle_render_s": round(t1 - t0, 1)}
        recs.append(rec)
        print(json.dumps(rec))
    if a.json:
        Path(a.json).write_text(json.dumps(recs, indent=1) + "\n")


if __name__ == "__main__":
    main()
