#!/usr/bin/env python3
"""Per-configuration work counters of one frame (COUNT pass), normalised per query: BVH / batch
node tests, triangle tests and batch-gate tests per closest-hit or shadow query.

  python tools/scene_stats.py [--configs ref C3 C4] [--walk]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["ref", "C3", "C4"])
    ap.add_argument("--walk", action="store_true", help="also the reference-order batch walk")
    a = ap.parse_args()
    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

    r = trt.Renderer(0)
    for cfg in a.configs:
        sc = S.config_reference_default() if cfg == "ref" else S.CONFIGS[cfg]()
        r.upload_scene(sc)
        for walk in ([False, True] if a.walk else [False]):
            p = sc.params()
            if walk:
                p.flags |= T.FLAG_BATCH_WALK
            _, _, st = r.draw_frame(p, count=True, timing=True, want8=False)
            q = st["primary_rays"] + st["secondary_rays"] + st["shadow_rays"]
            out = {"config": cfg, "walk": walk, "queries": q, "ms": round(st["kernel_ms"], 3),
                   **{k: st[k] for k in T.Stats.COUNTERS},
                   "node_tests_per_query": round(st["node_tests"] / q, 2),
                   "tri_tests_per_query": round(st["tri_tests"] / q, 2),
                   "batch_tests_per_query": round(st["batch_tests"] / q, 2)}
            print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
