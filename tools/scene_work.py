#!/usr/bin/env python3
"""Counting pass of one configuration: prints the trt_stats work counters (rays, box and
triangle tests, Moller-Trumbore stages) per frame and per ray.

  python tools/scene_work.py --config C4
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    a = ap.parse_args()
    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = (S.config_reference_default() if a.config == "ref" else
          S.config_readme() if a.config == "readme" else S.CONFIGS[a.config]())
    r = trt.Renderer(0)
    r.upload_scene(sc)
    _, _, st = r.draw_frame(sc.params(), count=True)
    q = st["primary_rays"] + st["secondary_rays"] + st["shadow_rays"] - st["shadow_skipped"]
    st = {k: v for k, v in st.items() if k != "kernel_ms"}
    st["queries_traced"] = q
    st["box_tests_per_query"] = round((st["node_tests"] + st["batch_tests"] - st["skipped_box_tests"]) / q, 2)
    st["tri_tests_per_query"] = round((st["tri_tests"] - st["skipped_tri_tests"]) / q, 2)
    print(json.dumps({"config": a.config, **st}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
