#!/usr/bin/env python3
"""Per-pixel traversal work of one frame (diagnostic build TRT_LIB=variants/libtrt_work.so,
tools/build_variants.sh work): node visits, triangle tests, segments and the largest single
query per pixel; prints the distribution, the 8x8-tile maxima and the worst pixels.

  TRT_LIB=variants/libtrt_work.so python tools/pixel_work.py --config ref [--out f.npz]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ref")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = S.config_reference_default() if a.config == "ref" else S.CONFIGS[a.config]()
    p = sc.params()
    r = trt.Renderer(0)
    r.set_subtree_split(1)
    r.upload_scene(sc)
    out8 = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    w = torch.zeros((p.height, p.width, 4), dtype=torch.float32, device="cuda")
    r.draw_frame(p, out8=out8, out32=w)
    torch.cuda.synchronize()
    w = w.cpu().numpy()
    nodes, tris, segs, qmax = (w[..., k] for k in range(4))
    H, W = nodes.shape
    tiles = nodes[: H // 8 * 8, : W // 8 * 8].reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
    def tile_eff(a):
        """work / (64 x the tile's busiest lane): how much of an 8x8 one-wave tile's lane time the
        work fills if every lane walks as long as the tile's longest"""
        t = a[: H // 8 * 8, : W // 8 * 8].reshape(H // 8, 8, W // 8, 8)
        return float(t.sum() / max(64.0 * t.max(axis=(1, 3)).sum(), 1.0))
    order = np.argsort(nodes.ravel())[::-1][:10]
    res = {
        "config": a.config,
        "nodes_total": float(nodes.sum()), "tris_total": float(tris.sum()), "segments_total": float(segs.sum()),
        "nodes_per_pixel": float(nodes.mean()), "tris_per_pixel": float(tris.mean()),
        "tile_eff_nodes": tile_eff(nodes), "tile_eff_tris": tile_eff(tris), "tile_eff_work": tile_eff(nodes + tris),
        "nodes_pct": {q: float(np.percentile(nodes, q)) for q in (50, 90, 99, 99.9, 100)},
        "segs_pct": {q: float(np.percentile(segs, q)) for q in (50, 90, 99, 99.9, 100)},
        "qmax_pct": {q: float(np.percentile(qmax, q)) for q in (50, 90, 99, 99.9, 100)},
        "tile_max_nodes_pct": {q: float(np.percentile(tiles, q)) for q in (50, 90, 99, 100)},
        "worst": [{"y": int(i // W), "x": int(i % W), "nodes": float(nodes.flat[i]), "tris": float(tris.flat[i]),
                   "segs": float(segs.flat[i]), "qmax": float(qmax.flat[i])} for i in order],
    }
    print(json.dumps(res), flush=True)
    if a.out:
        np.savez_compressed(a.out, work=w)
    r.close()


if __name__ == "__main__":
    main()
