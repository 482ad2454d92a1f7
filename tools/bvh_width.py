#!/usr/bin/env python3
"""SAH estimate of a wider BVH for the product's BVH2 (trt_diag_bvh_export): the BVH2 collapsed
greedily to 2 / 4 / 8 children per node (opening the largest-area inner child while there is room,
as collapse_bvh4 does), and for each width the expected inner-node visits and triangle tests of a
random ray through the root box (sum of child areas / root area), the node count and the depth.

  python tools/bvh_width.py            (the shipped scene, the README scene, C4, C3)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from tests.test_bvh_layout import _export  # noqa: E402
from vkcomputeshader_tinyraytracer_amd import scene as S  # noqa: E402
from vkcomputeshader_tinyraytracer_amd.scene import load_golden_meshes  # noqa: E402

LEAF = 0x80000000


def area(lo, hi):
    d = np.maximum(hi - lo, 0)
    return 2 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0])


def main():
    gm = load_golden_meshes()
    for name in ["ref", "readme", "C4", "C3"]:
        if name == "ref":
            sc = S.config_reference_default(gm, env_size=(64, 32))
        elif name == "readme":
            sc = S.config_readme(gm, env_size=(64, 32))
        else:
            sc = S.CONFIGS[name](64, 48, env_size=(64, 32))
        nodes, _ = _export(sc)
        boxes = nodes[:, :12].view(np.float32).reshape(-1, 4, 3).astype(np.float64)
        child = nodes[:, 12:14]

        def kids(n):
            return [(int(child[n, k]), boxes[n, 2 * k], boxes[n, 2 * k + 1]) for k in range(2)
                    if int(child[n, k]) != 0xFFFFFFFF]

        ra = area(np.minimum(boxes[0, 0], boxes[0, 2]), np.maximum(boxes[0, 1], boxes[0, 3]))
        for W in (2, 4, 8):
            visits, tris, nnodes, depth = 1.0, 0.0, 0, 0
            todo = [(0, 1)]
            while todo:
                n, dep = todo.pop()
                nnodes += 1
                depth = max(depth, dep)
                s = kids(n)
                while len(s) < W:
                    inner = [i for i, (c, lo, hi) in enumerate(s) if not (c & LEAF)]
                    if not inner:
                        break
                    b = max(inner, key=lambda i: area(s[i][1], s[i][2]))
                    s.extend(kids(s.pop(b)[0]))
                for c, lo, hi in s:
                    a = area(lo, hi) / ra
                    if c & LEAF:
                        tris += a * (((c >> 27) & 15) + 1)
                    else:
                        visits += a
                        todo.append((c, dep + 1))
            print(f"{name:7s} width {W}: nodes {nnodes:6d}  visits {visits:6.2f}  triangle tests {tris:6.2f}  depth {depth}")


if __name__ == "__main__":
    main()
