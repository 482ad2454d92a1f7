"""Regenerates tests/golden/renders.npz + renders.json: small RGBA8 renders of the parity
configurations by the CPU oracle, so a GPU box compares the kernel against
committed images as well as against the oracle re-run there, and the CPU suite pins the
oracle build itself (same image on every host with this toolchain).

  renders.npz   "<name>" -> uint8 (H, W, 4) RGBA8 = floor(255 * pow(clamp(c), 2.2) + 0.5)
  renders.json  per render: scene, size, depth, flags, exact ray counters, SHA-256 of the image

Every scene is deterministic: reference spheres/lights/materials (main.cpp:125-143), the
seeded procedural envmap (scene.synthetic_envmap), icosphere / committed-asset meshes.
Usage: python tests/golden/make_renders.py
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

from oracle import oracle as orc  # noqa: E402  (test infrastructure: the checker)
from vkcomputeshader_tinyraytracer_amd import scene as S, types as T  # noqa: E402

W, H = 128, 96
ENV = (1024, 512)


def cases() -> dict:
    """name -> (scene, params); shared with the tests that read the fixture."""
    out = {}
    c1 = S.config_c1(W, H)
    out["C1"] = (c1, c1.params())
    c2 = S.config_c2(W, H, env_size=ENV)
    out["C2"] = (c2, c2.params())
    c2d = S.config_c2(W, H, env_size=ENV)
    c2d.max_depth = 20
    out["C2_depth20"] = (c2d, c2d.params())
    c3 = S.config_c3(W, H, env_size=ENV)
    out["C3"] = (c3, c3.params())
    ref = S.config_reference_default(env_size=ENV, width=W, height=H)
    out["reference_default"] = (ref, ref.params())
    c5 = S.config_c4(W, H, env_size=ENV, spp=4)
    out["C4_spp4"] = (c5, c5.params())
    # C5 (BASELINE configs[4]): the C4 scene at 16 PCG-jittered samples per pixel
    c5_16 = S.config_c5(64, 48, env_size=ENV)
    out["C5_spp16"] = (c5_16, c5_16.params())
    return out


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main() -> None:
    imgs, meta = {}, {}
    for name, (sc, p) in cases().items():
        o8, _, st = orc.render(sc, p, want32=False)
        imgs[name] = o8
        meta[name] = {"scene": sc.name, "size": [p.width, p.height], "max_depth": p.max_depth,
                      "spp": p.spp, "flags": p.flags, "triangles": int(len(sc.tris)),
                      "counts": {k: int(st[k]) for k in T.Stats.EXACT_WALK}, "sha256": sha(o8)}
        print(name, meta[name]["counts"], flush=True)
    np.savez_compressed(REPO / "tests" / "golden" / "renders.npz", **imgs)
    (REPO / "tests" / "golden" / "renders.json").write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
