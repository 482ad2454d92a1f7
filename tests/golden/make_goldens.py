"""Regenerates the committed golden fixtures in tests/golden/ (run in the build container,
where the read-only reference checkout exists; the GPU box only reads the outputs).

  meshes.npz         positions (float32, V x 3) and triangle vertex indices (uint32, F x 3)
                     of reference assets exactly as the reference's own vendored
                     tinyobjloader parses and triangulates them and as loadObjAsTriangles
                     keeps them (oracle/_ref/tinyobj_dump, built by `make -C oracle ref`).
  obj_goldens.json   per-asset vertex/triangle counts and SHA-256 of those arrays (all 11
                     assets), so the product's OBJ loader can be checked bit-for-bit.

Usage: python tests/golden/make_goldens.py
"""
from __future__ import annotations

import hashlib
import json
import subprocess
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
ASSETS = Path("/root/reference/VulkanComputeShaderApplication/assets")
DUMP = REPO / "oracle" / "_ref" / "tinyobj_dump"

# Meshes shipped in meshes.npz: the default scene (config.hpp:97-101), the C3-sized
# water_small, and the README-era scene (config.hpp:96) for the rotated-model path.
SHIP = ("glass.obj", "water.obj", "ice.obj", "water_small.obj", "asschercut-mesh.obj",
        "bunny-mesh.obj", "dragon-mesh.obj", "venus-mesh.obj", "fudanlogo-mesh.obj", "duck.obj")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main() -> None:
    subprocess.run(["make", "-s", "-C", str(REPO / "oracle"), "ref"], check=True)
    objs = sorted(ASSETS.glob("*.obj"))
    out: dict = {}
    meta: dict = {}
    with tempfile.TemporaryDirectory() as td:
        args = []
        for o in objs:
            args += [str(o), str(Path(td) / o.stem)]
        subprocess.run([str(DUMP), *args], check=True)
        for o in objs:
            pos = np.fromfile(Path(td) / f"{o.stem}.pos", np.float32).reshape(-1, 3)
            idx = np.fromfile(Path(td) / f"{o.stem}.idx", np.uint32).reshape(-1, 3)
            meta[o.name] = {"vertices": int(pos.shape[0]), "triangles": int(idx.shape[0]),
                            "pos_sha256": sha(pos), "idx_sha256": sha(idx),
                            "obj_sha256": hashlib.sha256(o.read_bytes()).hexdigest()}
            if o.name in SHIP:
                out[f"{o.name}:pos"] = pos
                out[f"{o.name}:idx"] = idx
    np.savez_compressed(REPO / "tests" / "golden" / "meshes.npz", **out)
    (REPO / "tests" / "golden" / "obj_goldens.json").write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")
    print(json.dumps({k: (v["vertices"], v["triangles"]) for k, v in meta.items()}))


if __name__ == "__main__":
    main()
