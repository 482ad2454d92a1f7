"""Writes tests/golden/dropin_meshes.bin: the shipped scene's meshes (glass, whisky, ice;
config.hpp:97-101) as parsed by the reference's own tinyobjloader (tests/golden/meshes.npz), in
the flat little-endian layout the C++ drop-in host reads (tests/native/drop_in_host.cpp):
"TRTMESH1", u32 count, then per mesh u32 name length, name, u32 nverts, u32 ntris,
float32 positions[3 nverts], u32 indices[3 ntris].

    python tests/golden/make_dropin_dump.py
"""
from __future__ import annotations

import struct
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
NAMES = ("glass.obj", "water.obj", "ice.obj")


def main() -> None:
    with np.load(HERE / "meshes.npz", allow_pickle=False) as z:
        parts = [b"TRTMESH1", struct.pack("<I", len(NAMES))]
        for n in NAMES:
            pos = np.ascontiguousarray(z[f"{n}:pos"], "<f4")
            idx = np.ascontiguousarray(z[f"{n}:idx"], "<u4")
            parts += [struct.pack("<I", len(n)), n.encode(), struct.pack("<II", len(pos), len(idx)),
                      pos.tobytes(), idx.tobytes()]
    (HERE / "dropin_meshes.bin").write_bytes(b"".join(parts))


if __name__ == "__main__":
    main()
