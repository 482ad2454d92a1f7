"""The BVH pipeline of trt_upload_scene on the host (no GPU): the 4-wide collapse, the
quantized nodes and their 48-byte form with implicit children (trt_device.h Bvh4CNode) build
for every mesh configuration, and the compression's self-check passes — the kernel's own decode
of every node (bvh4c_children, shared host/device) yields the remapped child references slot by
slot and every leaf keeps its triangles.  The GPU parity tests then run the walk over them."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd import lib, scene as S, types as T


def _build(sc):
    L = lib()
    L.trt_diag_bvh_build.restype = ctypes.c_int
    L.trt_diag_bvh_build.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_uint64)]
    tris = np.ascontiguousarray(sc.tris, T.TRIANGLE)
    models = np.ascontiguousarray(sc.models, T.MODEL)
    out = (ctypes.c_uint64 * 6)()
    rc = L.trt_diag_bvh_build(tris.ctypes.data, len(tris), models.ctypes.data, len(models), out)
    assert rc == 0
    return dict(zip(("bvh2", "bvh4", "quantized", "compressed", "stack", "tris"), list(out)))


@pytest.mark.parametrize("name", ["C3", "C4", "ref", "readme"])
def test_bvh4_compressed_layout(name, golden_meshes):
    if name == "ref":
        sc = S.config_reference_default(golden_meshes, env_size=(64, 32))
    elif name == "readme":
        sc = S.config_readme(golden_meshes, env_size=(64, 32))
    else:
        sc = S.CONFIGS[name](64, 48, env_size=(64, 32))
    st = _build(sc)
    assert st["tris"] == len(sc.tris)
    assert 0 < st["bvh4"] < st["bvh2"] and st["stack"] <= 64
    assert st["quantized"] == 1 and st["compressed"] == 1, st
