"""Byte layouts of the reference's scene records (include/trt/scene_types.h) as numpy
dtypes, plus the ctypes views of the C-ABI parameter structs (include/trt/abi.h).

Reference records: Material/Sphere/Triangle/Model (geometry.hpp:5-46, shader.comp:3-38),
UniformBufferObject and Ray (main.cpp:145-187, shader.comp:14-17, 40-51).
"""
from __future__ import annotations

import ctypes

import numpy as np

F4 = ("<f4", (4,))

MATERIAL = np.dtype([("albedo", *F4), ("diffuse_specular", *F4), ("refractive", *F4)])
SPHERE = np.dtype([("center_radius", *F4), ("material", MATERIAL)])
TRIANGLE = np.dtype(
    [
        ("v0", *F4),
        ("v1", *F4),
        ("v2", *F4),
        ("material", MATERIAL),
        ("v0_norm", *F4),
        ("v1_norm", *F4),
        ("v2_norm", *F4),
    ]
)
MODEL = np.dtype(
    [("params0", "<i4", (4,)), ("bboxMin", *F4), ("bboxMax", *F4), ("material", MATERIAL)]
)
UBO = np.dtype(
    [
        ("sphere0", SPHERE),
        ("sphere1", SPHERE),
        ("sphere2", SPHERE),
        ("sphere3", SPHERE),
        ("light0", *F4),
        ("light1", *F4),
        ("light2", *F4),
        ("camPos", *F4),
        ("bboxMin", *F4),
        ("bboxMax", *F4),
    ]
)
RAY = np.dtype([("dir", *F4), ("resultColor", *F4)])

assert MATERIAL.itemsize == 48 and SPHERE.itemsize == 64
assert TRIANGLE.itemsize == 144 and MODEL.itemsize == 96
assert UBO.itemsize == 352 and RAY.itemsize == 32

# trt_params.flags (abi.h)
FLAG_SPHERES = 1 << 0
FLAG_FLOOR = 1 << 1
FLAG_CHECKER = 1 << 2
FLAG_ENVMAP = 1 << 3
FLAG_ROW_QUIRK = 1 << 4
FLAG_DEVICE_PTRS = 1 << 5
FLAG_COUNT = 1 << 6
FLAG_TIMING = 1 << 7
FLAG_BATCH_WALK = 1 << 8
FLAG_SRGB_OUT = 1 << 9
FLAG_BAND_IN_PLACE = 1 << 10  # band rows written at their frame rows (device outputs)
FLAGS_REFERENCE = FLAG_FLOOR | FLAG_ENVMAP | FLAG_ROW_QUIRK

MAX_DEPTH_LIMIT = 20

# status codes
TRT_OK = 0
TRT_ERR_INVALID = -1
TRT_ERR_HIP = -2
TRT_ERR_NOSCENE = -3
TRT_ERR_OOM = -4
TRT_ERR_IO = -5


class Params(ctypes.Structure):
    """trt_params (abi.h)."""

    _fields_ = [
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("max_depth", ctypes.c_uint32),
        ("spp", ctypes.c_uint32),
        ("seed", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("fov", ctypes.c_float),
        ("band_rows", ctypes.c_uint32),
        ("band_count", ctypes.c_uint32),
        ("band_index", ctypes.c_uint32),
        ("rays_in", ctypes.c_void_p),
    ]


class Stats(ctypes.Structure):
    """trt_stats (abi.h)."""

    _fields_ = [
        ("primary_rays", ctypes.c_uint64),
        ("secondary_rays", ctypes.c_uint64),
        ("shadow_rays", ctypes.c_uint64),
        ("misses", ctypes.c_uint64),
        ("tri_nearest", ctypes.c_uint64),
        ("sphere_tests", ctypes.c_uint64),
        ("batch_tests", ctypes.c_uint64),
        ("batch_hits", ctypes.c_uint64),
        ("tri_tests", ctypes.c_uint64),
        ("node_tests", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double),
        ("tri_past_a", ctypes.c_uint64),
        ("tri_past_u", ctypes.c_uint64),
        ("tri_past_v", ctypes.c_uint64),
        ("shadow_skipped", ctypes.c_uint64),
        ("skipped_sphere_tests", ctypes.c_uint64),
        ("skipped_box_tests", ctypes.c_uint64),
        ("skipped_tri_tests", ctypes.c_uint64),
        ("skipped_tri_past_a", ctypes.c_uint64),
        ("skipped_tri_past_u", ctypes.c_uint64),
        ("skipped_tri_past_v", ctypes.c_uint64),
    ]

    COUNTERS = ("primary_rays", "secondary_rays", "shadow_rays", "misses", "tri_nearest",
                "sphere_tests", "batch_tests", "batch_hits", "tri_tests", "node_tests",
                "tri_past_a", "tri_past_u", "tri_past_v", "shadow_skipped", "skipped_sphere_tests",
                "skipped_box_tests", "skipped_tri_tests", "skipped_tri_past_a", "skipped_tri_past_u",
                "skipped_tri_past_v")
    # counters that must equal the oracle's (the reference's work); batch_tests / node_tests
    # depend on the traversal (the kernel culls with a conservative hierarchy)
    EXACT = ("primary_rays", "secondary_rays", "shadow_rays", "misses", "tri_nearest",
             "sphere_tests")
    # with TRT_FLAG_BATCH_WALK the kernel also tests exactly the reference's batches/triangles
    EXACT_WALK = EXACT + ("batch_hits", "tri_tests")

    def as_dict(self) -> dict:
        d = {k: int(getattr(self, k)) for k in self.COUNTERS}
        d["kernel_ms"] = float(self.kernel_ms)
        return d


class BandLayout(ctypes.Structure):
    """trt_band_layout (abi.h): buffer shapes of a tiled batch."""

    _fields_ = [
        ("groups", ctypes.c_uint32),
        ("max_rows", ctypes.c_uint32),
        ("block_bytes", ctypes.c_uint64),
        ("local_bytes", ctypes.c_uint64),
        ("gather_bytes", ctypes.c_uint64),
    ]


class BandXfer(ctypes.Structure):
    """trt_band_xfer (abi.h): the compact band blocks one rank sends to one root."""

    _fields_ = [
        ("src", ctypes.c_uint32),
        ("dst", ctypes.c_uint32),
        ("frames", ctypes.c_uint32),
        ("groups", ctypes.c_uint32),
        ("first_slot", ctypes.c_uint32),
        ("pad", ctypes.c_uint32),
        ("src_offset", ctypes.c_uint64),
        ("dst_offset", ctypes.c_uint64),
        ("bytes", ctypes.c_uint64),
    ]


PLAN_SELF_GATHER = 1  # TRT_PLAN_SELF_GATHER
ROOT_ROTATE = -1  # TRT_ROOT_ROTATE

assert ctypes.sizeof(Params) == 48 and ctypes.sizeof(Stats) == 168
assert ctypes.sizeof(BandLayout) == 32 and ctypes.sizeof(BandXfer) == 48


def make_params(
    width: int = 1024,
    height: int = 768,
    max_depth: int = 20,
    spp: int = 1,
    seed: int = 0,
    flags: int = FLAGS_REFERENCE,
    fov: float = 1.05,
    band_rows: int = 0,
    band_count: int = 0,
    band_index: int = 0,
    rays_in: int | None = None,
) -> Params:
    """Defaults are the reference's (main.cpp:35-36, 1498; shader.comp:75)."""
    p = Params()
    p.width, p.height, p.max_depth, p.spp, p.seed = width, height, max_depth, spp, seed
    p.flags, p.fov = flags, fov
    p.band_rows, p.band_count, p.band_index = band_rows, band_count, band_index
    p.rays_in = rays_in
    return p


def output_rows(height: int, band_rows: int = 0, band_count: int = 0, band_index: int = 0) -> list[int]:
    """Image rows a banded render writes, in output order (trt_output_rows)."""
    if band_rows == 0 or band_count <= 1:
        return list(range(height))
    return [r for r in range(height) if (r // band_rows) % band_count == band_index]


def ptr(a: np.ndarray | None) -> ctypes.c_void_p | None:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays handed to the C-ABI must be C-contiguous"
    return ctypes.c_void_p(a.ctypes.data)
