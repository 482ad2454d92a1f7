"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/liboracle.so).

The oracle is a plain-C restatement of the reference hot path (shader.comp; see
oracle/trt_oracle.c for the line-by-line citations and the parity status: pinned to the
reference's own Vulkan screenshots (tests/test_reference_screens.py), to known-answer
vectors, by the literal-vs-fast mode equivalence, and by reference-built input goldens).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

from vkcomputeshader_tinyraytracer_amd import types as T

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"

MODE_FAST = 0
MODE_LITERAL = 1


def mode_split(window: int) -> int:
    """Fast mode + the kernel's subtree split (trt_set_subtree_split) with this window."""
    return 16 + int(window)


class OrcScene(ctypes.Structure):
    _fields_ = [
        ("ubo", ctypes.c_void_p),
        ("tris", ctypes.c_void_p),
        ("ntri", ctypes.c_uint32),
        ("models", ctypes.c_void_p),
        ("nmodel", ctypes.c_uint32),
        ("env", ctypes.c_void_p),
        ("env_w", ctypes.c_uint32),
        ("env_h", ctypes.c_uint32),
    ]


_L = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", os.fspath(HERE), "liboracle.so"], check=True)
    return LIB


def lib():
    global _L
    if _L is None:
        if not LIB.exists():
            build()
        L = ctypes.CDLL(os.fspath(LIB))
        vp, fp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)
        L.orc_render.restype = ctypes.c_int
        L.orc_render.argtypes = [ctypes.POINTER(OrcScene), ctypes.POINTER(T.Params), ctypes.c_int,
                                 ctypes.c_int, vp, vp, ctypes.POINTER(T.Stats)]
        L.orc_ray_aabb.restype = ctypes.c_int
        L.orc_ray_aabb.argtypes = [fp, fp, fp, fp]
        L.orc_ray_triangle.restype = ctypes.c_int
        L.orc_ray_triangle.argtypes = [fp, fp, fp, fp, fp, fp, fp, fp, ctypes.c_int, fp, fp]
        L.orc_ray_sphere.restype = ctypes.c_int
        L.orc_ray_sphere.argtypes = [fp, fp, fp, fp]
        L.orc_custom_refract.restype = None
        L.orc_custom_refract.argtypes = [fp, fp, ctypes.c_float, ctypes.c_float, fp]
        L.orc_direction_to_uv.restype = None
        L.orc_direction_to_uv.argtypes = [fp, fp]
        L.orc_sample_env.restype = None
        L.orc_sample_env.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, fp, fp]
        L.orc_primary_dir.restype = None
        L.orc_primary_dir.argtypes = [ctypes.POINTER(T.Params), ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, fp]
        L.orc_cast_ray.restype = None
        L.orc_cast_ray.argtypes = [ctypes.POINTER(OrcScene), ctypes.POINTER(T.Params), ctypes.c_int,
                                   fp, fp, fp, ctypes.POINTER(T.Stats)]
        _L = L
    return _L


def _f(v, n=3):
    a = (ctypes.c_float * n)(*[float(np.float32(x)) for x in v])
    return a


class _Bound:
    """Keeps the numpy arrays alive while the C struct points at them."""

    def __init__(self, scene):
        self.ubo = np.ascontiguousarray(scene.ubo)
        self.tris = np.ascontiguousarray(scene.tris, T.TRIANGLE)
        self.models = np.ascontiguousarray(scene.models, T.MODEL)
        self.env = None if scene.env is None else np.ascontiguousarray(scene.env, np.uint8)
        self.s = OrcScene(
            self.ubo.ctypes.data,
            self.tris.ctypes.data if len(self.tris) else None, len(self.tris),
            self.models.ctypes.data if len(self.models) else None, len(self.models),
            self.env.ctypes.data if self.env is not None else None,
            0 if self.env is None else self.env.shape[1], 0 if self.env is None else self.env.shape[0])


def render(scene, params: T.Params | None = None, mode: int = MODE_FAST, threads: int = 0,
           want32: bool = False):
    """Returns (rgba8 (rows, W, 4), rgba32f or None, stats dict)."""
    p = T.Params.from_buffer_copy(params if params is not None else scene.params())
    rows = len(T.output_rows(p.height, p.band_rows, p.band_count, p.band_index))
    b = _Bound(scene)
    out8 = np.empty((rows, p.width, 4), np.uint8)
    out32 = np.empty((rows, p.width, 4), np.float32) if want32 else None
    rays_keep = None
    st = T.Stats()
    rc = lib().orc_render(ctypes.byref(b.s), ctypes.byref(p), mode, threads, out8.ctypes.data,
                          out32.ctypes.data if out32 is not None else None, ctypes.byref(st))
    del rays_keep
    if rc != 0:
        raise RuntimeError(f"orc_render failed: {rc}")
    return out8, out32, st.as_dict()


def ray_aabb(o, d, bmin, bmax) -> bool:
    return bool(lib().orc_ray_aabb(_f(o), _f(d), _f(bmin), _f(bmax)))


def ray_triangle(o, d, v0, v1, v2, n0=(0, 0, 0), n1=(0, 0, 0), n2=(0, 0, 0), normal_interp=0):
    t = ctypes.c_float(0)
    n = (ctypes.c_float * 3)()
    h = lib().orc_ray_triangle(_f(o), _f(d), _f(v0), _f(v1), _f(v2), _f(n0), _f(n1), _f(n2),
                               normal_interp, ctypes.byref(t), n)
    return (bool(h), t.value, tuple(n)) if h else (False, None, None)


def ray_sphere(o, d, center_radius):
    t = ctypes.c_float(0)
    h = lib().orc_ray_sphere(_f(o), _f(d), _f(center_radius, 4), ctypes.byref(t))
    return (bool(h), t.value if h else None)


def custom_refract(I, N, eta_out, eta_in=1.0):
    out = (ctypes.c_float * 3)()
    lib().orc_custom_refract(_f(I), _f(N), eta_out, eta_in, out)
    return tuple(out)


def direction_to_uv(d):
    uv = (ctypes.c_float * 2)()
    lib().orc_direction_to_uv(_f(d), uv)
    return tuple(uv)


def sample_env(env: np.ndarray, uv):
    env = np.ascontiguousarray(env, np.uint8)
    out = (ctypes.c_float * 3)()
    lib().orc_sample_env(env.ctypes.data, env.shape[1], env.shape[0], _f(uv, 2), out)
    return tuple(out)


def primary_dir(params: T.Params, x: int, y: int, sample: int = 0):
    out = (ctypes.c_float * 3)()
    lib().orc_primary_dir(ctypes.byref(params), x, y, sample, out)
    return tuple(out)


def cast_ray(scene, params: T.Params, o, d, mode: int = MODE_FAST):
    b = _Bound(scene)
    out = (ctypes.c_float * 3)()
    st = T.Stats()
    lib().orc_cast_ray(ctypes.byref(b.s), ctypes.byref(params), mode, _f(o), _f(d), out, ctypes.byref(st))
    return tuple(out), st.as_dict()
