"""Hot-first dealing of single-frame launches (trt_kernel.hip trace_hot): a slot's frame deals the
tiles its previous frame found costliest first.  The lists only order the dispatch — every tile
is traced exactly once — so frames rendered with it equal frames rendered without it bit for
bit, while the camera moves, across image sizes (the lists are reset when the tiling changes)
and on several in-flight slots.  Run with `pytest -m gpu`."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd import scene as S

pytestmark = pytest.mark.gpu

SMALL_ENV = (1024, 512)


def _renderer(hot: int):
    import vkcomputeshader_tinyraytracer_amd as trt

    old = os.environ.get("TRT_HOT_FIRST")
    os.environ["TRT_HOT_FIRST"] = str(hot)
    try:
        return trt.Renderer(0)
    finally:
        if old is None:
            os.environ.pop("TRT_HOT_FIRST", None)
        else:
            os.environ["TRT_HOT_FIRST"] = old


def _hot_state(r, slot=0):
    from vkcomputeshader_tinyraytracer_amd._lib import lib

    f = lib().trt_diag_hot
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    out = (ctypes.c_uint32 * 8)()
    assert f(r._h, slot, out) == 0
    return list(out)


def _ubos(n):
    return [S.make_ubo(cam=(0.05 * i, 0.01 * (i % 3), -0.08 * i)) for i in range(n)]


@pytest.mark.parametrize("config,size", [("C2", (256, 192)), ("C2", (264, 200)), ("C3", (256, 144)), ("C1", (128, 64))])
def test_hot_first_frames_equal_plain_dealing(config, size):
    on, off = _renderer(1), _renderer(0)
    try:
        sc = S.CONFIGS[config](*size) if config == "C1" else S.CONFIGS[config](*size, env_size=SMALL_ENV)
        p = sc.params()
        on.upload_scene(sc)
        off.upload_scene(sc)
        for i, u in enumerate(_ubos(8)):
            on.update_ubo(u)
            off.update_ubo(u)
            a, _, _ = on.draw_frame(p)
            b, _, _ = off.draw_frame(p)
            assert np.array_equal(a, b), (config, size, i)
        st = _hot_state(on)
        assert st[7] > 0, st  # the slot ran hot-first frames
        assert max(st[0], st[2], st[4]) > 0, st  # and listed tiles
        assert _hot_state(off)[7] == 0
    finally:
        on.close()
        off.close()


def test_hot_first_survives_tiling_changes():
    """Alternating image sizes on one slot: the lists index the other tiling and are reset."""
    on, off = _renderer(1), _renderer(0)
    try:
        sc = S.CONFIGS["C2"](256, 192, env_size=SMALL_ENV)
        on.upload_scene(sc)
        off.upload_scene(sc)
        sizes = [(256, 192), (256, 192), (256, 192), (200, 136), (200, 136), (256, 192), (512, 64), (256, 192)]
        for i, (w, h) in enumerate(sizes):
            p = sc.params()
            p.width, p.height = w, h
            a, _, _ = on.draw_frame(p)
            b, _, _ = off.draw_frame(p)
            assert np.array_equal(a, b), (i, w, h)
    finally:
        on.close()
        off.close()


@pytest.mark.parametrize("inflight", [1, 2, 3])
def test_hot_first_one_launch_per_frame_in_flight(inflight):
    """drawFrame pacing: one launch per frame on `inflight` slots (each slot keeps its own
    lists); every frame equals trt_render without hot-first dealing."""
    torch = pytest.importorskip("torch")
    on, off = _renderer(1), _renderer(0)
    try:
        sc = S.CONFIGS["C2"](256, 192, env_size=SMALL_ENV)
        p = sc.params()
        on.upload_scene(sc)
        off.upload_scene(sc)
        n = 12
        ubos = np.stack(_ubos(n))
        out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        stream = torch.cuda.Stream()
        on.set_stream(stream)
        on.set_frame_batch(1)
        on.set_frames_in_flight(inflight)
        for _ in range(2):  # twice: the second pass deals from lists of the first
            on.render_frames(p, out, n, ubos=ubos, frame_stride=p.height * p.width * 4)
        stream.synchronize()
        on.set_stream(None)
        got = out.cpu().numpy()
        for i in range(n):
            off.update_ubo(ubos[i])
            one, _, _ = off.draw_frame(p)
            assert np.array_equal(got[i], one), i
        assert _hot_state(on, 0)[7] > 0
    finally:
        on.close()
        off.close()
