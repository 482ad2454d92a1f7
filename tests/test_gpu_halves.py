"""Two waves per tile for triangle-free single-frame launches (trace_halves, KArgs::tile_halves =
S): the helper wave follows each pixel's spine (the last-popped children) to depth S unshaded and
traces the subtree there, whose colour terms the owner wave adds after its own in the reference's
pop order (shader.comp:447-583).  For every split depth S = 1, 2, 3 the result must equal the
one-wave kernel BIT FOR BIT (RGBA8 and rayOut) and the counting pass (which keeps the one-wave
kernel) — on every depth the launch serves (2..4), the depths it does not (1, 5, 6: one-wave
kernel; S >= depth: one-wave kernel), flags, ragged sizes, replayed rays (binding 1) and bands."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests.helpers import assert_float_close, assert_rgba8_close
from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

pytestmark = pytest.mark.gpu

SMALL_ENV = (1024, 512)


def _renderer(halves: int):
    import vkcomputeshader_tinyraytracer_amd as trt

    old = os.environ.get("TRT_TILE_HALVES")
    os.environ["TRT_TILE_HALVES"] = str(halves)
    try:
        return trt.Renderer(0)
    finally:
        if old is None:
            os.environ.pop("TRT_TILE_HALVES", None)
        else:
            os.environ["TRT_TILE_HALVES"] = old


SPLITS = (1, 2, 3)


@pytest.fixture(scope="module")
def pair():
    rs = {s: _renderer(s) for s in (0,) + SPLITS}
    yield rs
    for r in rs.values():
        r.close()


def _same(pair, sc, p=None):
    p = p if p is not None else sc.params()
    for r in pair.values():
        r.upload_scene(sc)
    b8, b32, _ = pair[0].draw_frame(p, want32=True)
    c8, c32, _ = pair[0].draw_frame(p, want32=True, count=True)  # the counting pass
    assert np.array_equal(b8, c8) and np.array_equal(b32.view(np.uint32), c32.view(np.uint32))
    for s in SPLITS:
        a8, a32, _ = pair[s].draw_frame(p, want32=True)
        assert np.array_equal(a8, b8), s
        assert np.array_equal(a32.view(np.uint32), b32.view(np.uint32)), s
    return b8, b32


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 6])
def test_halves_depths_bit_identical(pair, depth):
    sc = S.config_c2(256, 192, env_size=SMALL_ENV)
    sc.max_depth = depth
    _same(pair, sc)


@pytest.mark.parametrize("flags", [
    T.FLAG_SPHERES,
    T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_CHECKER,
    T.FLAG_SPHERES | T.FLAG_ENVMAP,
    T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_SRGB_OUT,
])
def test_halves_flags_bit_identical(pair, flags):
    sc = S.config_c2(128, 96, env_size=SMALL_ENV)
    sc.flags = flags
    _same(pair, sc)


def test_halves_ragged_sizes(pair):
    for w, h in [(1, 1), (17, 5), (33, 65), (100, 3)]:
        _same(pair, S.config_c2(w, h, env_size=SMALL_ENV))


def test_halves_bands(pair):
    sc = S.config_c2(128, 100, env_size=SMALL_ENV)
    for rows, count, index in [(8, 4, 1), (1, 24, 11), (3, 5, 4)]:
        p = sc.params()
        p.band_rows, p.band_count, p.band_index = rows, count, index
        _same(pair, sc, p)


def test_halves_rays_in_replay(pair):
    """Binding 1 (rayIn): directions from the buffer, not the kernel's generator."""
    sc = S.config_c2(64, 48, env_size=SMALL_ENV)
    rng = np.random.default_rng(7)
    d = rng.normal(size=(48 * 64, 3)).astype(np.float32)
    d[:, 2] = -np.abs(d[:, 2]) - 0.5
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros(48 * 64, T.RAY)
    rays["dir"][:, :3] = d
    rays["dir"][:, 3] = 1.0
    out = []
    for r in pair.values():
        r.upload_scene(sc)
        out.append(r.draw_frame(sc.params(), want32=True, rays_in=rays))
    for o in out[1:]:
        assert np.array_equal(o[0], out[0][0])
        assert np.array_equal(o[1].view(np.uint32), out[0][1].view(np.uint32))


def test_halves_full_c2_frame_vs_oracle(pair):
    """The headline frame at full size through the two-wave launch, against the oracle."""
    sc = S.config_c2()
    a8, a32 = _same(pair, sc)
    o8, o32, _ = orc.render(sc, sc.params(), want32=True)
    assert_rgba8_close(a8, o8)
    assert_float_close(a32, o32)
