"""GPU: subtree split (trt_set_subtree_split) — deep refraction trees traced in depth windows
by task rounds.  Against the oracle's split mode (the same decomposition, same fixed-point
sums): ray and work counters exact, RGBA8 within 1 LSB, rayOut within FLOAT_TOL; bitwise
deterministic run to run; the same counters as the unsplit frame."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests.helpers import assert_float_close, assert_rgba8_close
from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

pytestmark = pytest.mark.gpu

SMALL_ENV = (1024, 512)


def _scenes(golden_meshes):
    ref = S.config_reference_default(golden_meshes, env_size=SMALL_ENV, width=160, height=120)
    c3 = S.config_c3(240, 136, env_size=SMALL_ENV)
    c2 = S.config_c2(128, 96, env_size=SMALL_ENV)
    c2.max_depth = 12
    return {"ref": ref, "c3": c3, "c2d12": c2}


@pytest.fixture(scope="module")
def scenes(golden_meshes):
    return _scenes(golden_meshes)


def _render(r, sc, window, flags=0):
    # the fixed-point split of the per-pixel loop (deferred-shadow frames keep the reference
    # order through LINK events instead: tests/test_gpu_defer.py)
    r.set_subtree_split(window)
    r.set_deferred_shadows(1)
    try:
        p = sc.params()
        p.flags |= flags
        return r.draw_frame(p, want32=True, count=True)
    finally:
        r.set_subtree_split(0)
        r.set_deferred_shadows(0)


@pytest.mark.parametrize("name", ["ref", "c3", "c2d12"])
@pytest.mark.parametrize("window", [2, 3, 4, 5])
def test_split_matches_oracle_split(gpu_renderer, scenes, name, window):
    sc = scenes[name]
    if window >= sc.max_depth:
        pytest.skip("window covers the whole tree: no split")
    gpu_renderer.upload_scene(sc)
    g8, g32, gst = _render(gpu_renderer, sc, window)
    o8, o32, ost = orc.render(sc, sc.params(), mode=orc.mode_split(window), want32=True)
    for k in T.Stats.EXACT:
        assert gst[k] == ost[k], (k, gst, ost)
    assert_rgba8_close(g8, o8)
    assert_float_close(g32, o32)
    # deterministic: the fixed-point pixel sums do not depend on task order
    h8, h32, _ = _render(gpu_renderer, sc, window)
    assert np.array_equal(h8, g8) and np.array_equal(h32, g32)
    # the unsplit frame traces the same rays
    u8, u32, ust = _render(gpu_renderer, sc, 1)
    for k in T.Stats.EXACT:
        assert ust[k] == gst[k]
    assert_rgba8_close(g8, u8)


def test_split_batch_walk_equals_bvh(gpu_renderer, scenes):
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    a8, a32, ast = _render(gpu_renderer, sc, 4)
    b8, b32, bst = _render(gpu_renderer, sc, 4, flags=T.FLAG_BATCH_WALK)
    assert np.array_equal(a8, b8) and np.array_equal(a32, b32)


def test_split_queue_overflow_falls_back_in_place(gpu_renderer, scenes, monkeypatch):
    """A queue far too small: children that do not fit are traced by their own lane (the hybrid
    deferred stack's private tail); rays are unchanged and colours stay within the bar."""
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    monkeypatch.setenv("TRT_SPLIT_QCAP", "64")
    g8, g32, gst = _render(gpu_renderer, sc, 2)
    monkeypatch.delenv("TRT_SPLIT_QCAP")
    o8, o32, ost = orc.render(sc, sc.params(), want32=True)
    for k in T.Stats.EXACT:
        assert gst[k] == ost[k]
    assert_rgba8_close(g8, o8)
    assert_float_close(g32, o32)


@pytest.mark.parametrize("defer", [1, 2])
def test_split_with_frames_in_flight(gpu_renderer, scenes, defer):
    """Concurrent split frames use per-slot queues: each equals the single-frame render
    (per-pixel loop with fixed-point split sums, and deferred shadows with LINK events)."""
    torch = pytest.importorskip("torch")
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    gpu_renderer.set_deferred_shadows(defer)
    n, H, W = 5, sc.height, sc.width
    ubos = np.stack([S.make_ubo(cam=(0.03 * i, 0.0, -0.05 * i)) for i in range(n)])
    out = torch.zeros((n, H, W, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    stream = torch.cuda.Stream()
    gpu_renderer.set_stream(stream)
    try:
        gpu_renderer.set_subtree_split(2)
        gpu_renderer.set_frames_in_flight(3)
        gpu_renderer.render_frames(sc.params(), out, n, ubos=ubos, frame_stride=H * W * 4)
        stream.synchronize()
        for i in range(n):
            gpu_renderer.update_ubo(ubos[i])
            one, _, _ = gpu_renderer.draw_frame(sc.params())
            assert np.array_equal(out[i].cpu().numpy(), one), i
    finally:
        gpu_renderer.set_frames_in_flight(0)
        gpu_renderer.set_subtree_split(0)
        gpu_renderer.set_deferred_shadows(0)
        gpu_renderer.set_stream(None)
        gpu_renderer.update_ubo(sc.ubo)
