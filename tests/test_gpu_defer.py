"""GPU: deferred frames (trt_set_deferred_shadows): pass A traces every pixel's tree without
shadow rays and logs its colour events, the tile's lanes sharing pending segments, pass B traces
the frame's shadow queries densely, and pass C sums each pixel's events in the reference's pop
order.

The bar is bitwise: a deferred frame must equal the per-pixel loop without subtree split (the
reference's single running sum, shader.comp:423-583) in both outputs, and — through it — the
reference-order oracle within the usual RGBA8 / rayOut bar, at the shipped frame's full size.
Pixels whose event log does not fit (tiny capacities forced through the test hooks
TRT_DEFER_EVCAP / TRT_DEFER_QCAP) are re-traced in place and must not change a bit either."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests.helpers import assert_float_close, assert_rgba8_close
from tests.test_gpu_parity import _host_ray
from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

pytestmark = pytest.mark.gpu

SMALL_ENV = (1024, 512)
DEFER_AUTO, DEFER_OFF, DEFER_ON = 0, 1, 2

def _frame(r, sc, defer, split=1, p=None):
    r.set_deferred_shadows(defer)
    r.set_subtree_split(split)
    try:
        p = p if p is not None else sc.params()
        g8, g32, _ = r.draw_frame(p, want32=True)
        return g8, g32
    finally:
        r.set_deferred_shadows(DEFER_AUTO)
        r.set_subtree_split(0)


def _scenes(golden_meshes):
    c2 = S.config_c2(128, 96, env_size=SMALL_ENV)
    c2.max_depth = 12
    return {
        "ref": S.config_reference_default(golden_meshes, env_size=SMALL_ENV, width=256, height=192),
        "readme": S.config_readme(golden_meshes, env_size=SMALL_ENV, width=200, height=150),
        "c3": S.config_c3(240, 136, env_size=SMALL_ENV),
        "c2d12": c2,
        "c1": S.config_c1(96, 64),
    }


@pytest.fixture(scope="module")
def scenes(golden_meshes):
    return _scenes(golden_meshes)


@pytest.mark.parametrize("name", ["ref", "readme", "c3", "c2d12", "c1"])
def test_deferred_frame_is_bit_identical_to_the_unsplit_loop(gpu_renderer, scenes, name):
    sc = scenes[name]
    gpu_renderer.upload_scene(sc)
    d8, d32 = _frame(gpu_renderer, sc, DEFER_ON)
    u8, u32 = _frame(gpu_renderer, sc, DEFER_OFF)
    assert np.array_equal(d8, u8)
    assert np.array_equal(d32, u32)
    st = gpu_renderer.defer_stats(0)
    assert st["fallback_pixels"] == 0, st
    assert st["queries"] <= st["query_cap"] and st["chunks"] <= st["chunk_cap"]


@pytest.mark.parametrize("name", ["ref", "readme", "c3", "c2d12"])
@pytest.mark.parametrize("window", [2, 3, 4, 5])
def test_deferred_split_keeps_the_reference_order(gpu_renderer, scenes, name, window):
    """Subtree split of a deferred frame: subtrees traced by other lanes log into chains of
    their own, reached through LINK events at the place of their events: the image is still the
    unsplit loop's bit for bit (no fixed-point sums)."""
    sc = scenes[name]
    if window >= sc.max_depth:
        pytest.skip("window covers the whole tree: no split")
    gpu_renderer.upload_scene(sc)
    d8, d32 = _frame(gpu_renderer, sc, DEFER_ON, split=window)
    st = gpu_renderer.defer_stats(0)
    u8, u32 = _frame(gpu_renderer, sc, DEFER_OFF, split=1)
    assert st["fallback_pixels"] == 0, st
    assert np.array_equal(d8, u8) and np.array_equal(d32, u32)


def test_deferred_split_task_queue_overflow(gpu_renderer, scenes, monkeypatch):
    """A task queue far too small: pixels whose subtree does not fit are re-traced in place."""
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    u8, u32 = _frame(gpu_renderer, sc, DEFER_OFF, split=1)
    monkeypatch.setenv("TRT_SPLIT_QCAP", "64")
    d8, d32 = _frame(gpu_renderer, sc, DEFER_ON, split=2)
    st = gpu_renderer.defer_stats(0)
    monkeypatch.delenv("TRT_SPLIT_QCAP")
    assert st["fallback_pixels"] > 0, st
    assert np.array_equal(d8, u8) and np.array_equal(d32, u32)


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 7, 20])
def test_deferred_depths(gpu_renderer, scenes, depth):
    sc = scenes["c3"]
    gpu_renderer.upload_scene(sc)
    p = sc.params()
    p.max_depth = depth
    d8, d32 = _frame(gpu_renderer, sc, DEFER_ON, p=p)
    u8, u32 = _frame(gpu_renderer, sc, DEFER_OFF, p=p)
    assert np.array_equal(d8, u8) and np.array_equal(d32, u32)


def test_shipped_frame_full_size_deferred_vs_reference_order_oracle(gpu_renderer, golden_meshes):
    """The shipped frame (glass + water + ice, depth 20) at 1024x768 through the default
    (automatic) path — a deferred frame — against the oracle's reference-order running sum."""
    sc = S.config_reference_default(golden_meshes, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    g8, g32, _ = gpu_renderer.draw_frame(sc.params(), want32=True)
    st = gpu_renderer.defer_stats(0)
    assert st["queries"] > 0 and st["fallback_pixels"] == 0, st
    o8, o32, _ = orc.render(sc, sc.params(), want32=True)
    assert_rgba8_close(g8, o8)
    assert_float_close(g32, o32)


@pytest.mark.parametrize("hook,value", [("TRT_DEFER_EVCAP", "8"), ("TRT_DEFER_QCAP", "300"), ("TRT_DEFER_EVCAP", "0")])
def test_overflow_pixels_are_retraced_in_place(gpu_renderer, scenes, monkeypatch, hook, value):
    """Children that do not fit (event chunks or the query queue) send their pixels to the
    in-place fallback: the image must not change a bit.  TRT_DEFER_EVCAP=0 leaves no event slot
    at all (every pixel is re-traced)."""
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    u8, u32 = _frame(gpu_renderer, sc, DEFER_OFF)
    monkeypatch.setenv(hook, value)
    for split in (1, 3):
        d8, d32 = _frame(gpu_renderer, sc, DEFER_ON, split=split)
        st = gpu_renderer.defer_stats(0)
        assert st["fallback_pixels"] > 0, (split, st)
        # the stats count against the capacity the frame ran with (the hook's), not the allocation
        if hook == "TRT_DEFER_QCAP":
            assert st["queries"] <= int(value) * 128, st
        assert np.array_equal(d8, u8) and np.array_equal(d32, u32), split
    monkeypatch.delenv(hook)


def test_deferred_frames_in_flight(gpu_renderer, scenes):
    """render_frames with 1..4 frames in flight (one scratch set per slot): every frame equals
    the single deferred frame."""
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    u8, _ = _frame(gpu_renderer, sc, DEFER_OFF)
    p = sc.params()
    out = torch.empty((6, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    gpu_renderer.set_deferred_shadows(DEFER_ON)
    try:
        for n in (1, 2, 3, 4, 8, 0):
            out.zero_()
            gpu_renderer.set_frames_in_flight(n)
            gpu_renderer.render_frames(p, out, 6, frame_stride=p.height * p.width * 4)
            torch.cuda.synchronize()
            for f in range(6):
                assert np.array_equal(out[f].cpu().numpy(), u8), (n, f)
    finally:
        gpu_renderer.set_frames_in_flight(0)
        gpu_renderer.set_deferred_shadows(DEFER_AUTO)


def test_deferred_bands_and_ray_replay(gpu_renderer, scenes):
    """Band launches (the multi-GPU tiling's unit) and binding-1 ray replay go through the
    deferred passes unchanged."""
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    full8, _ = _frame(gpu_renderer, sc, DEFER_OFF)
    for idx in range(3):
        p = sc.params()
        p.band_rows, p.band_count, p.band_index = 8, 3, idx
        b8, _ = _frame(gpu_renderer, sc, DEFER_ON, p=p)
        rows = [y for y in range(p.height) if (y // 8) % 3 == idx]
        assert np.array_equal(b8, full8[rows])
    p = sc.params()
    rays = np.zeros(p.width * p.height, T.RAY)
    for y in range(p.height):
        for x in range(p.width):
            rays[y * p.width + x]["dir"] = (*_host_ray(p, x, y), 1.0)
    gpu_renderer.set_deferred_shadows(DEFER_ON)
    try:
        r8, _, _ = gpu_renderer.draw_frame(p, rays_in=rays)
    finally:
        gpu_renderer.set_deferred_shadows(DEFER_AUTO)
    assert np.array_equal(r8, full8)


def test_batch_walk_deferred(gpu_renderer, scenes):
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    p = sc.params()
    p.flags |= T.FLAG_BATCH_WALK
    d8, d32 = _frame(gpu_renderer, sc, DEFER_ON, p=p)
    u8, u32 = _frame(gpu_renderer, sc, DEFER_OFF)
    assert np.array_equal(d8, u8) and np.array_equal(d32, u32)


def test_count_frames_keep_reference_counters(gpu_renderer, scenes):
    """COUNT frames always run the per-pixel loop: same counters as the oracle."""
    sc = scenes["ref"]
    gpu_renderer.upload_scene(sc)
    gpu_renderer.set_deferred_shadows(DEFER_ON)
    try:
        _, _, gst = gpu_renderer.draw_frame(sc.params(), count=True)
    finally:
        gpu_renderer.set_deferred_shadows(DEFER_AUTO)
    _, _, ost = orc.render(sc, sc.params())
    for k in T.Stats.EXACT:
        assert gst[k] == ost[k], k


@pytest.mark.parametrize("ppw", ["8", "16", "32", "64"])
def test_pass_a_pixels_per_wave(scenes, ppw):
    """TRT_DEFER_PPW: pass A with 64 / 32 / 16 / 8 pixels per wave (1, 2, 4, 8 waves per 8x8
    tile, the other lanes fed by the wave's segment pool) — the frame is the unsplit loop's bit
    for bit (the automatic choice, 4 waves per tile at <= 2 frames in flight, is what trt_render
    runs)."""
    import os

    import vkcomputeshader_tinyraytracer_amd as trt

    old = os.environ.get("TRT_DEFER_PPW")
    os.environ["TRT_DEFER_PPW"] = ppw
    try:
        r = trt.Renderer(0)
    finally:
        if old is None:
            os.environ.pop("TRT_DEFER_PPW", None)
        else:
            os.environ["TRT_DEFER_PPW"] = old
    try:
        for name in ("ref", "readme"):
            sc = scenes[name]
            r.upload_scene(sc)
            d8, d32 = _frame(r, sc, DEFER_ON)
            u8, u32 = _frame(r, sc, DEFER_OFF)
            assert np.array_equal(d8, u8) and np.array_equal(d32, u32), name
            assert r.defer_stats(0)["fallback_pixels"] == 0
    finally:
        r.close()


def test_auto_in_flight_drops_a_slot_that_runs_out_of_memory(scenes, monkeypatch):
    """Auto frames in flight: a slot whose deferred scratch cannot be allocated (out of memory,
    injected for slot 2 through the test hooks) is dropped with the slots after it, the failed
    allocation's error does not leak into the next launch, and every frame still equals the
    single deferred frame."""
    import vkcomputeshader_tinyraytracer_amd as trt

    sc = scenes["ref"]
    r = trt.Renderer(0)
    try:
        r.upload_scene(sc)
        u8, _ = _frame(r, sc, DEFER_OFF)
        monkeypatch.setenv("TRT_ENABLE_TEST_HOOKS", "1")
        monkeypatch.setenv("TRT_TEST_FAIL_DEFER_SLOT", "2")
        p = sc.params()
        n = 24  # enough frames to reach slot 2 with any automatic shape (8 slots x 3 at >= 16 queues)
        out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        r.set_deferred_shadows(DEFER_ON)
        r.render_frames(p, out, n, frame_stride=p.height * p.width * 4)
        torch.cuda.synchronize()
        for f in range(n):
            assert np.array_equal(out[f].cpu().numpy(), u8), f
        # an explicit in-flight count is the caller's: the same failure is reported, not hidden
        r.set_frames_in_flight(4)
        with pytest.raises(trt.TrtError):
            r.render_frames(p, out, 6, frame_stride=p.height * p.width * 4)
    finally:
        monkeypatch.delenv("TRT_TEST_FAIL_DEFER_SLOT", raising=False)
        r.close()


@pytest.mark.parametrize("group,inflight,inter", [(2, 0, 2), (3, 2, 2), (4, 4, 2), (8, 1, 2), (16, 0, 2),
                                                 (3, 2, 0), (8, 1, 0), (3, 2, 1), (8, 1, 1)])
def test_deferred_frame_groups(scenes, group, inflight, inter):
    """TRT_DEFER_GROUP: consecutive deferred frames of a frame loop traced by one launch sequence
    (pass A over every frame's tiles, one pass B and one pass C over all of them, each frame with
    its own scratch), their blocks dealt frame-major (TRT_DEFER_INTER=0), interleaved frame by
    frame in pass A (1) or in all three passes (2, the default).  Ragged groups (the loop's last
    group is shorter), groups in flight and both scenes: every frame equals the single deferred
    frame of its UBO bit for bit."""
    import vkcomputeshader_tinyraytracer_amd as trt

    knobs = {"TRT_DEFER_GROUP": str(group), "TRT_DEFER_INTER": str(inter)}
    old = {k: os.environ.get(k) for k in knobs}
    os.environ.update(knobs)
    try:
        r = trt.Renderer(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for name in ("ref", "readme"):
            sc = scenes[name]
            r.upload_scene(sc)
            p = sc.params()
            n = 2 * group + 1
            ubos = np.stack(S.camera_path(sc.ubo, n))
            out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            r.set_deferred_shadows(DEFER_ON)
            r.set_frames_in_flight(inflight)
            r.render_frames(p, out, n, ubos=ubos, frame_stride=p.height * p.width * 4)
            torch.cuda.synchronize()
            r.set_frames_in_flight(0)
            got = out.cpu().numpy()
            for i in range(n):
                r.update_ubo(ubos[i])
                one, _ = _frame(r, sc, DEFER_ON)
                assert np.array_equal(got[i], one), (name, i)
    finally:
        r.close()
