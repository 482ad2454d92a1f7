"""GPU parity: the HIP kernel (through the C-ABI) against the CPU oracle on the same seeded
inputs.  Bar: RGBA8 within 1 LSB per channel, rayOut floats within FLOAT_TOL, and the ray
counts (which depend only on geometry) EXACTLY equal.  Run with `pytest -m gpu`."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as orc
from tests.helpers import MAX_FRAC, assert_float_close, assert_rgba8_close
from vkcomputeshader_tinyraytracer_amd import TrtError, scene as S, types as T

pytestmark = pytest.mark.gpu

SMALL_ENV = (1024, 512)


def _counts(st, keys=T.Stats.EXACT):
    return tuple(st[k] for k in keys)


def _check(r, sc, params=None, want32=True, max_frac=MAX_FRAC):
    """Kernel vs oracle; for mesh scenes both the per-ray BVH (default) and the
    reference-order batch walk (TRT_FLAG_BATCH_WALK) must match, the walk also in its
    batch/triangle work counters."""
    p = params if params is not None else sc.params()
    r.upload_scene(sc)
    g8, g32, gst = r.draw_frame(p, want32=want32, count=True)
    o8, o32, ost = orc.render(sc, p, want32=want32)
    assert _counts(gst) == _counts(ost), (gst, ost)
    if len(sc.models):
        pw = T.Params.from_buffer_copy(p)
        pw.flags |= T.FLAG_BATCH_WALK
        w8, w32, wst = r.draw_frame(pw, want32=want32, count=True)
        assert _counts(wst, T.Stats.EXACT_WALK) == _counts(ost, T.Stats.EXACT_WALK), (wst, ost)
        assert np.array_equal(w8, g8) and (not want32 or np.array_equal(w32, g32))
    rep = assert_rgba8_close(g8, o8, max_frac=max_frac)
    if want32:
        assert_float_close(g32, o32)
    return rep, gst


def test_c1_full_frame(gpu_renderer):
    rep, st = _check(gpu_renderer, S.config_c1())
    assert st["primary_rays"] == 1024 * 768 and st["secondary_rays"] == 0


def test_c2_full_frame_reference_envmap_size(gpu_renderer):
    """Headline config at full size: 1024x768, depth 4, 7616x3808 envmap."""
    rep, st = _check(gpu_renderer, S.config_c2())
    assert st["secondary_rays"] > 0


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 6, 8, 12, 20])
def test_c2_depths(gpu_renderer, depth):
    """Every deferred-stack instantiation (register shift-stack and private array)."""
    sc = S.config_c2(256, 192, env_size=SMALL_ENV)
    sc.max_depth = depth
    _check(gpu_renderer, sc)


def test_c3_mesh(gpu_renderer):
    _check(gpu_renderer, S.config_c3(480, 270, env_size=SMALL_ENV))


def test_c4_many_batches(gpu_renderer):
    _check(gpu_renderer, S.config_c4(384, 216, env_size=SMALL_ENV))


def test_reference_default_scene(gpu_renderer, golden_meshes):
    """The shipped frame: glass+water+ice, spheres off, floor on, MAX_DEPTH 20."""
    sc = S.config_reference_default(golden_meshes, env_size=SMALL_ENV, width=256, height=192)
    assert len(sc.tris) == 37956 and len(sc.models) == 594
    _check(gpu_renderer, sc)


def test_readme_scene_rotated_models(gpu_renderer, golden_meshes):
    """README-era scene (config.hpp:96): rotated + flat-shaded models, checker floor."""
    tris, models = S.build_models(S.README_MODEL_LIST, golden_meshes)
    sc = S.Scene("readme", S.make_ubo(), tris, models, S.cached_envmap(*SMALL_ENV), 200, 150, 6,
                 flags=T.FLAG_FLOOR | T.FLAG_CHECKER | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)
    _check(gpu_renderer, sc)


@pytest.mark.parametrize("spp", [2, 4])
def test_jittered_spp(gpu_renderer, spp):
    sc = S.config_c2(160, 120, env_size=SMALL_ENV)
    sc.spp = spp
    _check(gpu_renderer, sc)


def test_c5_sixteen_spp(gpu_renderer):
    """C5 (BASELINE configs[4]): the ~100k-triangle C4 scene at 16 jittered samples per pixel,
    reduced size; the per-pixel average of 16 clamped samples, then gamma."""
    sc = S.config_c5(96, 64, env_size=SMALL_ENV)
    assert sc.spp == 16
    rep, st = _check(gpu_renderer, sc)
    assert st["primary_rays"] == 96 * 64 * 16


@pytest.mark.parametrize("flags", [
    0,
    T.FLAG_FLOOR,
    T.FLAG_SPHERES,
    T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_CHECKER,
    T.FLAG_SPHERES | T.FLAG_ENVMAP,
])
def test_flag_combinations(gpu_renderer, flags):
    sc = S.config_c2(128, 96, env_size=SMALL_ENV)
    sc.flags = flags
    _check(gpu_renderer, sc)


def test_row_quirk_off(gpu_renderer):
    sc = S.config_c2(128, 96, env_size=SMALL_ENV)
    sc.flags &= ~T.FLAG_ROW_QUIRK
    _check(gpu_renderer, sc)


def test_ragged_sizes(gpu_renderer):
    """Image sizes that are not multiples of the 16x16 workgroup tile."""
    for w, h in [(1, 1), (17, 5), (33, 65), (100, 3)]:
        sc = S.config_c2(w, h, env_size=SMALL_ENV)
        _check(gpu_renderer, sc)


def test_bands_equal_rows_of_full_frame(gpu_renderer):
    sc = S.config_c2(128, 100, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    full, _, _ = gpu_renderer.draw_frame(sc.params())
    for count in (2, 3, 8):
        parts = []
        for idx in range(count):
            p = sc.params(band_rows=8, band_count=count, band_index=idx)
            band, _, _ = gpu_renderer.draw_frame(p)
            rows = T.output_rows(sc.height, 8, count, idx)
            assert band.shape[0] == len(rows)
            assert np.array_equal(band, full[rows])
            parts.append(rows)
        assert sorted(sum(parts, [])) == list(range(sc.height))


@pytest.mark.parametrize("which", ["C2", "reference"])
def test_bands_in_place_assemble_the_frame(gpu_renderer, golden_meshes, which):
    """TRT_FLAG_BAND_IN_PLACE: each band launch writes its rows at their frame rows, so the
    bands of one frame rendered into one device image give the whole frame (the multi-GPU root
    renders its own bands this way); also through the deferred-shadow passes."""
    torch = pytest.importorskip("torch")
    sc = (S.config_c2(128, 100, env_size=SMALL_ENV) if which == "C2" else
          S.config_reference_default(golden_meshes, env_size=SMALL_ENV, width=160, height=120))
    gpu_renderer.upload_scene(sc)
    full, full32, _ = gpu_renderer.draw_frame(sc.params(), want32=True)
    out8 = torch.zeros((sc.height, sc.width, 4), dtype=torch.uint8, device="cuda")
    out32 = torch.zeros((sc.height, sc.width, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    for idx in range(3):
        p = sc.params(band_rows=8, band_count=3, band_index=idx)
        p.flags |= T.FLAG_BAND_IN_PLACE
        gpu_renderer.draw_frame(p, out8=out8, out32=out32)
    torch.cuda.synchronize()
    assert np.array_equal(out8.cpu().numpy(), full)
    assert np.array_equal(out32.cpu().numpy(), full32)
    p = sc.params(band_rows=8, band_count=3, band_index=0)
    p.flags |= T.FLAG_BAND_IN_PLACE
    with pytest.raises(TrtError):  # host outputs cannot hold a band in place
        gpu_renderer.draw_frame(p)


def test_rays_in_replay(gpu_renderer):
    """Binding 1 replay: host rays built as main.cpp:1496-1506 does give the same frame."""
    sc = S.config_c2(96, 64, env_size=SMALL_ENV)
    p = sc.params()
    rays = np.zeros(p.width * p.height, T.RAY)
    for y in range(p.height):
        for x in range(p.width):
            rays[y * p.width + x]["dir"] = (*_host_ray(p, x, y), 1.0)
    gpu_renderer.upload_scene(sc)
    a, _, _ = gpu_renderer.draw_frame(p)
    b, _, _ = gpu_renderer.draw_frame(p, rays_in=rays)
    assert np.array_equal(a, b)


def _host_ray(p, x, y):
    """Host primary ray exactly as main.cpp:1499-1505 (double, then glm::normalize in float)."""
    W, H = p.width, p.height
    pix = y * W + x
    dx = np.float32((pix % W + 0.5) - W / 2.0)
    dy = np.float32(-((pix + 1) // W + 0.5) + H / 2.0)
    dz = np.float32(-1.0 * (H / (2.0 * np.tan(np.float64(np.float32(p.fov)) / 2.0))))
    s = (dx * dx + dy * dy) + dz * dz
    inv = np.float32(1.0) / np.sqrt(np.float32(s))
    return dx * inv, dy * inv, dz * inv


def test_device_pointers_torch(gpu_renderer):
    torch = pytest.importorskip("torch")
    sc = S.config_c2(160, 96, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    host8, host32, _ = gpu_renderer.draw_frame(sc.params(), want32=True)
    out8 = torch.empty((96, 160, 4), dtype=torch.uint8, device="cuda")
    out32 = torch.empty((96, 160, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.Stream()
    gpu_renderer.set_stream(stream)
    gpu_renderer.draw_frame(sc.params(), out8=out8, out32=out32)
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        gpu_renderer.set_stream(torch.cuda.default_stream())
    gpu_renderer.set_stream(None)
    assert np.array_equal(out8.cpu().numpy(), host8)
    assert np.array_equal(out32.cpu().numpy(), host32)


def test_deterministic(gpu_renderer):
    sc = S.config_c3(200, 120, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    a, _, sa = gpu_renderer.draw_frame(sc.params(), count=True)
    b, _, sb = gpu_renderer.draw_frame(sc.params(), count=True)
    assert np.array_equal(a, b) and sa == sb


def test_update_ubo_moves_camera(gpu_renderer):
    """updateUniformBuffer (main.cpp:2165-2179): a new camPos without re-uploading geometry."""
    sc = S.config_c2(128, 96, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    sc2 = S.config_c2(128, 96, env_size=SMALL_ENV)
    sc2.ubo = S.make_ubo(cam=(0.5, 0.25, -1.0))
    gpu_renderer.update_ubo(sc2.ubo)
    g8, _, _ = gpu_renderer.draw_frame(sc2.params())
    o8, _, _ = orc.render(sc2, sc2.params())
    assert_rgba8_close(g8, o8)


def test_errors(gpu_renderer):
    sc = S.config_c2(64, 48, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    with pytest.raises(TrtError):
        gpu_renderer.draw_frame(sc.params(max_depth=0))
    with pytest.raises(TrtError):
        gpu_renderer.draw_frame(sc.params(max_depth=21))
    with pytest.raises(TrtError):
        gpu_renderer.draw_frame(sc.params(band_rows=8, band_count=2, band_index=2))
    bad = S.Scene("bad", S.make_ubo(), sc.tris, np.zeros(1, T.MODEL))
    bad.models["params0"] = (0, 5, 0, 0)  # range beyond the (empty) triangle buffer
    with pytest.raises(TrtError):
        gpu_renderer.upload_scene(bad)
    no_env = S.Scene("noenv", S.make_ubo(), flags=T.FLAG_ENVMAP)
    gpu_renderer.upload_scene(no_env)
    with pytest.raises(TrtError):
        gpu_renderer.draw_frame(no_env.params(width=8, height=8))


def test_frame_loop_matches_single_frames(gpu_renderer):
    """trt_render_frames (native frame loop with per-frame UBOs) == trt_render per frame."""
    torch = pytest.importorskip("torch")
    sc = S.config_c2(96, 64, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    ubos = np.stack([S.make_ubo(cam=(0.1 * i, 0.0, -0.2 * i)) for i in range(4)])
    out = torch.zeros((4, 64, 96, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    stream = torch.cuda.Stream()
    gpu_renderer.set_stream(stream)
    try:
        # one launch per frame: every launch timed, per-frame times
        gpu_renderer.set_frame_batch(1)
        assert gpu_renderer.render_frames(sc.params(), out, 4, ubos=ubos, frame_stride=64 * 96 * 4, timing=True) == 4
        ms = gpu_renderer.frame_times(4)
        torch.cuda.synchronize()
        assert (ms > 0).all()
        assert list(gpu_renderer.launch_frames()) == [1, 1, 1, 1]
        # sampled timing: launches 0 and 3 of 4 are bracketed; asking for more is an error
        assert gpu_renderer.render_frames(sc.params(), out, 4, ubos=ubos, frame_stride=64 * 96 * 4,
                                          timing=True, time_every=3) == 2
        assert (gpu_renderer.frame_times(2) > 0).all()
        with pytest.raises(TrtError):
            gpu_renderer.frame_times(3)
        # auto batching on one in-flight slot: the 4 camera-only frames are one launch; its
        # time is per frame
        gpu_renderer.set_frame_batch(0)
        gpu_renderer.set_frames_in_flight(1)
        assert gpu_renderer.render_frames(sc.params(), out, 4, ubos=ubos, frame_stride=64 * 96 * 4, timing=True) == 1
        assert list(gpu_renderer.launch_frames()) == [4]
        assert (gpu_renderer.frame_times(1) > 0).all()
        # with 2 slots the frames are spread over two launches (one per hardware queue)
        gpu_renderer.set_frames_in_flight(2)
        assert gpu_renderer.render_frames(sc.params(), out, 4, ubos=ubos, frame_stride=64 * 96 * 4, timing=True) == 2
        assert list(gpu_renderer.launch_frames()) == [2, 2]
        torch.cuda.synchronize()
    finally:
        gpu_renderer.set_frame_batch(0)
        gpu_renderer.set_frames_in_flight(0)
        gpu_renderer.set_stream(None)
    for i in range(4):
        gpu_renderer.update_ubo(ubos[i])
        one, _, _ = gpu_renderer.draw_frame(sc.params())
        assert np.array_equal(out[i].cpu().numpy(), one)


def test_prepared_frame_list_matches_render_frames(gpu_renderer):
    """Renderer.frames_call (the bench's timed loop: checks done once, one native call per
    issue) renders what render_frames renders, and re-issuing it renders the same frames."""
    torch = pytest.importorskip("torch")
    sc = S.config_c2(96, 64, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    ubos = np.stack([S.make_ubo(cam=(0.1 * i, 0.0, -0.2 * i)) for i in range(5)])
    fb = 64 * 96 * 4
    a = torch.zeros((5, 64, 96, 4), dtype=torch.uint8, device="cuda")
    b = torch.zeros_like(a)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    gpu_renderer.set_stream(stream)
    try:
        gpu_renderer.render_frames(sc.params(), a, 5, ubos=ubos, frame_stride=fb)
        call = gpu_renderer.frames_call(sc.params(), b, 5, ubos=ubos, frame_stride=fb)
        call()
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        b.zero_()
        torch.cuda.synchronize()
        call()
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        with pytest.raises(ValueError):
            gpu_renderer.frames_call(sc.params(), b[:2], 5, ubos=ubos, frame_stride=fb)
        with pytest.raises(ValueError):
            gpu_renderer.frames_call(sc.params(), b, 5, ubos=ubos[:3], frame_stride=fb)
    finally:
        gpu_renderer.set_stream(None)


def _moving_ubos(n, sphere_every=0):
    """Per-frame UBOs: the camera moves every frame (main.cpp:391-403); with sphere_every > 0
    sphere 0 also moves every sphere_every frames, which splits a multi-frame launch there."""
    ubos = []
    for i in range(n):
        u = S.make_ubo(cam=(0.07 * i, 0.02 * (i % 3), -0.1 * i))
        if sphere_every and (i // sphere_every) % 2:
            u["sphere0"]["center_radius"][0] += 0.25
        ubos.append(u)
    return np.stack(ubos)


@pytest.mark.parametrize("batch,inflight", [(0, 0), (1, 0), (2, 1), (3, 2), (5, 3), (64, 1), (0, 4)])
@pytest.mark.parametrize("config,sphere_every", [("C2", 0), ("C2", 4), ("C3", 3), ("C5", 0)])
def test_multi_frame_launches_match_single_frames(gpu_renderer, config, sphere_every, batch, inflight):
    """Multi-frame launches (trt_set_frame_batch): frame k of a launch owns blocks [k * ntiles,
    (k + 1) * ntiles) with its own camera and image.  Every frame equals one-at-a-time trt_render
    bit for bit, for launch sizes that divide the loop unevenly, UBOs that change more than the
    camera (the launch splits there), a mesh scene (BVH walk) and 4 spp (the C5 sampler)."""
    torch = pytest.importorskip("torch")
    if config == "C5":
        sc = S.CONFIGS["C3"](72, 40, env_size=SMALL_ENV)
        p = sc.params(spp=4)
    else:
        sc = S.CONFIGS[config](88, 56, env_size=SMALL_ENV)
        p = sc.params()
    gpu_renderer.upload_scene(sc)
    n = 11
    ubos = _moving_ubos(n, sphere_every)
    fb = p.height * p.width * 4
    out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    stream = torch.cuda.Stream()
    gpu_renderer.set_stream(stream)
    try:
        gpu_renderer.set_frame_batch(batch)
        gpu_renderer.set_frames_in_flight(inflight)
        gpu_renderer.render_frames(p, out, n, ubos=ubos, frame_stride=fb, timing=True)
        launches = gpu_renderer.launch_frames()
        stream.synchronize()
    finally:
        gpu_renderer.set_frame_batch(0)
        gpu_renderer.set_frames_in_flight(0)
        gpu_renderer.set_stream(None)
    assert int(launches.sum()) == n
    # frames per launch: ceil(n / in-flight slots), at most the batch size (auto: one slot)
    per = max(1, min(batch or 64, -(-n // (inflight or 1))))
    assert launches.max() <= per
    if sphere_every:
        assert len(launches) >= (n + sphere_every - 1) // sphere_every
    else:
        assert len(launches) == -(-n // per)
    got = out.cpu().numpy()
    for i in range(n):
        gpu_renderer.update_ubo(ubos[i])
        one, _, _ = gpu_renderer.draw_frame(p)
        assert np.array_equal(got[i], one), i
    gpu_renderer.update_ubo(sc.ubo)


@pytest.mark.parametrize("rot,skew,inter,pair", [(1, 0, 0, 1), (2, 3, 0, 1), (0, 5, 0, 1), (4, 1, 0, 1), (0, 0, 1, 1),
                                                (1, 3, 1, 1), (1, 0, 1, 2), (0, 3, 1, 2), (1, 0, 2, 2), (0, 3, 2, 1)])
@pytest.mark.parametrize("size", [(264, 200), (256, 128), (88, 56)])
def test_xcd_dealing_knobs_match_single_frames(rot, skew, inter, pair, size):
    """TRT_XCD_ROT / TRT_XCD_SKEW / TRT_XCD_INTER re-deal a multi-frame launch's tiles to the
    XCDs (rotated chunk classes per frame, diagonal classes, frames interleaved per chunk group;
    INTER=2: no rotation, chunk classes permuted by a coprime multiplier)
    and TRT_FRAME_GROUP=2 has a workgroup trace its tile in two consecutive frames (9 frames: the
    last pair is one frame): a bijection, so every frame still equals
    trt_render bit for bit — image sizes with leftover chunks, an odd tile column and row
    (264x200), whole chunk rows (256x128) and fewer chunks than XCDs per row (88x56)."""
    torch = pytest.importorskip("torch")
    import os

    import vkcomputeshader_tinyraytracer_amd as trt

    knobs = {"TRT_XCD_ROT": rot, "TRT_XCD_SKEW": skew, "TRT_XCD_INTER": inter, "TRT_FRAME_GROUP": pair}
    old = {k: os.environ.get(k) for k in knobs}
    os.environ.update({k: str(v) for k, v in knobs.items()})
    try:
        r = trt.Renderer(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        sc = S.CONFIGS["C2"](*size, env_size=SMALL_ENV)
        p = sc.params()
        r.upload_scene(sc)
        n = 9
        ubos = _moving_ubos(n)
        fb = p.height * p.width * 4
        out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        stream = torch.cuda.Stream()
        r.set_stream(stream)
        r.render_frames(p, out, n, ubos=ubos, frame_stride=fb, timing=True)
        assert list(r.launch_frames()) == [n]
        stream.synchronize()
        r.set_stream(None)
        got = out.cpu().numpy()
        for i in range(n):
            r.update_ubo(ubos[i])
            one, _, _ = r.draw_frame(p)
            assert np.array_equal(got[i], one), i
    finally:
        r.close()


def test_frame_batch_bounds(gpu_renderer):
    for bad in (65, 1000):
        with pytest.raises(TrtError):
            gpu_renderer.set_frame_batch(bad)
    gpu_renderer.set_frame_batch(0)


@pytest.mark.parametrize("inflight", [1, 2, 3, 4, 8, 16, 0])
def test_frames_in_flight_match_single_frames(gpu_renderer, inflight):
    """Frames in flight (trt_set_frames_in_flight, main.cpp:45): concurrent frames with
    distinct UBOs and images equal one-at-a-time trt_render, and all of them have landed on
    the caller's stream when render_frames returns (no explicit join by the caller)."""
    torch = pytest.importorskip("torch")
    sc = S.config_c2(96, 64, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    n = 9
    ubos = np.stack([S.make_ubo(cam=(0.07 * i, 0.02 * i, -0.1 * i)) for i in range(n)])
    out = torch.zeros((n, 64, 96, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    stream = torch.cuda.Stream()
    gpu_renderer.set_stream(stream)
    try:
        gpu_renderer.set_frames_in_flight(inflight)
        gpu_renderer.render_frames(sc.params(), out, n, ubos=ubos, frame_stride=64 * 96 * 4)
        # work enqueued on the caller's stream after the call sees every frame
        with torch.cuda.stream(stream):
            snap = out.clone()
        stream.synchronize()
    finally:
        gpu_renderer.set_frames_in_flight(0)
        gpu_renderer.set_stream(None)
    for i in range(n):
        gpu_renderer.update_ubo(ubos[i])
        one, _, _ = gpu_renderer.draw_frame(sc.params())
        assert np.array_equal(snap[i].cpu().numpy(), one), i


def test_frames_in_flight_bounds(gpu_renderer):
    for bad in (33, 100):  # TRT_MAX_FRAMES_IN_FLIGHT = 32
        with pytest.raises(TrtError):
            gpu_renderer.set_frames_in_flight(bad)
    gpu_renderer.set_frames_in_flight(32)
    gpu_renderer.set_frames_in_flight(0)


def test_duplicate_triangles_first_batch_wins(gpu_renderer):
    """Two copies of one mesh at the same place with different materials: every hit is a t
    tie, and the reference's strict `t < nearest` (shader.comp:349) keeps the copy in the
    earlier batch.  Exercises the BVH's (t, batch, triangle) tie-break."""
    pos, idx = S.icosphere(2)
    b = S.SceneBuilder()
    b.add_mesh(pos, idx, S.GLASS_MESH_MAT, scale=(2, 2, 2), translation=(0.5, -1, -9), normal_interp=1)
    b.add_mesh(pos, idx, S.DRAGON_MAT, scale=(2, 2, 2), translation=(0.5, -1, -9), normal_interp=0)
    tris, models = b.arrays()
    sc = S.Scene("dup", S.make_ubo(), tris, models, S.cached_envmap(*SMALL_ENV), 96, 72, 6,
                 flags=T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)
    _check(gpu_renderer, sc)


def test_overlapping_batches_fall_back_to_walk(gpu_renderer):
    """Model records whose triangle ranges overlap (possible through the ABI, never built by
    the reference's host code): no BVH is built, the batch walk runs, results match."""
    pos, idx = S.icosphere(2)
    b = S.SceneBuilder()
    b.add_mesh(pos, idx, S.ICE_MAT, scale=(1.5, 1.5, 1.5), translation=(-1, -1, -8), normal_interp=1)
    tris, models = b.arrays()
    extra = models[:2].copy()
    extra["params0"][:, 0] = (10, 40)
    extra["params0"][:, 1] = (60, 60)
    extra["material"] = S.RED_RUBBER
    models = np.concatenate([models, extra])
    sc = S.Scene("overlap", S.make_ubo(), tris, models, S.cached_envmap(*SMALL_ENV), 80, 60, 5,
                 flags=T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)
    _check(gpu_renderer, sc)


def test_bvh_four_wave_build_bit_identical(gpu_renderer, golden_meshes, monkeypatch):
    """The BVH walk compiled for 4 waves per SIMD (GEOM 3, picked for large meshes; forced here
    with TRT_BVH_WAVES4, read at trt_create) renders exactly what the 3-wave build renders:
    images, rayOut and the reference-work counters, with and without the subtree split.  (The
    4-wave build walks the quantized 64-B nodes, so its traversal work counters differ.)"""
    from vkcomputeshader_tinyraytracer_amd import Renderer

    scenes = [S.config_c3(240, 136, env_size=SMALL_ENV),
              S.config_reference_default(golden_meshes, env_size=SMALL_ENV, width=160, height=120)]
    out = {}
    for force in ("0", "1"):
        monkeypatch.setenv("TRT_BVH_WAVES4", force)
        with Renderer(0) as r:
            for i, sc in enumerate(scenes):
                r.upload_scene(sc)
                out[force, i] = r.draw_frame(sc.params(), want32=True, count=True)
                r.set_subtree_split(3)
                out[force, i, "split"] = r.draw_frame(sc.params(), want32=True, count=True)
                r.set_subtree_split(0)
    monkeypatch.delenv("TRT_BVH_WAVES4")
    for key in [k for k in out if k[0] == "0"]:
        a8, a32, ast = out[key]
        b8, b32, bst = out[("1",) + key[1:]]
        assert np.array_equal(a8, b8) and np.array_equal(a32, b32), key
        assert {k: ast[k] for k in T.Stats.EXACT} == {k: bst[k] for k in T.Stats.EXACT}


def _cube():
    pos = np.array([(x, y, z) for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    idx = np.array([t for a, b, c, d in quads for t in ((a, b, c), (a, c, d))], np.uint32)
    return pos, idx


def test_axis_aligned_rays_replay(gpu_renderer):
    """Rays with exact-zero direction components (1/d = inf in the reference's slab test) through
    an axis-aligned cube whose faces lie on the origin's planes and an icosphere, replayed
    through binding 1: the BVH's culling (finite culling reciprocals, tests/DESIGN §4.5) must
    keep every triangle the reference accepts.  Kernel vs oracle, counters exact."""
    pos, idx = _cube()
    ipos, iidx = S.icosphere(3)
    b = S.SceneBuilder()
    b.add_mesh(pos, idx, S.ICE_MAT, scale=(1.0, 1.0, 1.0), translation=(1.0, 1.0, -4.0), normal_interp=0)
    b.add_mesh(ipos, iidx, S.GLASS_MESH_MAT, scale=(1.5, 1.5, 1.5), translation=(0.0, 0.0, -9.0), normal_interp=1)
    tris, models = b.arrays()
    b.close()
    W, H = 48, 32
    sc = S.Scene("axis", S.make_ubo(), tris, models, S.cached_envmap(*SMALL_ENV), W, H, 6,
                 flags=T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_SPHERES)
    rng = np.random.default_rng(11)
    rays = np.zeros(W * H, T.RAY)
    comps = np.array([0.0, 0.0, 0.0, -0.0, 0.25, -0.25, 0.5, -0.125], np.float32)
    for i in range(W * H):
        d = np.array([rng.choice(comps), rng.choice(comps), -1.0], np.float32)
        if i % 7 == 0:
            d = np.array([0.0, 0.0, -1.0], np.float32)
        elif i % 11 == 0:
            d = np.array([0.0, -1.0, 0.0], np.float32)
        d /= np.float32(np.sqrt(np.float32(d @ d)))
        rays[i]["dir"] = (*d, 1.0)
    p = sc.params()
    gpu_renderer.upload_scene(sc)
    g8, g32, gst = gpu_renderer.draw_frame(p, rays_in=rays, want32=True, count=True)
    q = T.Params.from_buffer_copy(p)
    q.rays_in = rays.ctypes.data
    o8, o32, ost = orc.render(sc, q, want32=True)
    assert _counts(gst) == _counts(ost), (gst, ost)
    assert gst["tri_nearest"] > 0
    assert_rgba8_close(g8, o8)
    assert_float_close(g32, o32)


@pytest.mark.parametrize("far", [1e18, 1e25])
def test_far_lights_mesh_scene(gpu_renderer, far):
    """Lights so far away that shadow distance bounds are huge (1e18) or overflow to inf
    (1e25: |L - p|^2 overflows): the BVH walk must neither enter unused node slots nor
    fault, and the frame equals the oracle's (same overflow semantics)."""
    sc = S.config_c3(96, 64, env_size=SMALL_ENV)
    sc.ubo = S.make_ubo(lights=((far, far, far), (-far, far, 0.5 * far), (3.0, 50.0, -25.0)))
    _check(gpu_renderer, sc)


def test_single_leaf_bvh_tests_each_triangle_once(gpu_renderer):
    """A mesh small enough for one BVH leaf is wrapped in a root node whose second slot is
    empty (an all-NaN box, never entered): every query entering the leaf tests its triangles
    once, so the BVH's triangle-test count stays at the reference batch loop's (up to queries
    that enter the leaf's padded box but not the batch box)."""
    pos = np.array([[-2, -1, -10], [2, -1, -10], [2, 2, -10], [-2, 2, -10]], np.float32)
    idx = np.array([[0, 1, 2], [0, 2, 3]], np.uint32)
    b = S.SceneBuilder()
    b.add_mesh(pos, idx, S.GLASS_MESH_MAT, normal_interp=0)
    tris, models = b.arrays()
    b.close()
    sc = S.Scene("quad", S.make_ubo(), tris, models, None, 64, 48, 2, flags=T.FLAG_ROW_QUIRK)
    gpu_renderer.upload_scene(sc)
    _, _, bst = gpu_renderer.draw_frame(sc.params(), count=True)
    pw = sc.params(flags=T.FLAG_ROW_QUIRK | T.FLAG_BATCH_WALK)
    _, _, wst = gpu_renderer.draw_frame(pw, count=True)
    assert wst["tri_tests"] > 0
    assert bst["tri_tests"] <= wst["tri_tests"] * 1.05 + 8, (bst, wst)
    _check(gpu_renderer, sc)


@pytest.mark.parametrize("which", ["C2", "C3", "reference", "readme"])
def test_skipped_dark_shadow_queries_exact(gpu_renderer, golden_meshes, which):
    """A frame does not trace shadow queries whose light adds nothing lit or shadowed (zero
    diffuse and specular terms, or zero albedo weights); the counting pass traces them and adds
    their terms like the reference.  The two images are bit-identical, and the skipped
    queries are reported."""
    if which == "reference":
        sc = S.config_reference_default(golden_meshes, env_size=SMALL_ENV, width=200, height=150)
    elif which == "readme":
        sc = S.config_readme(golden_meshes, env_size=SMALL_ENV, width=200, height=150)
    else:
        sc = S.CONFIGS[which](200, 150, env_size=SMALL_ENV)
    gpu_renderer.upload_scene(sc)
    for split in (1, 0):
        gpu_renderer.set_subtree_split(split)
        c8, c32, st = gpu_renderer.draw_frame(sc.params(), want32=True, count=True)
        f8, f32, _ = gpu_renderer.draw_frame(sc.params(), want32=True)
        assert np.array_equal(c8, f8) and np.array_equal(c32, f32), split
    gpu_renderer.set_subtree_split(0)
    assert 0 < st["shadow_skipped"] < st["shadow_rays"]
    assert st["skipped_sphere_tests"] <= st["sphere_tests"] and st["skipped_tri_tests"] <= st["tri_tests"]
