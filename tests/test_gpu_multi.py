"""Multi-GPU frame tiling through the C-ABI (trt_multi_* / trt_render_multi, csrc/trt_multi.cpp):
RCCL scene broadcast, band renders, the grouped ncclSend/ncclRecv exchange of trt_band_plan and
the re-interleave kernel.  Every frame must equal trt_render of the whole frame bit for bit
(SURVEY §8(e)).

The box has one GPU, so the communicator has one rank, and by default a root renders its own
bands in place (nothing travels at one rank).  With trt_multi_set_self_gather the root's own
band groups take the path a peer's take: compact band buffers, an ncclSend / ncclRecv pair to
itself inside the group, the gather-buffer layout (slot * groups + g) * block and the
re-interleave kernel (its 16-byte path for widths that are multiples of 4, the 4-byte path for
236-pixel rows).  Band groups per rank > 1 make the one rank hold several interleaved groups, so
the re-interleave of many groups runs too."""
from __future__ import annotations

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd import scene as S
from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, MultiRenderer, unique_id

pytestmark = pytest.mark.gpu

ENV = (1024, 512)


@pytest.fixture(scope="module")
def multi():
    m = MultiRenderer([0])
    yield m
    m.close()


def _whole(renderer, sc, params=None):
    renderer.upload_scene(sc)
    img, _, st = renderer.draw_frame(params if params is not None else sc.params(), count=True)
    return img, st


def _ubos(n):
    return np.stack([S.make_ubo(cam=(0.05 * i, 0.01 * (i % 2), -0.1 * i)) for i in range(n)])


def _single_frames(renderer, sc, p, ubos):
    renderer.upload_scene(sc)
    out = []
    for u in ubos:
        renderer.update_ubo(u)
        one, _, _ = renderer.draw_frame(p)
        out.append(one)
    renderer.update_ubo(sc.ubo)
    return out


@pytest.mark.parametrize("self_gather", [False, True])
@pytest.mark.parametrize("groups,band_rows", [(1, 8), (3, 8), (4, 1), (5, 16)])
@pytest.mark.parametrize("config", ["C2", "C3"])
def test_render_multi_host_output_bit_exact(gpu_renderer, multi, config, groups, band_rows, self_gather):
    sc = S.CONFIGS[config](236, 150, env_size=ENV)  # width not a multiple of 4: scalar interleave
    want, wst = _whole(gpu_renderer, sc)
    multi.set_band_groups(groups)
    multi.set_self_gather(self_gather)
    try:
        multi.upload_scene(sc)
        out = np.zeros_like(want)
        st = multi.draw_frame(sc.params(), band_rows=band_rows, root=0, outs=[out], count=True)
    finally:
        multi.set_band_groups(1)
        multi.set_self_gather(False)
    assert np.array_equal(out, want)
    for k in ("primary_rays", "secondary_rays", "shadow_rays", "misses", "tri_nearest"):
        assert st[k] == wst[k], (k, st, wst)


@pytest.mark.parametrize("width,height", [(236, 90), (1024, 72)])
@pytest.mark.parametrize("groups,band_rows", [(1, 8), (3, 1), (3, 8), (5, 16)])
@pytest.mark.parametrize("config", ["C2", "C3"])
def test_self_gather_frame_batches(gpu_renderer, multi, config, groups, band_rows, width, height):
    """The whole exchange at one rank: 7 frames with their own cameras in batches of 3 (3 + 3 +
    1, alternating buffer slots), rotating root, every band group sent to itself over RCCL and
    re-interleaved into device outputs."""
    torch = pytest.importorskip("torch")
    sc = S.CONFIGS[config](width, height, env_size=ENV)
    p = sc.params()
    n = 7
    ubos = _ubos(n)
    want = _single_frames(gpu_renderer, sc, p, ubos)
    fb = p.height * p.width * 4
    out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    stream = torch.cuda.Stream()
    multi.set_band_groups(groups)
    multi.set_self_gather(True)
    multi.set_stream(0, stream)
    try:
        multi.upload_scene(sc)
        multi.render_frames(p, n, band_rows=band_rows, root=ROOT_ROTATE, frames_per_gather=3, outs=[out],
                            frame_stride=fb, ubos=ubos)
        stream.synchronize()
    finally:
        multi.set_stream(0, None)
        multi.set_band_groups(1)
        multi.set_self_gather(False)
    got = out.cpu().numpy()
    for i in range(n):
        assert np.array_equal(got[i], want[i]), i


@pytest.mark.parametrize("self_gather", [False, True])
def test_render_multi_frames_device_batches(gpu_renderer, multi, self_gather):
    """The pipelined frame loop: 7 frames with their own cameras, 3 frames per gather, two
    batches in flight, rotating root (one rank: always 0), device outputs."""
    torch = pytest.importorskip("torch")
    sc = S.config_c3(256, 144, env_size=ENV)
    ubos = _ubos(7)
    multi.set_band_groups(3)
    multi.set_self_gather(self_gather)
    multi.upload_scene(sc)
    p = sc.params()
    out = torch.zeros((7, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    stream = torch.cuda.Stream()
    multi.set_stream(0, stream)
    try:
        multi.render_frames(p, 7, band_rows=8, root=ROOT_ROTATE, frames_per_gather=3, outs=[out],
                            frame_stride=p.height * p.width * 4, ubos=ubos)
        stream.synchronize()
    finally:
        multi.set_stream(0, None)
        multi.set_band_groups(1)
        multi.set_self_gather(False)
    got = out.cpu().numpy()
    want = _single_frames(gpu_renderer, sc, p, ubos)
    for i in range(7):
        assert np.array_equal(got[i], want[i]), i


@pytest.mark.parametrize("self_gather", [False, True])
def test_prepared_multi_frame_list(gpu_renderer, multi, self_gather):
    """MultiRenderer.frames_call (the bench's tiled timed loop) renders what render_frames
    renders, re-issued twice (the batches keep alternating their slots)."""
    torch = pytest.importorskip("torch")
    sc = S.config_c2(160, 96, env_size=ENV)
    ubos = _ubos(5)
    multi.set_self_gather(self_gather)
    multi.upload_scene(sc)
    p = sc.params()
    fb = p.height * p.width * 4
    out = torch.zeros((5, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    multi.set_stream(0, stream)
    try:
        call = multi.frames_call(p, 5, band_rows=8, root=ROOT_ROTATE, frames_per_gather=2, outs=[out],
                                 frame_stride=fb, ubos=ubos)
        for _ in range(2):
            out.zero_()
            torch.cuda.synchronize()
            call()
            stream.synchronize()
            got = out.cpu().numpy()
            want = _single_frames(gpu_renderer, sc, p, ubos)
            for i in range(5):
                assert np.array_equal(got[i], want[i]), i
        with pytest.raises(ValueError):
            multi.frames_call(p, 5, outs=[out[:2]], frame_stride=fb, ubos=ubos)
    finally:
        multi.set_stream(0, None)
        multi.set_self_gather(False)


def test_render_multi_frames_first_batches_after_upload():
    """Batches straight after an upload with the full-size envmap: the first batch (slot 0)
    builds the envmap pair rows, and the second batch's render stream (slot 1) forked before
    that build, so the build must be complete before any other stream samples them."""
    torch = pytest.importorskip("torch")
    from vkcomputeshader_tinyraytracer_amd import Renderer

    sc = S.config_c2(320, 200)  # reference envmap size 7616 x 3808
    p = sc.params()
    with Renderer(0) as r:
        r.upload_scene(sc)
        want, _, _ = r.draw_frame(p)
    out = torch.zeros((4, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    with MultiRenderer([0]) as m:
        m.upload_scene(sc)
        m.render_frames(p, 4, band_rows=8, root=0, frames_per_gather=1, outs=[out],
                        frame_stride=p.height * p.width * 4)
        m.synchronize()
    got = out.cpu().numpy()
    for i in range(4):
        assert np.array_equal(got[i], want), i


@pytest.mark.parametrize("self_gather", [False, True])
def test_render_multi_deep_mesh_frames(gpu_renderer, multi, golden_meshes, self_gather):
    """The depth-20 shipped frame (deferred shadows: per-frame launch sequences on the in-flight
    slots, not multi-frame launches) through the tiled loop, 4 frames with their own cameras in
    batches of 2, two band groups."""
    torch = pytest.importorskip("torch")
    sc = S.config_reference_default(golden_meshes, env_size=ENV, width=160, height=120)
    p = sc.params()
    ubos = _ubos(4)
    want = _single_frames(gpu_renderer, sc, p, ubos)
    multi.set_band_groups(2)
    multi.set_self_gather(self_gather)
    multi.upload_scene(sc)
    out = torch.zeros((4, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    try:
        multi.render_frames(p, 4, band_rows=8, root=ROOT_ROTATE, frames_per_gather=2, outs=[out],
                            frame_stride=p.height * p.width * 4, ubos=ubos)
        multi.synchronize()
    finally:
        multi.set_band_groups(1)
        multi.set_self_gather(False)
    got = out.cpu().numpy()
    for i in range(4):
        assert np.array_equal(got[i], want[i]), i


def test_for_rank_communicator(gpu_renderer):
    """One-process-per-GPU form (ncclCommInitRank with an out-of-band id), world size 1."""
    sc = S.config_c2(200, 120, env_size=ENV)
    want, _ = _whole(gpu_renderer, sc)
    with MultiRenderer.for_rank(0, 1, 0, unique_id()) as m:
        assert m.ranks == 1 and m.local_count == 1
        m.upload_scene(sc)
        out = np.zeros_like(want)
        m.draw_frame(sc.params(), band_rows=8, outs=[out])
        m.set_self_gather(True)
        out2 = np.zeros_like(want)
        m.draw_frame(sc.params(), band_rows=8, outs=[out2])
    assert np.array_equal(out, want)
    assert np.array_equal(out2, want)


def test_render_multi_errors(multi):
    from vkcomputeshader_tinyraytracer_amd import TrtError, types as T

    torch = pytest.importorskip("torch")
    sc = S.config_c2(64, 48, env_size=ENV)
    multi.upload_scene(sc)
    p = sc.params()
    with pytest.raises(TrtError):
        multi.draw_frame(p, band_rows=0)
    with pytest.raises(TrtError):
        multi.draw_frame(p, root=3)
    pb = T.Params.from_buffer_copy(p)
    pb.band_rows, pb.band_count, pb.band_index = 8, 2, 0
    with pytest.raises(TrtError):
        multi.draw_frame(pb)
    with pytest.raises(TrtError):
        multi.set_band_groups(0)
    # outputs are checked before anything is written
    with pytest.raises(ValueError):
        multi.draw_frame(p, outs=[np.zeros((10, 10, 4), np.uint8)])  # too small
    with pytest.raises(ValueError):
        multi.draw_frame(p, outs=[np.zeros((48, 64, 4), np.float32)])  # wrong dtype
    small = torch.zeros((2, 48, 64, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before our streams
    with pytest.raises(ValueError):  # 3 frames do not fit 2 frames' worth of bytes
        multi.render_frames(p, 3, outs=[small], frame_stride=48 * 64 * 4)
    with pytest.raises(ValueError):
        multi.render_frames(p, 2, outs=[small], frame_stride=48 * 64 * 4, ubos=_ubos(1))
    with pytest.raises(ValueError):
        multi.render_frames(p, 1, outs=[small, small])  # more outputs than local devices


def test_failed_batch_allocation_then_retry(gpu_renderer, monkeypatch):
    """A batch-buffer allocation that fails on slot 1 after slot 0 grew (TRT_TEST_FAIL_GROW=3:
    slot-0 local, slot-0 gather, then slot-1 local fails) returns TRT_ERR_OOM; the agreement
    frees both slots on every rank, so the retry of the same shape grows and agrees again and
    renders correct frames instead of tracing into a half-grown slot."""
    torch = pytest.importorskip("torch")
    from vkcomputeshader_tinyraytracer_amd import TrtError

    sc = S.config_c2(200, 120, env_size=ENV)
    p = sc.params()
    ubos = _ubos(4)
    want = _single_frames(gpu_renderer, sc, p, ubos)
    monkeypatch.setenv("TRT_ENABLE_TEST_HOOKS", "1")
    monkeypatch.setenv("TRT_TEST_FAIL_GROW", "3")
    m = MultiRenderer([0])
    monkeypatch.delenv("TRT_TEST_FAIL_GROW")
    out = torch.zeros((4, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    try:
        m.set_self_gather(True)
        m.upload_scene(sc)
        with pytest.raises(TrtError, match="injected"):
            m.render_frames(p, 4, band_rows=8, root=0, frames_per_gather=2, outs=[out],
                            frame_stride=p.height * p.width * 4, ubos=ubos)
        m.synchronize()
        m.render_frames(p, 4, band_rows=8, root=0, frames_per_gather=2, outs=[out],
                        frame_stride=p.height * p.width * 4, ubos=ubos)
        m.synchronize()
    finally:
        m.close()
    got = out.cpu().numpy()
    for i in range(4):
        assert np.array_equal(got[i], want[i]), i


def test_failed_host_frame_allocation_then_retry(gpu_renderer, monkeypatch):
    """Host output: the frame buffer's growth (call 1) is agreed on by every rank before the
    exchange; a failure is TRT_ERR_OOM on every rank (no rank is left in a send), and the retry
    succeeds."""
    from vkcomputeshader_tinyraytracer_amd import TrtError

    sc = S.config_c3(160, 96, env_size=ENV)
    want, _ = _whole(gpu_renderer, sc)
    monkeypatch.setenv("TRT_ENABLE_TEST_HOOKS", "1")
    monkeypatch.setenv("TRT_TEST_FAIL_GROW", "1")
    m = MultiRenderer([0])
    monkeypatch.delenv("TRT_TEST_FAIL_GROW")
    try:
        m.upload_scene(sc)
        out = np.zeros_like(want)
        with pytest.raises(TrtError, match="injected"):
            m.draw_frame(sc.params(), band_rows=8, outs=[out])
        m.draw_frame(sc.params(), band_rows=8, outs=[out])
    finally:
        m.close()
    assert np.array_equal(out, want)
