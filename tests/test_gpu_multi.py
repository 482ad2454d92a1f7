"""Multi-GPU frame tiling through the C-ABI (trt_multi_* / trt_render_multi, csrc/trt_multi.cpp):
RCCL scene broadcast, band renders, grouped ncclSend/ncclRecv gather and the re-interleave
kernel.  The box has one GPU, so the communicator has one rank; band groups per rank > 1
make that rank render several interleaved band groups and gather them through RCCL to
itself, so the re-interleave of many groups is exercised.  Every frame must equal trt_render
of the whole frame bit for bit."""
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


@pytest.mark.parametrize("groups,band_rows", [(1, 8), (3, 8), (4, 1), (5, 16)])
@pytest.mark.parametrize("config", ["C2", "C3"])
def test_render_multi_host_output_bit_exact(gpu_renderer, multi, config, groups, band_rows):
    sc = S.CONFIGS[config](236, 150, env_size=ENV)  # width not a multiple of 4: scalar interleave
    want, wst = _whole(gpu_renderer, sc)
    multi.set_band_groups(groups)
    multi.upload_scene(sc)
    out = np.zeros_like(want)
    st = multi.draw_frame(sc.params(), band_rows=band_rows, root=0, outs=[out], count=True)
    assert np.array_equal(out, want)
    for k in ("primary_rays", "secondary_rays", "shadow_rays", "misses", "tri_nearest"):
        assert st[k] == wst[k], (k, st, wst)
    multi.set_band_groups(1)


def test_render_multi_frames_device_batches(gpu_renderer, multi):
    """The pipelined frame loop: 7 frames with their own cameras, 3 frames per gather, two
    batches in flight, rotating root (one rank: always 0), device outputs."""
    torch = pytest.importorskip("torch")
    sc = S.config_c3(256, 144, env_size=ENV)
    ubos = np.stack([S.make_ubo(cam=(0.05 * i, 0.0, -0.1 * i)) for i in range(7)])
    multi.set_band_groups(3)
    multi.upload_scene(sc)
    p = sc.params()
    out = torch.zeros((7, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    multi.set_stream(0, stream)
    try:
        multi.render_frames(p, 7, band_rows=8, root=ROOT_ROTATE, frames_per_gather=3, outs=[out],
                            frame_stride=p.height * p.width * 4, ubos=ubos)
        stream.synchronize()
    finally:
        multi.set_stream(0, None)
        multi.set_band_groups(1)
    got = out.cpu().numpy()
    gpu_renderer.upload_scene(sc)
    for i in range(7):
        gpu_renderer.update_ubo(ubos[i])
        one, _, _ = gpu_renderer.draw_frame(p)
        assert np.array_equal(got[i], one), i


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
    with MultiRenderer([0]) as m:
        m.upload_scene(sc)
        m.render_frames(p, 4, band_rows=8, root=0, frames_per_gather=1, outs=[out],
                        frame_stride=p.height * p.width * 4)
        m.synchronize()
    got = out.cpu().numpy()
    for i in range(4):
        assert np.array_equal(got[i], want), i


def test_render_multi_deep_mesh_frame_split_active(gpu_renderer, multi, golden_meshes):
    """Depth-20 mesh frame (the subtree split is on): consecutive batches on the two render
    streams share the context's split scratch only through its stream fences."""
    torch = pytest.importorskip("torch")
    sc = S.config_reference_default(golden_meshes, env_size=ENV, width=160, height=120)
    want, _ = _whole(gpu_renderer, sc)
    multi.set_band_groups(2)
    multi.upload_scene(sc)
    p = sc.params()
    out = torch.zeros((4, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    try:
        multi.render_frames(p, 4, band_rows=8, root=0, frames_per_gather=1, outs=[out],
                            frame_stride=p.height * p.width * 4)
        multi.synchronize()
    finally:
        multi.set_band_groups(1)
    got = out.cpu().numpy()
    for i in range(4):
        assert np.array_equal(got[i], want), i


def test_for_rank_communicator(gpu_renderer):
    """One-process-per-GPU form (ncclCommInitRank with an out-of-band id), world size 1."""
    sc = S.config_c2(200, 120, env_size=ENV)
    want, _ = _whole(gpu_renderer, sc)
    with MultiRenderer.for_rank(0, 1, 0, unique_id()) as m:
        assert m.ranks == 1 and m.local_count == 1
        m.upload_scene(sc)
        out = np.zeros_like(want)
        m.draw_frame(sc.params(), band_rows=8, outs=[out])
    assert np.array_equal(out, want)


def test_render_multi_errors(multi):
    from vkcomputeshader_tinyraytracer_amd import TrtError, types as T

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
