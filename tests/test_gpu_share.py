"""Subtree hand-off of single-frame triangle-free launches (trt_kernel.hip share_kernel): a lane
whose own pixel is done traces another pixel's refraction subtree and records its colour terms,
which the owner folds into its running sum in pop order (shader.comp:530-575).  The frame must be
the per-pixel loop's bit for bit — both outputs — for every depth the kernel serves (2..5), ragged
image sizes (edge tiles: invalid lanes start as helpers), the checker floor, the constant
background, and both the drawFrame binding (trt_render) and one-launch-per-frame loops with
frames in flight.  Run with `pytest -m gpu`."""
from __future__ import annotations

import os

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

pytestmark = pytest.mark.gpu

SMALL_ENV = (1024, 512)


def _renderer(share: int):
    import vkcomputeshader_tinyraytracer_amd as trt

    old = os.environ.get("TRT_SHARE")
    os.environ["TRT_SHARE"] = str(share)
    try:
        return trt.Renderer(0)
    finally:
        if old is None:
            os.environ.pop("TRT_SHARE", None)
        else:
            os.environ["TRT_SHARE"] = old


@pytest.fixture(scope="module")
def pair():
    on, off = _renderer(1), _renderer(0)
    yield on, off
    on.close()
    off.close()


@pytest.mark.parametrize("config,size,depth,flags", [
    ("C2", (256, 192), 4, 0), ("C2", (264, 200), 4, 0), ("C2", (1024, 768), 4, 0),
    ("C2", (200, 136), 2, 0), ("C2", (200, 136), 3, 0), ("C2", (200, 136), 5, 0),
    ("C2", (96, 64), 4, T.FLAG_CHECKER), ("C2", (96, 64), 4, -T.FLAG_ENVMAP), ("C1", (128, 64), 1, 0),
])
def test_share_frames_equal_the_per_pixel_loop(pair, config, size, depth, flags):
    on, off = pair
    sc = S.CONFIGS[config](*size) if config == "C1" else S.CONFIGS[config](*size, env_size=SMALL_ENV)
    p = sc.params()
    if config != "C1":
        p.max_depth = depth
    if flags > 0:
        p.flags |= flags
    elif flags < 0:
        p.flags &= ~(-flags)
    on.upload_scene(sc)
    off.upload_scene(sc)
    for i, u in enumerate(S.camera_path(sc.ubo, 3)):
        on.update_ubo(u)
        off.update_ubo(u)
        a8, a32, _ = on.draw_frame(p, want32=True)
        b8, b32, _ = off.draw_frame(p, want32=True)
        assert np.array_equal(a8, b8), (config, size, depth, i)
        assert np.array_equal(a32, b32), (config, size, depth, i)


@pytest.mark.parametrize("inflight", [1, 2, 4])
def test_share_one_launch_per_frame_in_flight(pair, inflight):
    """drawFrame pacing: one launch per frame on `inflight` slots (the c2_per_frame_launch leg)."""
    torch = pytest.importorskip("torch")
    on, off = pair
    sc = S.config_c2(256, 192, env_size=SMALL_ENV)
    p = sc.params()
    on.upload_scene(sc)
    off.upload_scene(sc)
    n = 9
    ubos = np.stack(S.camera_path(sc.ubo, n))
    out = torch.zeros((n, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    on.set_stream(stream)
    try:
        on.set_frame_batch(1)
        on.set_frames_in_flight(inflight)
        on.render_frames(p, out, n, ubos=ubos, frame_stride=p.height * p.width * 4)
        stream.synchronize()
    finally:
        on.set_frame_batch(0)
        on.set_frames_in_flight(0)
        on.set_stream(None)
    got = out.cpu().numpy()
    for i in range(n):
        off.update_ubo(ubos[i])
        one, _, _ = off.draw_frame(p)
        assert np.array_equal(got[i], one), i
