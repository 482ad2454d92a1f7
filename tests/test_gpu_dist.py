"""Frame tiling with the HIP kernel ("single-GPU and multi-GPU images must be
bit-identical").

* In one process: every rank's row bands (trt_params.band_*) rendered by the kernel and
  re-interleaved equal the whole-frame render bit for bit, for several world sizes, band
  heights and scenes (spheres-only and mesh/BVH).
* Two and three processes on the one GPU of the box: dist.TiledFrames runs the native exchange
  plan (trt_band_plan, the transfers trt_multi.cpp issues over RCCL) with gloo as transport
  (RCCL wants one device per rank), the HIP kernel rendering each rank's band groups; every
  frame lands on its rotating root equal to the single-process frame."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd import dist as D
from vkcomputeshader_tinyraytracer_amd import scene as S
from vkcomputeshader_tinyraytracer_amd import types as T

pytestmark = pytest.mark.gpu

ENV = (1024, 512)


def _assemble(renderer, sc, world, band_rows):
    p0 = sc.params()
    frame = np.zeros((p0.height, p0.width, 4), np.uint8)
    seen = np.zeros(p0.height, np.int32)
    for r in range(world):
        p = D.band_params(p0, band_rows, world, r)
        img, _, _ = renderer.draw_frame(p)
        rows = D.band_rows_of(p0.height, band_rows, world, r)
        assert img.shape[0] == len(rows)
        frame[rows] = img
        seen[rows] += 1
    assert (seen == 1).all()
    return frame


@pytest.mark.parametrize("world,band_rows", [(2, 8), (3, 8), (8, 8), (8, 1), (5, 16)])
@pytest.mark.parametrize("config", ["C2", "C3"])
def test_bands_reassemble_bit_exact(gpu_renderer, config, world, band_rows):
    sc = S.CONFIGS[config](320, 200, env_size=ENV)
    gpu_renderer.upload_scene(sc)
    full, _, _ = gpu_renderer.draw_frame(sc.params())
    assert np.array_equal(_assemble(gpu_renderer, sc, world, band_rows), full)


def test_bands_counters_add_up(gpu_renderer):
    """Per-band ray counters sum to the whole frame's (the bench's whole-job ray count)."""
    sc = S.config_c3(256, 160, env_size=ENV)
    gpu_renderer.upload_scene(sc)
    _, _, whole = gpu_renderer.draw_frame(sc.params(), count=True)
    tot = dict.fromkeys(T.Stats.EXACT, 0)
    for r in range(4):
        _, _, st = gpu_renderer.draw_frame(D.band_params(sc.params(), 8, 4, r), count=True)
        for k in tot:
            tot[k] += st[k]
    assert tot == {k: whole[k] for k in T.Stats.EXACT}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, band_rows, groups, nframes, q):
    import torch
    import torch.distributed as dist

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = S.config_c3(W, H, env_size=ENV)
        ubos = np.stack([S.make_ubo(cam=(0.05 * i, 0.0, -0.1 * i)) for i in range(nframes)])
        r = trt.Renderer(0)
        r.upload_scene(sc)
        tf = D.TiledFrames(sc.params(), band_rows=band_rows, groups_per_rank=groups, root=ROOT_ROTATE)
        frames = tf.render(D.hip_render_fn(r, ubos), nframes)  # gloo moves host tensors
        ok = True
        for i, f in frames.items():
            r.update_ubo(ubos[i])
            full, _, _ = r.draw_frame(sc.params())
            ok = ok and bool(np.array_equal(f.numpy(), full))
        q.put((rank, sorted(frames), ok))
        r.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,groups", [(2, 1), (3, 2)])
def test_tiled_frames_processes(world, groups):
    import torch.multiprocessing as mp

    W, H, n = 200, 120, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, 8, groups, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(world)]
    assert sorted(i for _, fr, _ in res for i in fr) == list(range(n))
    assert all(ok for _, _, ok in res)
