"""Frame tiling with the HIP kernel ("single-GPU and multi-GPU images must be
bit-identical").

* In one process: every rank's row bands (trt_params.band_*) rendered by the kernel and
  re-interleaved equal the whole-frame render bit for bit, for several world sizes, band
  heights and scenes (spheres-only and mesh/BVH).
* Two processes on the one GPU of the box (gloo for the gather, since RCCL wants one device
  per rank): TiledFrame + hip_render_fn give rank 0 exactly the single-process frame.  On an
  8-GPU node the same code runs with backend "nccl" and one device per rank (bench.py)."""
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


def _worker(rank, world, port, W, H, band_rows, q):
    import torch
    import torch.distributed as dist

    import vkcomputeshader_tinyraytracer_amd as trt

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = S.config_c2(W, H, env_size=ENV)
        r = trt.Renderer(0)
        r.upload_scene(sc)
        tf = D.TiledFrame(W, H, band_rows=band_rows)  # gloo gathers host tensors
        dev = torch.empty((tf.max_rows, W, 4), dtype=torch.uint8, device="cuda")
        fn = D.hip_render_fn(r, sc.params(), band_rows, world, rank)

        def render_fn(out):
            fn(dev)
            torch.cuda.synchronize()
            out.copy_(dev.cpu())

        frame = tf.render(render_fn)
        if rank == 0:
            full, _, _ = r.draw_frame(sc.params())
            q.put(bool(np.array_equal(frame.numpy(), full)))
        r.close()
    finally:
        dist.destroy_process_group()


def test_tiled_frame_two_processes():
    import torch.multiprocessing as mp

    W, H, world = 200, 120, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_pipelined_tiles_frames_in_flight(gpu_renderer):
    """dist.PipelinedTiles (the bench's tiled-frame leg): with two frames in flight every
    submitted frame (distinct cameras) comes out equal to the one-at-a-time render."""
    torch = pytest.importorskip("torch")
    sc = S.config_c3(160, 96, env_size=ENV)
    gpu_renderer.upload_scene(sc)
    p = sc.params()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ubos = [S.make_ubo(cam=(0.05 * i, 0.0, -0.1 * i)) for i in range(5)]

    def render(out, stream):
        gpu_renderer.set_stream(stream)
        gpu_renderer.draw_frame(p, out8=out)

    try:
        pipe = D.PipelinedTiles(p.width, p.height, 8, torch.device("cuda", 0), streams)
        got = []
        for u in ubos:
            gpu_renderer.update_ubo(u)
            img = pipe.submit(render)
            pipe.comm.synchronize()
            got.append(img.cpu().numpy().copy())
    finally:
        gpu_renderer.set_stream(None)
    for u, g in zip(ubos, got):
        gpu_renderer.update_ubo(u)
        one, _, _ = gpu_renderer.draw_frame(p)
        assert np.array_equal(g, one)
    gpu_renderer.update_ubo(sc.ubo)


def test_pipelined_tiles_deep_mesh_frame(gpu_renderer, golden_meshes):
    """PipelinedTiles alternates trt_render between two streams; on a depth-20 mesh frame the
    subtree split is active, so the two renders must not share task-queue scratch unfenced
    (each stream gets its own split slot; a slot reused from another stream waits for it)."""
    torch = pytest.importorskip("torch")
    sc = S.config_reference_default(golden_meshes, env_size=ENV, width=160, height=120)
    gpu_renderer.upload_scene(sc)
    p = sc.params()
    want, _, _ = gpu_renderer.draw_frame(p)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def render(out, stream):
        gpu_renderer.set_stream(stream)
        gpu_renderer.draw_frame(p, out8=out)

    try:
        pipe = D.PipelinedTiles(p.width, p.height, 8, torch.device("cuda", 0), streams)
        got = []
        for _ in range(6):
            img = pipe.submit(render)
            got.append(img)
            if len(got) >= 2:  # the buffer of two submits ago is reused next: read it first
                pipe.comm.synchronize()
                got[-2] = got[-2].cpu().numpy().copy()
        pipe.comm.synchronize()
        got[-1] = got[-1].cpu().numpy().copy()
    finally:
        gpu_renderer.set_stream(None)
    for g in got:
        assert np.array_equal(g, want)


def _nccl_worker(W, H, q):
    import torch
    import torch.distributed as dist

    import vkcomputeshader_tinyraytracer_amd as trt

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        sc = S.config_c3(W, H, env_size=ENV)
        r = trt.Renderer(0)
        r.upload_scene(sc)
        p = sc.params()
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]

        def render(out, stream):
            r.set_stream(stream)
            r.draw_frame(p, out8=out)

        pipe = D.PipelinedTiles(W, H, 8, torch.device("cuda", 0), streams)
        assert pipe.tf[0].collective  # the gather runs through the process group
        imgs = []
        for _ in range(3):
            img = pipe.submit(render)
            pipe.comm.synchronize()
            imgs.append(img.cpu().numpy().copy())
        r.set_stream(None)
        full, _, _ = r.draw_frame(p)
        q.put(all(np.array_equal(i, full) for i in imgs))
        r.close()
    finally:
        dist.destroy_process_group()


def test_pipelined_tiles_nccl_world1():
    """The RCCL ("nccl" backend) gather path of TiledFrame / PipelinedTiles executes at world
    size 1 (the gather is not skipped when a process group exists)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_nccl_worker, args=(200, 120, q))
    pr.start()
    pr.join(240)
    assert pr.exitcode == 0
    assert q.get(timeout=5) is True
