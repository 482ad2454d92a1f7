"""Multi-process frame tiling on the CPU (gloo, world sizes 2 and 3): row-band assignment,
the gather to rank 0 and the re-interleave give exactly the single-process frame.  The CPU
oracle stands in for the per-rank HIP render here (the GPU path is the same TiledFrame with
hip_render_fn, exercised by tests/test_gpu_dist.py)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vkcomputeshader_tinyraytracer_amd import dist as D
from vkcomputeshader_tinyraytracer_amd import types as T


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, band_rows, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as orc
        from vkcomputeshader_tinyraytracer_amd import scene as S

        sc = S.config_c2(W, H, env_size=(256, 128))
        tf = D.TiledFrame(W, H, band_rows=band_rows)
        p = D.band_params(sc.params(), band_rows, world, rank)

        def render_fn(out):
            img, _, _ = orc.render(sc, p, threads=2)
            out[: img.shape[0]] = torch.from_numpy(img)

        frame = tf.render(render_fn)
        if rank == 0:
            full, _, _ = orc.render(sc, sc.params(), threads=2)
            q.put(bool(np.array_equal(frame.numpy(), full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band_rows,W,H", [(2, 8, 64, 50), (3, 4, 40, 33), (2, 64, 32, 20)])
def test_tiled_frame_gloo(world, band_rows, W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_rows, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("H,band_rows,world", [(768, 8, 8), (100, 8, 3), (7, 8, 4), (2160, 16, 8), (1, 1, 2)])
def test_band_partition(H, band_rows, world):
    """Every image row is rendered by exactly one rank; banded output rows match trt_output_rows."""
    rows = [D.band_rows_of(H, band_rows, world, r) for r in range(world)]
    flat = sorted(sum(rows, []))
    assert flat == list(range(H))
    assert D.max_band_rows(H, band_rows, world) == max(len(r) for r in rows)
    from vkcomputeshader_tinyraytracer_amd import lib

    L = lib()
    for r in range(world):
        p = T.make_params(height=H, band_rows=band_rows, band_count=world, band_index=r)
        import ctypes

        assert L.trt_output_rows(ctypes.byref(p)) == len(rows[r])
