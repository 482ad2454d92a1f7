"""The tiled path's partition and exchange with more than one rank, on the CPU.

The native multi-GPU path (csrc/trt_multi.cpp) runs the exchange plan of `trt_band_plan`
(csrc/band_plan.cpp) over RCCL; dist.TiledFrames runs the same plan — the same C function,
same transfers, offsets and row mapping — over torch.distributed.  Here world sizes 2 and 3
(gloo, spawned processes) render their band groups with the CPU oracle, exchange them per the
plan and assemble every frame on its root (rotating per frame, or fixed); each frame must equal
the oracle's whole frame bit for bit.  The plan's own invariants (every row of
every frame delivered exactly once, buffers in bounds, no overlaps) are checked directly for
the 8-GPU shapes the bench uses."""
from __future__ import annotations

import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vkcomputeshader_tinyraytracer_amd import dist as D
from vkcomputeshader_tinyraytracer_amd import types as T
from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, band_frame_row, band_plan, frame_root


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, band_rows, groups, root, nframes, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as orc
        from vkcomputeshader_tinyraytracer_amd import scene as S

        sc = S.config_c2(W, H, env_size=(256, 128))
        ubos = np.stack([S.make_ubo(cam=(0.1 * i, 0.0, -0.15 * i)) for i in range(nframes)])

        def render_fn(frame, g, p, out):
            s2 = S.Scene(sc.name, ubos[frame], sc.tris, sc.models, sc.env, flags=sc.flags,
                         max_depth=sc.max_depth)
            img, _, _ = orc.render(s2, p, threads=2)
            out.copy_(torch.from_numpy(np.ascontiguousarray(img)))

        tf = D.TiledFrames(sc.params(), band_rows=band_rows, groups_per_rank=groups, root=root)
        got = {}
        # two batches, the second starting mid-loop (its roots continue the rotation)
        half = nframes // 2
        got.update(tf.render(render_fn, half, 0))
        got.update(tf.render(render_fn, nframes - half, half))
        ok = True
        for i, frame in got.items():
            assert frame_root(i, world, root) == rank
            s2 = S.Scene(sc.name, ubos[i], sc.tris, sc.models, sc.env, flags=sc.flags, max_depth=sc.max_depth)
            full, _, _ = orc.render(s2, sc.params(), threads=2)
            ok = ok and bool(np.array_equal(frame.numpy(), full))
        q.put((rank, sorted(got), ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band_rows,groups,root,W,H", [
    (2, 8, 1, ROOT_ROTATE, 64, 50),
    (3, 4, 1, ROOT_ROTATE, 40, 33),
    (3, 8, 2, 1, 48, 41),
    (2, 64, 1, 0, 32, 20),
])
def test_tiled_frames_gloo(world, band_rows, groups, root, W, H):
    nframes = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_rows, groups, root, nframes, W, H, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(world)]
    seen = sorted(i for _, frames, _ in res for i in frames)
    assert seen == list(range(nframes))  # every frame assembled exactly once, on its root
    assert all(ok for _, _, ok in res)


@pytest.mark.parametrize("H,band_rows,world", [(768, 8, 8), (100, 8, 3), (7, 8, 4), (2160, 16, 8), (1, 1, 2)])
def test_band_partition(H, band_rows, world):
    """Every image row is rendered by exactly one rank; banded output rows match trt_output_rows
    and the C row mapping."""
    rows = [D.band_rows_of(H, band_rows, world, r) for r in range(world)]
    flat = sorted(sum(rows, []))
    assert flat == list(range(H))
    assert D.max_band_rows(H, band_rows, world) == max(len(r) for r in rows)
    from vkcomputeshader_tinyraytracer_amd import lib

    L = lib()
    for r in range(world):
        p = T.make_params(height=H, band_rows=band_rows, band_count=world, band_index=r)
        assert L.trt_output_rows(ctypes.byref(p)) == len(rows[r])
        if world > 1:
            assert [band_frame_row(k, band_rows, world, r) for k in range(len(rows[r]))] == rows[r]


@pytest.mark.parametrize("W,H,B,N,G,F,root,self_gather", [
    (1024, 768, 8, 8, 1, 16, ROOT_ROTATE, False),
    (1024, 768, 8, 8, 1, 13, ROOT_ROTATE, True),
    (3840, 2160, 8, 8, 1, 1, 0, False),
    (236, 150, 16, 5, 3, 7, 2, False),
    (64, 7, 8, 4, 2, 3, ROOT_ROTATE, False),
    (1024, 768, 8, 1, 1, 4, ROOT_ROTATE, True),
])
def test_band_plan_invariants(W, H, B, N, G, F, root, self_gather):
    """The plan moves, for every frame, every non-empty band group of every other rank (and the
    root's own with self_gather) to the frame's root exactly once, in one transfer per (sender,
    root) pair whose byte ranges stay inside the buffers the layout sizes and do not overlap."""
    lay, plan = band_plan(W, H, B, N, G, 0, F, root, self_gather)
    NG = N * G
    assert lay.groups == NG
    assert lay.block_bytes == lay.max_rows * W * 4
    assert lay.local_bytes == F * G * lay.block_bytes
    rows_of = [len(T.output_rows(H, B, NG, g)) if NG > 1 else H for g in range(NG)]
    assert lay.max_rows == max(rows_of)
    roots = [frame_root(f, N, root) for f in range(F)]
    J = [roots.count(r) for r in range(N)]
    off = [sum(J[:r]) for r in range(N)]
    pairs = set()
    for x in plan:
        assert (x.src, x.dst) not in pairs  # one transfer per (sender, root)
        pairs.add((x.src, x.dst))
        assert x.src != x.dst or self_gather
        assert x.frames == J[x.dst] > 0 and x.groups == G and x.first_slot == off[x.dst]
        assert x.bytes == J[x.dst] * G * lay.block_bytes
        assert x.src_offset == off[x.dst] * G * lay.block_bytes
        assert x.dst_offset == x.src * J[x.dst] * G * lay.block_bytes
        assert x.src_offset + x.bytes <= lay.local_bytes
        assert x.dst_offset + x.bytes <= lay.gather_bytes
    # every frame's every group reaches the frame's root exactly once
    for f in range(F):
        r = roots[f]
        for g in range(NG):
            q = g // G
            moved = (q, r) in pairs
            if q == r and not self_gather:
                assert not moved
            else:
                assert moved
    # a sender's ranges for different roots, and a root's ranges from different senders, are disjoint
    for who in ("src", "dst"):
        for k in range(N):
            spans = sorted(((x.src_offset, x.bytes) if who == "src" else (x.dst_offset, x.bytes))
                           for x in plan if getattr(x, who) == k)
            for (a, n), (b, _) in zip(spans, spans[1:]):
                assert a + n <= b
    # with a rotating root every device roots ceil(F / N) frames at most
    if root == ROOT_ROTATE:
        assert lay.gather_bytes == -(-F // N) * NG * lay.block_bytes
    assert len(plan) == sum(1 for r in range(N) if J[r] for q in range(N) if q != r or self_gather)


def test_band_plan_rejects_bad_shapes():
    from vkcomputeshader_tinyraytracer_amd import TrtError

    for args in ((0, 8, 8, 2, 1, 0, 1, 0), (8, 8, 0, 2, 1, 0, 1, 0), (8, 8, 8, 2, 1, 0, 1, 2), (8, 8, 8, 0, 1, 0, 1, 0)):
        with pytest.raises(TrtError):
            band_plan(*args)
