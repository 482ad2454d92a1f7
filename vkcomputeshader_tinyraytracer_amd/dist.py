"""Frame tiling across GPUs: one process per GPU, row bands + one gather to rank 0.

The reference renders a frame on one GPU (single VkQueue, main.cpp:722-724).  Here a frame
is split into interleaved row bands (rows r with (r // band_rows) % world == rank), so the
expensive centre of the image (the glass / spheres) is spread over every rank instead of
landing on one or two contiguous blocks.  Each rank renders its bands into a compact RGBA8
buffer (trt_render with band_* params), and one collective — a gather of the equal-size
(padded) band buffers to rank 0 over RCCL (xGMI) — hands rank 0 the frame, which it
re-interleaves with one index_copy_.  The scene itself is replicated: each rank uploads the
same bindings (the broadcast of SURVEY §8e happens by construction: every rank builds the
same seeded scene).

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on the GPU, "gloo" on the
CPU for tests, where `render_fn` may be any callable returning the rank's compact bands.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from . import types as T


def band_rows_of(height: int, band_rows: int, world: int, rank: int) -> list[int]:
    return T.output_rows(height, band_rows, world, rank)


def max_band_rows(height: int, band_rows: int, world: int) -> int:
    return max(len(band_rows_of(height, band_rows, world, r)) for r in range(world))


def band_params(params: T.Params, band_rows: int, world: int, rank: int) -> T.Params:
    p = T.Params.from_buffer_copy(params)
    if world > 1:
        p.band_rows, p.band_count, p.band_index = band_rows, world, rank
    return p


class TiledFrame:
    """Renders frames tiled over the ranks of `group` and gathers them on `dst`."""

    def __init__(self, width: int, height: int, band_rows: int = 8, group=None, dst: int = 0,
                 device: torch.device | None = None):
        # with a process group the gather always runs, even at world size 1 (then it is the
        # backend's local copy), so the collective path is the one exercised at every N
        self.collective = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.collective else 1
        self.rank = dist.get_rank(group) if self.collective else 0
        self.group, self.dst = group, dst
        self.width, self.height, self.band_rows = width, height, band_rows
        self.device = device if device is not None else torch.device("cpu")
        self.max_rows = max_band_rows(height, band_rows, self.world)
        self.local = torch.zeros((self.max_rows, width, 4), dtype=torch.uint8, device=self.device)
        self.gathered = (
            [torch.empty_like(self.local) for _ in range(self.world)] if self.rank == dst else None
        )
        if self.rank == dst:
            idx = [torch.tensor(band_rows_of(height, band_rows, self.world, r), dtype=torch.long)
                   for r in range(self.world)]
            self.row_index = [i.to(self.device) for i in idx]
            self.frame = torch.empty((height, width, 4), dtype=torch.uint8, device=self.device)

    def my_rows(self) -> list[int]:
        return band_rows_of(self.height, self.band_rows, self.world, self.rank)

    def render(self, render_fn: Callable[[torch.Tensor], None]) -> torch.Tensor | None:
        """`render_fn(out)` renders this rank's compact bands into out[:len(my_rows)].  Returns
        the full (H, W, 4) frame on `dst`, None elsewhere."""
        render_fn(self.local)
        if not self.collective:
            return self.local[: self.height]
        dist.gather(self.local, self.gathered, dst=self.dst, group=self.group)
        if self.rank != self.dst:
            return None
        for r in range(self.world):
            n = len(self.row_index[r])
            if n:
                self.frame.index_copy_(0, self.row_index[r], self.gathered[r][:n])
        return self.frame


class PipelinedTiles:
    """Two TiledFrame buffers used alternately, so frame i's gather (on a communication
    stream) overlaps frame i+1's band render — the tiled analogue of the reference's two
    frames in flight (main.cpp:45, MAX_FRAMES_IN_FLIGHT = 2).  With two render streams the
    band renders of consecutive frames also overlap each other (frame i+1's tiles fill the
    GPU while frame i's slowest tiles finish).  CUDA (HIP) devices only: `render_fn(out,
    stream)` must enqueue its render of `out` on `stream`, and two of them must be able to run
    at once (trt_render into device outputs is, unless the frame uses the subtree split, whose
    scratch a context shares between its trt_render calls; trt_render_frames gives concurrent
    split frames their own slots).

    submit() returns the frame tensor rank `dst` will hold once the communication stream has
    run (None on the other ranks); that buffer is reused two submits later, so read it (on the
    communication stream, or after synchronize()) before then."""

    def __init__(self, width: int, height: int, band_rows: int, device: torch.device, render_streams,
                 group=None, dst: int = 0):
        self.tf = [TiledFrame(width, height, band_rows, group, dst, device) for _ in range(2)]
        rs = list(render_streams) if isinstance(render_streams, (list, tuple)) else [render_streams]
        self.render_streams = [rs[0], rs[-1]]
        self.comm = torch.cuda.Stream(device)
        self.rendered = [torch.cuda.Event(), torch.cuda.Event()]
        self.gathered = [None, None]
        self.i = 0

    def submit(self, render_fn: Callable[[torch.Tensor, object], None]) -> torch.Tensor | None:
        b = self.i % 2
        tf = self.tf[b]
        rs = self.render_streams[b]
        if self.gathered[b] is not None:  # the gather that last read this buffer is done
            rs.wait_event(self.gathered[b])
        render_fn(tf.local, rs)
        self.rendered[b].record(rs)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.rendered[b])
            out = tf.render(lambda _: None)
            ev = torch.cuda.Event()
            ev.record(self.comm)
            self.gathered[b] = ev
        self.i += 1
        return out


def hip_render_fn(renderer, params: T.Params, band_rows: int, world: int, rank: int):
    """render_fn for TiledFrame backed by the HIP kernel (device output pointers)."""
    p = band_params(params, band_rows, world, rank)

    def fn(out: torch.Tensor) -> None:
        renderer.draw_frame(p, out8=out)

    return fn
