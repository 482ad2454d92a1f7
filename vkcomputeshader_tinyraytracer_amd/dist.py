"""Tiled frames over torch.distributed: the native exchange plan on a host-chosen transport.

The reference renders a frame on one GPU (single VkQueue, main.cpp:722-724).  The native
multi-GPU path (csrc/trt_multi.cpp, `MultiRenderer`) deals a frame's rows to band groups over
the ranks, traces each rank's groups with the HIP kernel and moves the compact band buffers to
each frame's root over RCCL, following the plan of `trt_band_plan` (csrc/band_plan.cpp).  This
module runs THE SAME plan — same transfers, same buffer offsets, same row mapping, all computed
by the C library — over any torch.distributed backend: the way a host with its own transport
(MPI, gloo, ...) would drive the tiled path, and the code the multi-process CPU tests (gloo,
world sizes 2-3) exercise, so the partition and exchange the bench's RCCL path executes are
checked with more than one rank.

`render_fn(frame, group, params, out)` renders one band group of one frame compactly into
`out` (a uint8 tensor view of the group's block): the HIP kernel (`hip_render_fn`) on the GPU,
or the CPU oracle in tests.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from . import types as T
from .multi import ROOT_ROTATE, band_frame_row, band_plan, frame_root


def band_rows_of(height: int, band_rows: int, world: int, rank: int) -> list[int]:
    return T.output_rows(height, band_rows, world, rank)


def max_band_rows(height: int, band_rows: int, world: int) -> int:
    return max(len(band_rows_of(height, band_rows, world, r)) for r in range(world))


def band_params(params: T.Params, band_rows: int, groups: int, g: int) -> T.Params:
    """trt_params of band group g of `groups` (the whole frame when groups == 1)."""
    p = T.Params.from_buffer_copy(params)
    if groups > 1:
        p.band_rows, p.band_count, p.band_index = band_rows, groups, g
    return p


class TiledFrames:
    """Batches of frames row-tiled over the ranks of `group` and assembled on each frame's
    root (frame_root(i, world, root): rank i % world with ROOT_ROTATE)."""

    def __init__(self, params: T.Params, band_rows: int = 8, groups_per_rank: int = 1, root: int = ROOT_ROTATE,
                 group=None, device: torch.device | None = None):
        self.collective = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.collective else 1
        self.rank = dist.get_rank(group) if self.collective else 0
        self.group, self.root = group, root
        self.params = T.Params.from_buffer_copy(params)
        self.band_rows, self.G = band_rows, groups_per_rank
        self.device = device if device is not None else torch.device("cpu")

    def render(self, render_fn: Callable[[int, int, T.Params, torch.Tensor], None], nframes: int,
               first_frame: int = 0) -> dict[int, torch.Tensor]:
        """Renders frames first_frame .. first_frame + nframes - 1; returns {frame: (H, W, 4)
        uint8 tensor} for the frames this rank roots."""
        W, H = self.params.width, self.params.height
        N, G, r = self.world, self.G, self.rank
        lay, plan = band_plan(W, H, self.band_rows, N, G, first_frame, nframes, self.root, self_gather=True)
        NG, blk = lay.groups, lay.block_bytes
        # the plan's buffer layout (abi.h trt_band_plan): batch frames ordered by root
        roots = [frame_root(first_frame + f, N, self.root) for f in range(nframes)]
        J = [roots.count(q) for q in range(N)]
        off = [sum(J[:q]) for q in range(N)]
        jth = [roots[:f].count(roots[f]) for f in range(nframes)]
        local = torch.zeros(max(lay.local_bytes, 1), dtype=torch.uint8, device=self.device)
        gather = torch.zeros(max(lay.gather_bytes, 1), dtype=torch.uint8, device=self.device)
        # 1. this rank's band groups of every frame, compactly at ((off_root + j) * G + v) * blk
        for f in range(nframes):
            for v in range(G):
                g = r * G + v
                q = band_params(self.params, self.band_rows, NG, g)
                rows = len(T.output_rows(H, q.band_rows, q.band_count, q.band_index))
                if rows:
                    o = ((off[roots[f]] + jth[f]) * G + v) * blk
                    render_fn(first_frame + f, g, q, local[o:o + rows * W * 4].view(rows, W, 4))
        # 2. the plan's transfers, one per (sender, root) (a rank's own blocks are a local copy:
        #    torch.distributed has no send-to-self)
        reqs = []
        for x in plan:
            src = local[x.src_offset:x.src_offset + x.bytes]
            if x.src == r and x.dst == r:
                gather[x.dst_offset:x.dst_offset + x.bytes].copy_(src)
            elif x.src == r:
                reqs.append(dist.isend(src.contiguous(), x.dst, group=self.group, tag=x.dst))
            elif x.dst == r:
                reqs.append(dist.irecv(gather[x.dst_offset:x.dst_offset + x.bytes], x.src, group=self.group, tag=x.dst))
        for q in reqs:
            q.wait()
        # 3. re-interleave the frames this rank roots: sender q's group v of the j-th frame at
        #    ((q * J + j) * G + v) * blk
        out: dict[int, torch.Tensor] = {}
        for f in range(nframes):
            if roots[f] != r:
                continue
            j = jth[f]
            frame = torch.empty((H, W, 4), dtype=torch.uint8, device=self.device)
            for g in range(NG):
                q = band_params(self.params, self.band_rows, NG, g)
                rows = len(T.output_rows(H, q.band_rows, q.band_count, q.band_index))
                if not rows:
                    continue
                o = (((g // G) * J[r] + j) * G + g % G) * blk
                src = gather[o:o + rows * W * 4].view(rows, W, 4)
                idx = torch.tensor([band_frame_row(k, self.band_rows, NG, g) for k in range(rows)],
                                   dtype=torch.long, device=self.device)
                frame.index_copy_(0, idx, src)
            out[first_frame + f] = frame
        return out


def hip_render_fn(renderer, ubos=None):
    """render_fn for TiledFrames backed by the HIP kernel: trt_render of the band group into a
    device staging buffer (copied into `out` when that lives on the host)."""

    def fn(frame: int, g: int, q: T.Params, out: torch.Tensor) -> None:
        if ubos is not None:
            renderer.update_ubo(ubos[frame])
        if out.is_cuda:
            renderer.draw_frame(q, out8=out)
            renderer.synchronize()
        else:
            img, _, _ = renderer.draw_frame(q)
            out.copy_(torch.from_numpy(img))

    return fn
