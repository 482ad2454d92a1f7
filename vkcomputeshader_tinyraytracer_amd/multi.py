"""Host-side mirror of the multi-GPU C-ABI (include/trt/abi.h, trt_multi_* / trt_render_multi).

One frame row-tiled over the GPUs of a node and gathered over RCCL (xGMI) by the native
library (csrc/trt_multi.cpp) — the multi-GPU replacement of the reference's single-queue
dispatch (main.cpp:2108-2131, 2181-2205).

  MultiRenderer(devices=[0, 1, ...])            one process, N devices (ncclCommInitAll)
  MultiRenderer.for_rank(dev, nranks, rank, id) one process per GPU (ncclCommInitRank); every
                                                rank passes the id of unique_id() made on
                                                one rank (exchange it with torch.distributed)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import types as T
from ._lib import TrtError, lib
from .scene import Scene

ROOT_ROTATE = -1  # TRT_ROOT_ROTATE
ID_BYTES = 128  # TRT_MULTI_ID_BYTES


def frame_root(frame: int, nranks: int, root: int) -> int:
    """trt_frame_root: the rank frame `frame` of a tiled loop is assembled on."""
    return int(lib().trt_frame_root(int(frame), int(nranks), int(root)))


def band_frame_row(k: int, band_rows: int, groups: int, g: int) -> int:
    """trt_band_frame_row: frame row of compact row k of band group g."""
    return int(lib().trt_band_frame_row(int(k), int(band_rows), int(groups), int(g)))


def band_plan(width: int, height: int, band_rows: int, nranks: int, groups_per_rank: int, first_frame: int,
              nframes: int, root: int, self_gather: bool = False):
    """trt_band_plan: (layout, [transfers]) of a tiled batch — the exact exchange
    trt_render_multi_frames runs over RCCL (host arithmetic, no GPU)."""
    L = lib()
    lay = T.BandLayout()
    n = ctypes.c_uint32()
    flags = T.PLAN_SELF_GATHER if self_gather else 0
    args = (int(width), int(height), int(band_rows), int(nranks), int(groups_per_rank), int(first_frame),
            int(nframes), int(root), flags)
    rc = L.trt_band_plan(*args, ctypes.byref(lay), None, 0, ctypes.byref(n))
    if rc != 0:
        raise TrtError(rc, f"trt_band_plan{args} failed")
    xs = (T.BandXfer * max(n.value, 1))()
    rc = L.trt_band_plan(*args, ctypes.byref(lay), xs, n.value, ctypes.byref(n))
    if rc != 0:
        raise TrtError(rc, f"trt_band_plan{args} failed")
    return lay, [xs[i] for i in range(n.value)]


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * ID_BYTES)()
    rc = lib().trt_multi_unique_id(buf)
    if rc != 0:
        raise TrtError(rc, "trt_multi_unique_id failed (RCCL)")
    return bytes(buf)


def _is_torch_cuda(x) -> bool:
    return hasattr(x, "is_cuda") and bool(x.is_cuda)


class MultiRenderer:
    def __init__(self, devices=(0,), _handle=None):
        self._L = lib()
        if _handle is None:
            h = ctypes.c_void_p()
            devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            rc = self._L.trt_multi_create(ctypes.byref(h), devs, len(devices))
            if rc != 0:
                raise TrtError(rc, f"trt_multi_create(devices={list(devices)}) failed")
            _handle = h
        self._h = _handle
        self.ranks = int(self._L.trt_multi_ranks(self._h))
        self.local_count = int(self._L.trt_multi_local_count(self._h))

    @classmethod
    def for_rank(cls, device: int, nranks: int, rank: int, uid: bytes) -> "MultiRenderer":
        L = lib()
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        rc = L.trt_multi_create_rank(ctypes.byref(h), int(device), int(nranks), int(rank), buf)
        if rc != 0:
            raise TrtError(rc, f"trt_multi_create_rank(device={device}, rank={rank}/{nranks}) failed")
        return cls(_handle=h)

    def _check(self, rc: int):
        if rc != 0:
            raise TrtError(rc, self._L.trt_multi_last_error(self._h).decode())

    def set_band_groups(self, groups_per_rank: int) -> None:
        self._check(self._L.trt_multi_set_band_groups(self._h, int(groups_per_rank)))

    def set_stream(self, local: int, stream) -> None:
        """The stream (torch.cuda.Stream) local device `local`'s work joins into."""
        ctx = self._L.trt_multi_context(self._h, int(local))
        s = getattr(stream, "cuda_stream", stream) if stream is not None else None
        rc = self._L.trt_set_stream(ctx, ctypes.c_void_p(s) if s else None)
        if rc != 0:
            raise TrtError(rc, "trt_set_stream failed")

    def set_subtree_split(self, window: int) -> None:
        for i in range(self.local_count):
            rc = self._L.trt_set_subtree_split(self._L.trt_multi_context(self._h, i), int(window))
            if rc != 0:
                raise TrtError(rc, "trt_set_subtree_split failed")

    def upload_scene(self, scene: Scene | None) -> None:
        """Rank 0 builds the bindings from `scene`; every rank receives them by broadcast
        (other ranks of a one-process-per-GPU run may pass None).  Collective."""
        if scene is None:
            ubo = np.ascontiguousarray(np.zeros((), T.UBO))
            self._check(self._L.trt_multi_upload_scene(self._h, ubo.ctypes.data, None, 0, None, 0, None, 0, 0))
            return
        ubo = np.ascontiguousarray(scene.ubo)
        tris = np.ascontiguousarray(scene.tris, T.TRIANGLE)
        models = np.ascontiguousarray(scene.models, T.MODEL)
        env = None if scene.env is None else np.ascontiguousarray(scene.env, np.uint8)
        self._check(self._L.trt_multi_upload_scene(
            self._h, ubo.ctypes.data, tris.ctypes.data if len(tris) else None, len(tris),
            models.ctypes.data if len(models) else None, len(models),
            env.ctypes.data if env is not None else None,
            0 if env is None else env.shape[1], 0 if env is None else env.shape[0]))

    def update_ubo(self, ubo: np.ndarray) -> None:
        u = np.ascontiguousarray(ubo)
        self._check(self._L.trt_multi_update_ubo(self._h, u.ctypes.data))

    def _outs(self, outs, need: int, device: bool):
        """The C array of output pointers, after checking every given output: contiguous uint8
        of >= `need` bytes, on the device (torch CUDA) or the host (numpy) as the call needs."""
        outs = list(outs or [])
        if len(outs) > self.local_count:
            raise ValueError(f"{len(outs)} outputs for {self.local_count} local device(s)")
        arr = (ctypes.c_void_p * self.local_count)()
        for i, o in enumerate(outs):
            if o is None:
                continue
            if _is_torch_cuda(o):
                if not device:
                    raise ValueError("mixing device and host outputs")
                ok = o.is_contiguous() and o.dtype.itemsize == 1 and o.numel() >= need
                arr[i] = o.data_ptr()
            else:
                if device or not isinstance(o, np.ndarray):
                    raise ValueError("outputs must all be torch CUDA tensors or all numpy arrays")
                ok = o.flags["C_CONTIGUOUS"] and o.dtype == np.uint8 and o.size >= need
                arr[i] = o.ctypes.data
            if not ok:
                raise ValueError(f"output {i} must be contiguous uint8 with >= {need} bytes")
        return arr

    def set_self_gather(self, on: bool) -> None:
        """trt_multi_set_self_gather: the root's own bands also travel through the gather (the
        whole exchange on a one-GPU communicator; tests)."""
        self._check(self._L.trt_multi_set_self_gather(self._h, 1 if on else 0))

    def draw_frame(self, params: T.Params, band_rows: int = 8, root: int = 0, outs=None, count: bool = False):
        """One frame gathered on rank `root`.  `outs`: one entry per local device (torch CUDA
        tensors: enqueue only; numpy arrays: synchronous; None: not the root / no output).
        Returns the stats dict (counters summed over all ranks when `count`)."""
        p = T.Params.from_buffer_copy(params)
        dev = any(_is_torch_cuda(o) for o in (outs or []) if o is not None)
        if dev:
            p.flags |= T.FLAG_DEVICE_PTRS
        else:
            p.flags &= ~T.FLAG_DEVICE_PTRS
        if count:
            p.flags |= T.FLAG_COUNT
        arr = self._outs(outs, p.width * p.height * 4, dev)
        st = T.Stats()
        self._check(self._L.trt_render_multi(self._h, ctypes.byref(p), int(band_rows), int(root), arr,
                                             ctypes.byref(st)))
        return st.as_dict()

    def render_frames(self, params: T.Params, nframes: int, band_rows: int = 8, root: int = 0,
                      frames_per_gather: int = 1, outs=None, frame_stride: int = 0, ubos=None) -> None:
        """trt_render_multi_frames into device tensors (enqueue only).  Frame i lands on rank
        frame_root(i, ranks, root) at outs[local index] + i * frame_stride bytes."""
        p = T.Params.from_buffer_copy(params)
        p.flags |= T.FLAG_DEVICE_PTRS
        p.flags &= ~(T.FLAG_COUNT | T.FLAG_TIMING)
        if frame_stride < 0 or frame_stride % 4:
            raise ValueError("frame_stride must be a non-negative multiple of 4")
        need = p.width * p.height * 4 + max(int(nframes) - 1, 0) * int(frame_stride)
        arr = self._outs(outs, need, True)
        u = None
        if ubos is not None:
            u = np.ascontiguousarray(ubos, T.UBO)
            if u.shape[0] < nframes:
                raise ValueError(f"{u.shape[0]} UBOs for {nframes} frames")
        self._check(self._L.trt_render_multi_frames(
            self._h, ctypes.byref(p), u.ctypes.data if u is not None else None, int(nframes), int(band_rows),
            int(root), int(frames_per_gather), arr, int(frame_stride)))

    def frames_call(self, params: T.Params, nframes: int, band_rows: int = 8, root: int = 0,
                    frames_per_gather: int = 1, outs=None, frame_stride: int = 0, ubos=None):
        """render_frames(...) with its checks and conversions done once: a zero-argument callable
        that only enqueues the frames (one trt_render_multi_frames call), for host loops that
        re-issue the same frame list (every rank must issue it the same number of times)."""
        p = T.Params.from_buffer_copy(params)
        p.flags |= T.FLAG_DEVICE_PTRS
        p.flags &= ~(T.FLAG_COUNT | T.FLAG_TIMING)
        if frame_stride < 0 or frame_stride % 4:
            raise ValueError("frame_stride must be a non-negative multiple of 4")
        need = p.width * p.height * 4 + max(int(nframes) - 1, 0) * int(frame_stride)
        arr = self._outs(outs, need, True)
        u = None
        if ubos is not None:
            u = np.ascontiguousarray(ubos, T.UBO)
            if u.shape[0] < nframes:
                raise ValueError(f"{u.shape[0]} UBOs for {nframes} frames")
        fn, h, pp = self._L.trt_render_multi_frames, self._h, ctypes.byref(p)
        args = (u.ctypes.data if u is not None else None, int(nframes), int(band_rows), int(root),
                int(frames_per_gather), arr, int(frame_stride))
        keep = (p, u, arr, list(outs or []))

        def call() -> None:
            rc = fn(h, pp, *args)
            if rc:
                self._check(rc)
        call.keep = keep
        return call

    def synchronize(self) -> None:
        self._check(self._L.trt_multi_synchronize(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.trt_multi_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
