"""Host-side mirror of the reference's compute path, over the C-ABI.

The reference's ComputeShaderApplication drives the hot path as
  createShaderStorageBuffers() + createUniformBuffers()  -> Renderer.upload_scene()
  updateUniformBuffer()                                  -> Renderer.update_ubo()
  recordComputeCommandBuffer() + vkQueueSubmit()         -> Renderer.draw_frame()
(main.cpp:1494-1664, 2108-2205).  Output pointers may be numpy arrays (host) or torch CUDA
tensors (device, rendered in place on the context's stream).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import types as T
from ._lib import TrtError, lib
from .scene import Scene


def _is_torch_cuda(x) -> bool:
    return hasattr(x, "is_cuda") and bool(x.is_cuda)


class Renderer:
    def __init__(self, device: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        rc = self._L.trt_create(ctypes.byref(h), int(device))
        if rc != 0:
            raise TrtError(rc, f"trt_create(device={device}) failed: no usable HIP device")
        self._h = h
        self.device = device
        self.scene: Scene | None = None

    # -- errors ----------------------------------------------------------------------------
    def _check(self, rc: int):
        if rc != 0:
            raise TrtError(rc, self._L.trt_last_error(self._h).decode())

    # -- bindings --------------------------------------------------------------------------
    def upload_scene(self, scene: Scene) -> None:
        ubo = np.ascontiguousarray(scene.ubo)
        tris = np.ascontiguousarray(scene.tris, T.TRIANGLE)
        models = np.ascontiguousarray(scene.models, T.MODEL)
        env = None if scene.env is None else np.ascontiguousarray(scene.env, np.uint8)
        self._check(self._L.trt_upload_scene(
            self._h, ubo.ctypes.data, tris.ctypes.data if len(tris) else None, len(tris),
            models.ctypes.data if len(models) else None, len(models),
            env.ctypes.data if env is not None else None,
            0 if env is None else env.shape[1], 0 if env is None else env.shape[0]))
        self.scene = scene

    def update_ubo(self, ubo: np.ndarray) -> None:
        u = np.ascontiguousarray(ubo)
        self._check(self._L.trt_update_ubo(self._h, u.ctypes.data))

    def set_frames_in_flight(self, n: int) -> None:
        """Frames of render_frames that may run concurrently (trt_set_frames_in_flight; the
        reference's MAX_FRAMES_IN_FLIGHT = 2, main.cpp:45): 1..32, or 0 = auto (4; 16 for
        deferred-shadow frames)."""
        self._check(self._L.trt_set_frames_in_flight(self._h, int(n)))

    def set_frame_batch(self, n: int) -> None:
        """Frames per launch of render_frames (trt_set_frame_batch): 0 = auto (up to 64 plain
        frames per launch), 1 = one launch per frame (the reference's dispatch per frame),
        2..64."""
        self._check(self._L.trt_set_frame_batch(self._h, int(n)))

    def set_subtree_split(self, window: int) -> None:
        """trt_set_subtree_split: 0 = auto (default), 1 = off, 2..5 = depth window."""
        self._check(self._L.trt_set_subtree_split(self._h, int(window)))

    def set_deferred_shadows(self, mode: int) -> None:
        """trt_set_deferred_shadows: 0 = auto (default: mesh scenes at max_depth >= 8), 1 = off,
        2 = on."""
        self._check(self._L.trt_set_deferred_shadows(self._h, int(mode)))

    def defer_stats(self, slot: int = 0) -> dict:
        """trt_defer_stats of in-flight slot `slot` (waits for the context's stream): event
        chunks taken / shadow queries appended, pixels re-traced in place, and the slot's
        capacities."""
        out = (ctypes.c_uint64 * 5)()
        self._check(self._L.trt_defer_stats(self._h, int(slot), out))
        return {"chunks": out[0], "queries": out[1], "fallback_pixels": out[2], "chunk_cap": out[3],
                "query_cap": out[4]}

    def set_stream(self, stream) -> None:
        """`stream`: a torch.cuda.Stream (not the legacy default stream), a raw hipStream_t
        int, or None (the context's own stream)."""
        if stream is None:
            self._check(self._L.trt_set_stream(self._h, None))
            return
        s = getattr(stream, "cuda_stream", stream)
        if not s:
            raise ValueError("the legacy null stream cannot be selected; use a torch.cuda.Stream()")
        self._check(self._L.trt_set_stream(self._h, ctypes.c_void_p(s)))

    def synchronize(self) -> None:
        self._check(self._L.trt_synchronize(self._h))

    # -- frames ----------------------------------------------------------------------------
    def draw_frame(self, params: T.Params, out8=None, out32=None, rays_in=None, count: bool = False,
                   timing: bool = False, want8: bool = True, want32: bool = False):
        """Renders one frame.  With numpy/None outputs returns host arrays
        (rows, W, 4) uint8 / float32; with torch CUDA tensors renders into them in place.
        Returns (rgba8, rgba32f, stats_dict)."""
        p = T.Params.from_buffer_copy(params)
        rows = int(self._L.trt_output_rows(ctypes.byref(p)))
        if p.flags & T.FLAG_BAND_IN_PLACE:  # bands written at their frame rows: full-size outputs
            rows = p.height
        dev = _is_torch_cuda(out8) or _is_torch_cuda(out32) or _is_torch_cuda(rays_in)
        if dev:
            p.flags |= T.FLAG_DEVICE_PTRS
            for x in (out8, out32, rays_in):
                if x is not None and not _is_torch_cuda(x):
                    raise ValueError("mixing host and device pointers in one draw_frame call")
            if out8 is not None:
                assert out8.is_contiguous() and out8.numel() >= rows * p.width * 4
            if out32 is not None:
                assert out32.is_contiguous() and out32.numel() >= rows * p.width * 4
            o8 = out8.data_ptr() if out8 is not None else None
            o32 = out32.data_ptr() if out32 is not None else None
            if rays_in is not None:
                p.rays_in = rays_in.data_ptr()
        else:
            if out8 is None and want8:
                out8 = np.empty((rows, p.width, 4), np.uint8)
            if out32 is None and want32:
                out32 = np.empty((rows, p.width, 4), np.float32)
            if out8 is not None:
                assert out8.flags["C_CONTIGUOUS"] and out8.size >= rows * p.width * 4
            if out32 is not None:
                assert out32.flags["C_CONTIGUOUS"] and out32.size >= rows * p.width * 4
            o8 = out8.ctypes.data if out8 is not None else None
            o32 = out32.ctypes.data if out32 is not None else None
            if rays_in is not None:
                rays_in = np.ascontiguousarray(rays_in, T.RAY)
                assert rays_in.size >= p.width * p.height
                p.rays_in = rays_in.ctypes.data
        if count:
            p.flags |= T.FLAG_COUNT
        if timing:
            p.flags |= T.FLAG_TIMING
        st = T.Stats()
        self._check(self._L.trt_render(self._h, ctypes.byref(p), o8, o32, ctypes.byref(st)))
        return out8, out32, st.as_dict()

    def render_frames(self, params: T.Params, out8, nframes: int, ubos: np.ndarray | None = None,
                      frame_stride: int = 0, timing: bool = False, time_every: int = 1) -> int:
        """Native frame loop (trt_render_frames): `nframes` frames enqueued on the context's
        stream into the device tensor `out8` (+ i * frame_stride bytes); plain frames go out
        several per launch (set_frame_batch).

        With `timing`, launches 0, time_every, 2*time_every, ... are bracketed by HIP events;
        returns how many were (read them with frame_times / launch_frames)."""
        if not _is_torch_cuda(out8):
            raise ValueError("render_frames renders into a device (torch CUDA) tensor")
        p = T.Params.from_buffer_copy(params)
        p.flags |= T.FLAG_DEVICE_PTRS
        p.flags &= ~T.FLAG_COUNT
        if timing:
            p.flags |= T.FLAG_TIMING
        else:
            p.flags &= ~T.FLAG_TIMING
        rows = p.height if p.flags & T.FLAG_BAND_IN_PLACE else int(self._L.trt_output_rows(ctypes.byref(p)))
        need = rows * p.width * 4 + max(nframes - 1, 0) * frame_stride
        if not out8.is_contiguous() or out8.dtype.itemsize != 1 or out8.numel() < need:
            raise ValueError(f"out8 must be a contiguous uint8 tensor of >= {need} bytes")
        u = None
        if ubos is not None:
            u = np.ascontiguousarray(ubos, T.UBO)
            if u.shape[0] < nframes:
                raise ValueError(f"{u.shape[0]} UBOs for {nframes} frames")
        self._check(self._L.trt_render_frames(self._h, ctypes.byref(p), u.ctypes.data if u is not None else None,
                                              nframes, out8.data_ptr(), frame_stride, time_every))
        return int(self._L.trt_timed_launches(self._h, None, 0)) if timing else 0

    def frames_call(self, params: T.Params, out8, nframes: int, ubos: np.ndarray | None = None,
                    frame_stride: int = 0):
        """render_frames(params, out8, nframes, ubos, frame_stride) with its argument checks and
        conversions done once: returns a zero-argument callable that only enqueues the frames
        (one trt_render_frames call), for host loops that re-issue the same frame list."""
        if not _is_torch_cuda(out8):
            raise ValueError("render_frames renders into a device (torch CUDA) tensor")
        p = T.Params.from_buffer_copy(params)
        p.flags |= T.FLAG_DEVICE_PTRS
        p.flags &= ~(T.FLAG_COUNT | T.FLAG_TIMING)
        rows = p.height if p.flags & T.FLAG_BAND_IN_PLACE else int(self._L.trt_output_rows(ctypes.byref(p)))
        need = rows * p.width * 4 + max(nframes - 1, 0) * frame_stride
        if not out8.is_contiguous() or out8.dtype.itemsize != 1 or out8.numel() < need:
            raise ValueError(f"out8 must be a contiguous uint8 tensor of >= {need} bytes")
        u = None
        if ubos is not None:
            u = np.ascontiguousarray(ubos, T.UBO)
            if u.shape[0] < nframes:
                raise ValueError(f"{u.shape[0]} UBOs for {nframes} frames")
        fn, h, pp = self._L.trt_render_frames, self._h, ctypes.byref(p)
        up, op = (u.ctypes.data if u is not None else None), out8.data_ptr()
        keep = (p, u, out8)  # alive as long as the callable

        def call() -> None:
            rc = fn(h, pp, up, nframes, op, frame_stride, 0)
            if rc:
                self._check(rc)
        call.keep = keep
        return call

    def frame_times(self, n: int) -> np.ndarray:
        """Device ms per frame of each of the first n timed launches (span / frames traced)."""
        ms = (ctypes.c_float * n)()
        self._check(self._L.trt_frame_times(self._h, ms, n))
        return np.frombuffer(ms, np.float32).copy()

    def launch_frames(self) -> np.ndarray:
        """Frames traced by each launch timed by the last timed render_frames call."""
        n = int(self._L.trt_timed_launches(self._h, None, 0))
        out = (ctypes.c_uint32 * max(n, 1))()
        self._L.trt_timed_launches(self._h, out, n)
        return np.frombuffer(out, np.uint32)[:n].copy()

    # -- envmap JPEG -----------------------------------------------------------
    def decode_jpeg(self, jpeg, out=None):
        """stbi_load(..., STBI_rgb_alpha) of a JPEG (bytes, path or JpegFile): host entropy
        decode + GPU reconstruction.  Returns an (H, W, 4) uint8 numpy array, or renders into
        `out` when it is a torch CUDA tensor."""
        from .jpeg import JpegFile

        jf = jpeg if isinstance(jpeg, JpegFile) else JpegFile(jpeg)
        h, w = jf.shape
        if _is_torch_cuda(out):
            assert out.is_contiguous() and out.numel() >= h * w * 4
            self._check(self._L.trt_jpeg_decode(self._h, jf.handle, out.data_ptr(), T.FLAG_DEVICE_PTRS))
            return out
        img = np.empty((h, w, 4), np.uint8)
        self._check(self._L.trt_jpeg_decode(self._h, jf.handle, img.ctypes.data, 0))
        return img

    def upload_envmap_jpeg(self, data) -> None:
        """Binding 4 from JPEG bytes or a path (after upload_scene)."""
        if isinstance(data, (str, os.PathLike)):
            with open(data, "rb") as f:
                data = f.read()
        buf = bytes(data)
        self._check(self._L.trt_upload_envmap_jpeg(self._h, buf, len(buf)))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.trt_destroy(self._h)
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


def render(scene: Scene, device: int = 0, **kw):
    """One-shot convenience: upload + one frame with the scene's own settings."""
    with Renderer(device) as r:
        r.upload_scene(scene)
        return r.draw_frame(scene.params(), **kw)


def write_image(path, rgba8) -> None:
    """Writes an (H, W, 4) uint8 frame (numpy, or a torch tensor) as .png or .ppm through the
    C-ABI writers (trt_write_png / trt_write_ppm)."""
    if hasattr(rgba8, "detach"):
        rgba8 = rgba8.detach().cpu().numpy()
    a = np.ascontiguousarray(rgba8, np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError(f"expected (H, W, 4) RGBA8, got {a.shape}")
    path = os.fspath(path)
    ext = os.path.splitext(path)[1].lower()
    fn = {".png": "trt_write_png", ".ppm": "trt_write_ppm"}.get(ext)
    if fn is None:
        raise ValueError(f"unsupported image extension {ext!r} (.png or .ppm)")
    rc = getattr(lib(), fn)(path.encode(), a.ctypes.data, a.shape[1], a.shape[0])
    if rc != 0:
        raise TrtError(rc, f"{fn}({path!r}) failed")
