"""Envmap JPEG decoding over the C-ABI.

The reference loads its envmap with stb_image v2.22 — stbi_load(path, &w, &h, &n,
STBI_rgb_alpha), main.cpp:928-949 — and uploads the RGBA8 result as binding 4.  Here the
entropy decode runs on the host (JpegFile: trt_jpeg_parse) and the reconstruction on the GPU
(Renderer.decode_jpeg / Renderer.upload_envmap_jpeg: trt_jpeg_decode /
trt_upload_envmap_jpeg), producing the bytes stbi_load returns.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import TrtError, lib

GRAY, YCBCR, RGB, CMYK, YCCK = range(5)  # TRT_JPEG_*


class JpegInfo(ctypes.Structure):
    """trt_jpeg_info (abi.h)."""

    _fields_ = [
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("components", ctypes.c_uint32),
        ("progressive", ctypes.c_uint32),
        ("color", ctypes.c_int32),
        ("hmax", ctypes.c_uint32),
        ("vmax", ctypes.c_uint32),
        ("h", ctypes.c_uint32 * 4),
        ("v", ctypes.c_uint32 * 4),
        ("blocks_w", ctypes.c_uint32 * 4),
        ("blocks_h", ctypes.c_uint32 * 4),
    ]


class JpegFile:
    """A parsed (entropy-decoded) JPEG: header facts plus raw coefficient planes."""

    def __init__(self, data: bytes | bytearray | os.PathLike | str):
        if isinstance(data, (str, os.PathLike)):
            with open(data, "rb") as f:
                data = f.read()
        self._L = lib()
        h = ctypes.c_void_p()
        rc = self._L.trt_jpeg_create(ctypes.byref(h))
        if rc != 0:
            raise TrtError(rc, "trt_jpeg_create failed")
        self._h = h
        self._buf = bytes(data)
        rc = self._L.trt_jpeg_parse(self._h, self._buf, len(self._buf))
        if rc != 0:
            msg = self._L.trt_jpeg_last_error(self._h).decode()
            self.close()
            raise TrtError(rc, msg)
        self.info = JpegInfo()
        self._L.trt_jpeg_get_info(self._h, ctypes.byref(self.info))

    @property
    def handle(self):
        return self._h

    @property
    def shape(self) -> tuple[int, int]:
        return int(self.info.height), int(self.info.width)

    def coefficients(self, c: int) -> np.ndarray:
        """(blocks_h, blocks_w, 8, 8) int16 raw coefficients of component c (a copy)."""
        bh, bw = int(self.info.blocks_h[c]), int(self.info.blocks_w[c])
        ptr = self._L.trt_jpeg_coefficients(self._h, c)
        if not ptr:
            raise IndexError(c)
        a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_int16)), (bh * bw * 64,))
        return a.reshape(bh, bw, 8, 8).copy()

    def quant(self, c: int) -> np.ndarray:
        ptr = self._L.trt_jpeg_quant(self._h, c)
        if not ptr:
            raise IndexError(c)
        return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint16)), (64,)).reshape(8, 8).copy()

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.trt_jpeg_destroy(self._h)
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
