"""Output / presentation formats: the "as displayed" sRGB variant of the RGBA8
frame (TRT_FLAG_SRGB_OUT) and the PNG / PPM frame writers of the C-ABI."""
from __future__ import annotations

import struct
import zlib

import numpy as np
import pytest

from tests.helpers import assert_rgba8_close
from vkcomputeshader_tinyraytracer_amd import TrtError, lib, scene as S, types as T, write_image


def _read_png(path) -> np.ndarray:
    """Minimal PNG reader for the writer's output (8-bit RGBA, filters 0-4), checking CRCs."""
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    i, idat, hdr = 8, b"", None
    while i < len(b):
        n, typ = struct.unpack(">I4s", b[i:i + 8])
        data = b[i + 8:i + 8 + n]
        (crc,) = struct.unpack(">I", b[i + 8 + n:i + 12 + n])
        assert crc == zlib.crc32(typ + data) & 0xFFFFFFFF, typ
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", data)
        elif typ == b"IDAT":
            idat += data
        i += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    assert (depth, ctype, interlace) == (8, 6, 0)
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    out = np.zeros((h, 4 * w), np.int32)
    for y in range(h):
        f, row = raw[y, 0], raw[y, 1:].astype(np.int32)
        prev = out[y - 1] if y else np.zeros(4 * w, np.int32)
        cur = out[y]
        for x in range(4 * w):
            a = cur[x - 4] if x >= 4 else 0
            c = prev[x - 4] if x >= 4 else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = prev[x]
            elif f == 3:
                p = (a + prev[x]) // 2
            else:
                pa, pb, pc = abs(prev[x] - c), abs(a - c), abs(a + prev[x] - 2 * c)
                p = a if pa <= pb and pa <= pc else (prev[x] if pb <= pc else c)
            cur[x] = (row[x] + p) & 0xFF
    return out.astype(np.uint8).reshape(h, w, 4)


def _read_ppm(path) -> np.ndarray:
    b = open(path, "rb").read()
    magic, w, h, mx, rest = b.split(maxsplit=4)
    assert magic == b"P6" and mx == b"255"
    return np.frombuffer(rest, np.uint8).reshape(int(h), int(w), 3)


def _frame(h=23, w=37, seed=1):
    img = np.random.default_rng(seed).integers(0, 256, (h, w, 4), dtype=np.uint8)
    img[..., 3] = 255
    return img


def test_png_round_trip(tmp_path):
    img = _frame()
    write_image(tmp_path / "f.png", img)
    assert np.array_equal(_read_png(tmp_path / "f.png"), img)


def test_ppm_round_trip(tmp_path):
    img = _frame(5, 9)
    write_image(tmp_path / "f.ppm", img)
    assert np.array_equal(_read_ppm(tmp_path / "f.ppm"), img[..., :3])


def test_writer_errors(tmp_path):
    L = lib()
    img = _frame(2, 2)
    assert L.trt_write_png(None, img.ctypes.data, 2, 2) == T.TRT_ERR_INVALID
    assert L.trt_write_ppm(str(tmp_path / "x.ppm").encode(), None, 2, 2) == T.TRT_ERR_INVALID
    assert L.trt_write_png(str(tmp_path / "x.png").encode(), img.ctypes.data, 0, 2) == T.TRT_ERR_INVALID
    assert L.trt_write_png(str(tmp_path / "no" / "dir.png").encode(), img.ctypes.data, 2, 2) == T.TRT_ERR_IO
    with pytest.raises(ValueError):
        write_image(tmp_path / "f.bmp", img)
    with pytest.raises(TrtError):
        write_image(tmp_path / "no" / "dir.png", img)


def _srgb8(g: np.ndarray) -> np.ndarray:
    g = g.astype(np.float32)
    e = np.where(g <= np.float32(0.0031308), np.float32(12.92) * g,
                 np.float32(1.055) * np.power(g, np.float32(1.0 / 2.4)) - np.float32(0.055))
    return np.floor(e.astype(np.float32) * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


def test_oracle_srgb_out_is_srgb_of_rayout():
    """The sRGB variant encodes rayOut (pow(c, 2.2)) with the IEC 61966-2-1 transfer."""
    from oracle import oracle as orc

    sc = S.config_c2(64, 48, env_size=(256, 128))
    p = sc.params()
    _, o32, _ = orc.render(sc, p, want32=True)
    p.flags |= T.FLAG_SRGB_OUT
    s8, s32, _ = orc.render(sc, p, want32=True)
    assert np.array_equal(s32, o32)  # rayOut unchanged
    want = _srgb8(o32[..., :3])
    d = np.abs(s8[..., :3].astype(int) - want.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3
    assert (s8[..., 3] == 255).all()


@pytest.mark.gpu
def test_kernel_srgb_out_matches_oracle(gpu_renderer):
    from oracle import oracle as orc

    sc = S.config_c3(160, 120, env_size=(1024, 512))
    p = sc.params()
    p.flags |= T.FLAG_SRGB_OUT
    gpu_renderer.upload_scene(sc)
    g8, _, _ = gpu_renderer.draw_frame(p)
    o8, _, _ = orc.render(sc, p)
    assert_rgba8_close(g8, o8)
