"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reconstruction half of the reference's
JPEG loader, stb_image v2.22 (the reference's lib/stb_image.h, used by main.cpp:928-949 as
stbi_load(..., STBI_rgb_alpha)).  Given raw coefficient planes (from the product's host
entropy decoder, trt_jpeg_*), it applies, in stb's integer arithmetic:

  * dequantisation          data[i] *= dequant[i] in int16           (stbi__jpeg_dequantize
                             / the (short) products of stbi__jpeg_decode_block)
  * 8x8 IDCT                jidctint-derived islow IDCT, 12-bit constants, columns then rows,
                             +512 >> 10, then +65536 + (128 << 17) >> 17 and clamp
                                                                       (stbi__idct_block)
  * chroma upsampling       resample_row_1 / _v_2 / _h_2 / _hv_2 / _generic over stb's
                             near/far line walk                         (load_jpeg_image)
  * colour conversion       stbi__YCbCr_to_RGB_row (20-bit fixed point, Cb term of g
                             truncated to 16 bits), stbi__blinn_8x8 for CMYK / YCCK

It checks the product's GPU kernels (jpeg_kernel.hip) and, with the golden hashes that the
reference's own stb_image produced (tests/golden/jpeg_goldens.json), the product's entropy
decoder.  Vectorised over blocks / rows; the full 7616x3808 envmap takes a few seconds.
"""
from __future__ import annotations

import numpy as np

GRAY, YCBCR, RGB, CMYK, YCCK = range(5)


def _fx(x: float) -> int:  # stbi__f2f on the float literal
    return int(float(np.float32(x)) * 4096 + 0.5)


C = {k: _fx(v) for k, v in dict(
    a=0.5411961, b=-1.847759065, c=0.765366865, d=1.175875602, e=0.298631336, f=2.053119869,
    g=3.072711026, h=1.501321110, i=-0.899976223, j=-2.562915447, k=-1.961570560,
    l=-0.390180644).items()}


def _idct_1d(s, bias: int, shift: int):
    """s: list of 8 int32 arrays (one 1-D transform per element); returns 8 outputs."""
    i32 = np.int32
    p1 = (s[2] + s[6]) * i32(C["a"])
    t2 = p1 + s[6] * i32(C["b"])
    t3 = p1 + s[2] * i32(C["c"])
    t0 = (s[0] + s[4]) * i32(4096)
    t1 = (s[0] - s[4]) * i32(4096)
    x0, x3 = t0 + t3 + i32(bias), t0 - t3 + i32(bias)
    x1, x2 = t1 + t2 + i32(bias), t1 - t2 + i32(bias)
    u0, u1, u2, u3 = s[7], s[5], s[3], s[1]
    p3, p4, q1, q2 = u0 + u2, u1 + u3, u0 + u3, u1 + u2
    p5 = (p3 + p4) * i32(C["d"])
    u0, u1, u2, u3 = u0 * i32(C["e"]), u1 * i32(C["f"]), u2 * i32(C["g"]), u3 * i32(C["h"])
    q1 = p5 + q1 * i32(C["i"])
    q2 = p5 + q2 * i32(C["j"])
    p3 = p3 * i32(C["k"])
    p4 = p4 * i32(C["l"])
    u3 = u3 + q1 + p4
    u2 = u2 + q2 + p3
    u1 = u1 + q2 + p4
    u0 = u0 + q1 + p3
    out = [None] * 8
    out[0], out[7] = (x0 + u3) >> shift, (x0 - u3) >> shift
    out[1], out[6] = (x1 + u2) >> shift, (x1 - u2) >> shift
    out[2], out[5] = (x2 + u1) >> shift, (x2 - u1) >> shift
    out[3], out[4] = (x3 + u0) >> shift, (x3 - u0) >> shift
    return out


def idct_planes(coef: np.ndarray, quant: np.ndarray) -> np.ndarray:
    """coef (bh, bw, 8, 8) int16 raw, quant (8, 8) -> samples (bh*8, bw*8) uint8."""
    bh, bw = coef.shape[:2]
    d = (coef.astype(np.int32) * quant.astype(np.int32)).astype(np.int16).astype(np.int32)
    cols = _idct_1d([d[:, :, r, :] for r in range(8)], 512, 10)  # each (bh, bw, 8 cols)
    v = np.stack(cols, axis=2)  # (bh, bw, row, col)
    rows = _idct_1d([v[:, :, :, c] for c in range(8)], 65536 + (128 << 17), 17)  # (bh, bw, row)
    px = np.clip(np.stack(rows, axis=3), 0, 255).astype(np.uint8)  # (bh, bw, row, col)
    return px.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8)


def walk_rows(height: int, vs: int, px_h: int) -> np.ndarray:
    """stb's ystep / ypos / line0 / line1 walk: (height, 2) near, far sample rows."""
    out = np.zeros((height, 2), np.int64)
    ystep, line0, line1, ypos = vs >> 1, 0, 0, 0
    for j in range(height):
        bottom = ystep >= (vs >> 1)
        out[j] = (line1, line0) if bottom else (line0, line1)
        ystep += 1
        if ystep >= vs:
            ystep = 0
            line0 = line1
            ypos += 1
            if ypos < px_h:
                line1 += 1
    return out


def resample(samples: np.ndarray, width: int, height: int, hs: int, vs: int, px_h: int) -> np.ndarray:
    """One component at full resolution (height, width) int32, stb's row filters."""
    rows = walk_rows(height, vs, px_h)
    near = samples[rows[:, 0]].astype(np.int32)
    far = samples[rows[:, 1]].astype(np.int32)
    w = (width + hs - 1) // hs
    x = np.arange(width)
    if hs == 1 and vs == 1:
        return near[:, :width]
    if hs == 1 and vs == 2:
        return (3 * near[:, :width] + far[:, :width] + 2) >> 2
    if hs == 2 and vs == 1:
        if w == 1:
            return np.repeat(near[:, :1], width, axis=1)
        i = np.clip(x >> 1, 1, max(w - 2, 1))
        out = (3 * near[:, i] + 2 + np.where(x & 1, near[:, np.minimum(i + 1, w - 1)], near[:, i - 1])) >> 2
        out[:, x == 1] = ((3 * near[:, 0] + near[:, 1] + 2) >> 2)[:, None]
        out[:, x == 2 * w - 2] = ((3 * near[:, w - 2] + near[:, w - 1] + 2) >> 2)[:, None]
        out[:, x == 0] = near[:, :1]
        out[:, x == 2 * w - 1] = near[:, w - 1:w]
        return out
    if hs == 2 and vs == 2:
        t = 3 * near[:, :w] + far[:, :w]
        if w == 1:
            return np.repeat((t[:, :1] + 2) >> 2, width, axis=1)
        i = np.clip((x + 1) >> 1, 1, w - 1)
        ta, tb = t[:, i - 1], t[:, i]
        out = np.where(x & 1, (3 * ta + tb + 8) >> 4, (3 * tb + ta + 8) >> 4)
        out[:, x == 0] = (t[:, :1] + 2) >> 2
        out[:, x == 2 * w - 1] = (t[:, w - 1:w] + 2) >> 2
        return out
    return near[:, x // hs]


def _f2fix(x: float) -> int:  # stbi__float2fixed
    return int(np.float32(x) * np.float32(4096.0) + np.float32(0.5)) << 8


def ycbcr_to_rgb(y, cb, cr):
    i32 = np.int32
    yf = (y.astype(np.int32) << 20) + i32(1 << 19)
    cr = cr.astype(np.int32) - 128
    cb = cb.astype(np.int32) - 128
    r = yf + cr * i32(_f2fix(1.40200))
    cbg = ((cb * i32(-_f2fix(0.34414))).view(np.uint32) & np.uint32(0xFFFF0000)).view(np.int32)
    g = yf + cr * i32(-_f2fix(0.71414)) + cbg
    b = yf + cb * i32(_f2fix(1.77200))
    return [np.clip(c >> 20, 0, 255).astype(np.uint8) for c in (r, g, b)]


def blinn(x, m):
    t = x.astype(np.uint32) * m.astype(np.uint32) + 128
    return ((t + (t >> 8)) >> 8).astype(np.uint8)


def reconstruct(jf) -> np.ndarray:
    """RGBA8 (H, W, 4) of a product JpegFile (its raw coefficients) — stbi_load's output."""
    info = jf.info
    W, H = int(info.width), int(info.height)
    comps = []
    for k in range(int(info.components)):
        h, v = int(info.h[k]), int(info.v[k])
        hs, vs = int(info.hmax) // h, int(info.vmax) // v
        px_h = (H * v + int(info.vmax) - 1) // int(info.vmax)
        s = idct_planes(jf.coefficients(k), jf.quant(k))
        comps.append(resample(s, W, H, hs, vs, px_h))
    out = np.empty((H, W, 4), np.uint8)
    out[..., 3] = 255
    color = int(info.color)
    if color == GRAY:
        out[..., 0] = out[..., 1] = out[..., 2] = comps[0]
    elif color == RGB:
        for c in range(3):
            out[..., c] = comps[c]
    elif color == CMYK:
        for c in range(3):
            out[..., c] = blinn(comps[c], comps[3])
    else:
        rgb = ycbcr_to_rgb(comps[0], comps[1], comps[2])
        for c in range(3):
            out[..., c] = blinn(255 - rgb[c].astype(np.uint32), comps[3]) if color == YCCK else rgb[c]
    return out
