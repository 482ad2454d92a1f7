"""Exactness of the kernel's cheap replacements for correctly-rounded operations.

The kernel (csrc/trt_kernel.hip) may replace an IEEE operation of the oracle by a cheaper
sequence only where the two are bit-identical over the operation's whole input domain; these
tests prove that with exact rational arithmetic (no GPU needed).
"""
from __future__ import annotations

import math
from fractions import Fraction as F

import numpy as np


def rn32(x: F) -> F:
    """Round-to-nearest-even of an exact rational to binary32 (normal range), exactly."""
    if x == 0:
        return F(0)
    sign = -1 if x < 0 else 1
    x = abs(x)
    e = math.floor(math.log2(x))
    while F(2) ** e > x:
        e -= 1
    while F(2) ** (e + 1) <= x:
        e += 1
    ulp = F(2) ** (e - 23)
    q = x / ulp
    fl = math.floor(q)
    rem = q - fl
    if rem > F(1, 2) or (rem == F(1, 2) and fl % 2 == 1):
        fl += 1
    return sign * fl * ulp


def test_rn32_matches_numpy():
    rng = np.random.default_rng(0)
    for a, b in rng.integers(1, 1 << 20, size=(200, 2)):
        assert float(rn32(F(int(a), int(b)))) == float(np.float32(a) / np.float32(b))


def test_unorm8_fma_correction_is_the_correctly_rounded_quotient():
    """unorm8(c) = fma(fma(-q, 255, c), r, q) with q = RN(c*r), r = RN(1/255) equals
    RN(c/255) — the oracle's `(float)c / 255.0f` (shader.comp texture() of an R8G8B8A8_UNORM
    texel) — for every byte value c.  Each FMA is one rounding of the exact value."""
    r = rn32(F(1, 255))
    assert float(r) == float(np.float32(1) / np.float32(255))
    for c in range(256):
        q = rn32(F(c) * r)
        rem = rn32(F(c) - q * 255)
        got = rn32(rem * r + q)
        assert got == rn32(F(c, 255)), c
    # the plain product is NOT exact (why the correction step is needed)
    c = np.arange(256, dtype=np.float32)
    assert (c * np.float32(1 / 255) != c / np.float32(255)).any()
