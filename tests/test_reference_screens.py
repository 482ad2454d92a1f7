"""The oracle pinned to the reference's own output (build container only, marker `reference`).

The reference ships lossless PNG screenshots of its Vulkan compute shader (new_feature.md,
README.md).  Each is compared, in place, with the oracle's render of the same scene as
displayed (tests/ref_screens.py: config.hpp modelList, MAX_DEPTH 20, background.jpg through the
reference's own stb_image v2.22, pow(c, 2.2) + the sRGB swapchain encode).

Measured: 99.98-99.999 % of the compared pixels within 1 LSB on every channel.
The remaining pixels (11 of 192k in the shipped frame, 51 / 2 / 5 in the glass / whisky / ice
shots, 127 of 524k in the BaseCode shot) are chaotic: moving the pixel's primary direction by a
few float32 ulps moves the oracle's value by more than 1 LSB (depth-20 refraction chains
crossing a silhouette, a TIR threshold or a shadow-ray boundary; shadow acne on the BaseCode's
spheres), which is the size of the difference between the Vulkan driver's GLSL arithmetic
(inversesqrt/normalize/division at Vulkan's relaxed precision) and the oracle's IEEE-correct
arithmetic.  The test asserts both: the agreement bar, and that every pixel off by more than
1 LSB is such a chaotic pixel.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests import ref_screens as R

pytestmark = pytest.mark.reference

# Fraction of compared pixels within 1 LSB that each shot must reach (measured: shipped
# 0.99994, three-model 0.99996, glass 0.99978, whisky 0.99999, ice 0.99998, BaseCode 0.99976).
MIN_WITHIN1 = 0.9995


@pytest.mark.parametrize("shot", R.SHOTS, ids=[s.name for s in R.SHOTS])
def test_screenshot_matches_oracle(shot):
    frame = R.oracle_frame(shot)
    screen = R.load_screen(shot)
    rep = R.register(frame, screen, shot.offset, shot)
    assert rep is not None, "screenshot does not fit the frame at its offset"
    assert rep["px"] > 100_000, rep
    assert rep["within1"] >= MIN_WITHIN1, rep
    # The registration is the best one: a 1-pixel shift is far worse.
    for dy, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
        off = (shot.offset[0] + dy, shot.offset[1] + dx)
        if shot.screen_crop != (0, 0):  # chrome-cropped: shift the screenshot window instead
            s2 = R.load_screen(R.Shot(shot.name, shot.png, shot.models, shot.offset,
                                      flags=shot.flags, screen_crop=(shot.screen_crop[0] + dy,
                                                                     shot.screen_crop[1] + dx),
                                      max_depth=shot.max_depth, rows_below=shot.rows_below,
                                      direct_only=shot.direct_only))
            alt = R.register(frame, s2, shot.offset, shot)
        else:
            alt = R.register(frame, screen, off, shot)
        if alt is not None:
            assert alt["within1"] < rep["within1"] - 0.01, (off, alt, rep)


CURRENT = [s for s in R.SHOTS if not s.direct_only]
OLDER = [s for s in R.SHOTS if s.direct_only]


def _outliers(shot):
    frame = R.oracle_frame(shot)
    screen = R.load_screen(shot)
    d, m = R.pixel_diff(frame, screen, shot.offset, shot)
    ys, xs = np.nonzero((d > 1) & m)
    assert len(ys) <= (1 - MIN_WITHIN1) * m.sum()
    for a, b in zip(ys, xs):
        yield (shot.offset[0] + int(a), shot.offset[1] + int(b)), int(d[a, b]), screen[a, b], frame


@pytest.mark.parametrize("shot", CURRENT, ids=[s.name for s in CURRENT])
def test_outliers_are_chaotic(shot):
    """shader.comp's own screenshots: every compared pixel off by more than 1 LSB changes by
    more than 1 LSB in the oracle itself when its primary direction moves by a few ulps."""
    stable = []
    for (fy, fx), dv, scr, _ in _outliers(shot):
        r = R.instability(shot, fy, fx, scr)
        if not r["unstable"]:
            stable.append(((fy, fx), dv, r))
    assert not stable, f"{len(stable)} outliers are not chaotic: {stable[:5]}"


@pytest.mark.parametrize("shot", OLDER, ids=[s.name for s in OLDER])
def test_older_shader_outliers_explained(shot):
    """The BaseCode screenshot (an older shader): every compared pixel off by more than 1 LSB
    is shadow acne of that shader (the screenshot = the direct Phong term with a light
    dropped), an edge placed a fraction of a pixel apart, or a chaotic pixel, except at most
    one pixel in 100,000 compared.  Measured (profiles/r04_reference_screens.json): 32 edges
    (tested first), 94 acne pixels on the red and ivory spheres, 1 unexplained (ivory sphere
    (356, 465), 13 LSB brighter in the screenshot)."""
    unexplained = []
    n = 0
    for (fy, fx), dv, scr, frame in _outliers(shot):
        n += 1
        if R.edge_match(frame, fy, fx, scr) or R.sphere_acne(shot, fy, fx, scr):
            continue
        if not R.instability(shot, fy, fx, scr, radius3=2)["unstable"]:
            unexplained.append(((fy, fx), dv))
    px = R.register(R.oracle_frame(shot), R.load_screen(shot), shot.offset, shot)["px"]
    assert len(unexplained) <= px // 100_000, (n, unexplained)
