"""Committed golden renders (tests/golden/renders.npz, made by tests/golden/make_renders.py).

CPU: the oracle re-renders every golden bit-for-bit with the same ray counters (pins the
oracle build on this toolchain).  GPU: the HIP kernel, through the C-ABI, matches every golden
within the parity bar (RGBA8 +-1 LSB) with exactly the golden ray counters — the check that
does not depend on the oracle being rebuilt on the GPU box."""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_renders import cases
from tests.helpers import assert_rgba8_close
from vkcomputeshader_tinyraytracer_amd import types as T

GOLDEN = Path(__file__).resolve().parent / "golden"
META = json.loads((GOLDEN / "renders.json").read_text())
NAMES = sorted(META)


@pytest.fixture(scope="module")
def goldens():
    with np.load(GOLDEN / "renders.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def scenes():
    return cases()


def test_fixture_integrity(goldens):
    assert sorted(goldens) == NAMES
    for k in NAMES:
        img = goldens[k]
        w, h = META[k]["size"]
        assert img.shape == (h, w, 4) and img.dtype == np.uint8
        assert hashlib.sha256(img.tobytes()).hexdigest() == META[k]["sha256"]
        assert (img[..., 3] == 255).all()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(goldens, scenes, name):
    from oracle import oracle as orc

    sc, p = scenes[name]
    o8, _, st = orc.render(sc, p)
    assert {k: st[k] for k in T.Stats.EXACT_WALK} == META[name]["counts"]
    assert np.array_equal(o8, goldens[name])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_kernel_matches_golden(gpu_renderer, goldens, scenes, name):
    sc, p = scenes[name]
    gpu_renderer.upload_scene(sc)
    g8, _, st = gpu_renderer.draw_frame(p, count=True)
    want = META[name]["counts"]
    assert {k: st[k] for k in T.Stats.EXACT} == {k: want[k] for k in T.Stats.EXACT}
    assert_rgba8_close(g8, goldens[name])
    if len(sc.models):
        pw = T.Params.from_buffer_copy(p)
        pw.flags |= T.FLAG_BATCH_WALK
        w8, _, wst = gpu_renderer.draw_frame(pw, count=True)
        assert {k: wst[k] for k in T.Stats.EXACT_WALK} == want
        assert np.array_equal(w8, g8)
