"""The oracle's two restatements agree bit-for-bit: the literal one (shader.comp as written,
with the 32-entry volume stack copied into every PathSegment and the reference's 40-entry
push/pop stack) and the fast one (volume stack removed per SURVEY App. A.9, DFS as current
segment + deferred refraction children).  This is the evidence that deleting the volume
stack — which the HIP kernel also does — changes nothing."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as orc
from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

ENV = (512, 256)


def _both(sc, **kw):
    p = sc.params(**kw)
    a8, a32, ast = orc.render(sc, p, mode=orc.MODE_FAST, want32=True)
    b8, b32, bst = orc.render(sc, p, mode=orc.MODE_LITERAL, want32=True)
    assert np.array_equal(a8, b8)
    assert np.array_equal(a32.view(np.uint32), b32.view(np.uint32))  # bitwise, incl. signed zeros
    assert ast == bst
    return ast


@pytest.mark.parametrize("depth", [1, 2, 4, 7, 20])
def test_spheres_envmap(depth):
    sc = S.config_c2(80, 60, env_size=ENV)
    sc.max_depth = depth
    _both(sc)


def test_checker_c1():
    _both(S.config_c1(96, 72))


def test_mesh_c3():
    _both(S.config_c3(96, 54, env_size=ENV))


def test_reference_default_scene(golden_meshes):
    sc = S.config_reference_default(golden_meshes, env_size=ENV, width=48, height=36)
    st = _both(sc)
    assert st["tri_nearest"] > 0 and st["secondary_rays"] > 0


def test_repeated_material_is_still_air_incident():
    """Push() with a material equal to air_material (shader.comp:85) still yields
    incident = air, outgoing = material (App. A.9 step 5): a sphere made of 'air' with
    refraction weight renders identically in both modes."""
    air_like = S.material((0.0, 0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    glassy_air = S.material((0.0, 0.0, 0.5, 0.5), (0.0, 0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    spheres = ((S.SPHERES[0][0], air_like), (S.SPHERES[1][0], glassy_air), S.SPHERES[2], S.SPHERES[3])
    sc = S.Scene("airy", S.make_ubo(spheres=spheres), env=S.cached_envmap(*ENV), width=64, height=48,
                 max_depth=6, flags=T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_ENVMAP)
    _both(sc)


def test_jitter_and_bands():
    sc = S.config_c2(40, 30, env_size=ENV)
    sc.spp = 3
    _both(sc)
    _both(sc, band_rows=4, band_count=3, band_index=1)
