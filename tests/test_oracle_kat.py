"""Known-answer vectors for the CPU oracle, derived by hand from the shader formulas
(shader.comp line refs per test).  These pin the restatement: the reference ships no tests
or golden data and its GLSL cannot run here."""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import oracle as orc
from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

f32 = np.float32


# ---- ray_aabb_intersect, shader.comp:197-207 ---------------------------------------------

@pytest.mark.parametrize("o,d,bmin,bmax,hit", [
    ((0, 0, 0), (0, 0, -1), (-1, -1, -3), (1, 1, -2), True),    # straight ahead (1/0 = inf slabs)
    ((0, 0, 0), (0, 0, -1), (-1, -1, 2), (1, 1, 3), False),     # box behind: tFar < eps
    ((0, 0, 0), (1, 0, 0), (-1, -1, -1), (1, 1, 1), True),      # origin inside: tFar = 1 > eps
    ((0, 0, 0), (0, 0, -1), (2, 2, -3), (3, 3, -2), False),     # laterally outside
    ((1, 0, 0), (0, 0, -1), (-1, -1, -3), (1, 1, -2), False),   # on the x = bmax plane, dx = 0: 0*inf = NaN
    ((0, 0, 0), (0, 0, -1), (-1, -1, -1e-5), (1, 1, 0), False),  # box ends before MIN_EPSILON
])
def test_aabb(o, d, bmin, bmax, hit):
    assert orc.ray_aabb(o, d, bmin, bmax) is hit


# ---- ray_triangle_intersect, shader.comp:223-270 -----------------------------------------

TRI = ((-1, -1, -5), (1, -1, -5), (0, 1, -5))


def test_triangle_hit_exact():
    # e1 = (2,0,0), e2 = (1,2,0), h = (2,-1,0), a = 4, u = 0.25, v = 0.5, t = 5 (all exact)
    h, t, n = orc.ray_triangle((0, 0, 0), (0, 0, -1), *TRI)
    assert h and t == 5.0 and n == (0.0, 0.0, 1.0)  # flat: normalize(cross(e1, e2))


def test_triangle_smooth_normal():
    n0, n1, n2 = (0, 0, 1), (1, 0, 0), (0, 1, 0)
    h, t, n = orc.ray_triangle((0, 0, 0), (0, 0, -1), *TRI, n0, n1, n2, normal_interp=1)
    # w = 1 - u - v = 0.25 -> (0.25*n0 + 0.25*n1) + 0.5*n2 = (0.25, 0.5, 0.25), normalized
    v = np.array([0.25, 0.5, 0.25], np.float32)
    inv = f32(1.0) / np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    assert h and np.array_equal(np.array(n, np.float32), v * inv)


@pytest.mark.parametrize("o,d", [
    ((0, 0, 0), (1, 0, 0)),        # parallel to the plane: a = 0
    ((0, 0, -10), (0, 0, -1)),     # triangle behind: t = -5
    ((5, 0, 0), (0, 0, -1)),       # outside: u > 1
    ((-0.9, 0.9, 0), (0, 0, -1)),  # outside: u + v > 1 side
])
def test_triangle_miss(o, d):
    assert orc.ray_triangle(o, d, *TRI)[0] is False


def test_triangle_edges_inclusive():
    assert orc.ray_triangle((-1, -1, 0), (0, 0, -1), *TRI)[0]  # through v0: u = v = 0
    assert orc.ray_triangle((0, -1, 0), (0, 0, -1), *TRI)[0]   # on edge v0-v1: v = 0


def test_triangle_absolute_parallel_threshold():
    """|a| < 1e-4 is rejected in absolute terms (shader.comp:236): a 1e-3-sized triangle hit
    head-on has a = 1e-6 and is missed."""
    tiny = ((0, 0, -5), (1e-3, 0, -5), (0, 1e-3, -5))
    assert orc.ray_triangle((1e-4, 1e-4, 0), (0, 0, -1), *tiny)[0] is False
    big = ((0, 0, -5), (1, 0, -5), (0, 1, -5))
    assert orc.ray_triangle((0.1, 0.1, 0), (0, 0, -1), *big)[0] is True


# ---- ray_sphere_intersect, shader.comp:272-285 -------------------------------------------

@pytest.mark.parametrize("o,cr,t", [
    ((0, 0, 0), (0, 0, -10, 2), 8.0),   # t0 = tca - thc
    ((0, 0, -10), (0, 0, -10, 2), 2.0),  # inside: t0 < eps -> t1
    ((0, 0, 0), (2, 0, -10, 2), 10.0),  # tangent: d2 == r2 is not rejected
    ((0, 0, 0), (3, 0, -10, 2), None),  # d2 > r2
    ((0, 0, -20), (0, 0, -10, 2), None),  # sphere behind: t1 < eps
])
def test_sphere(o, cr, t):
    h, tt = orc.ray_sphere(o, (0, 0, -1), cr)
    assert h is (t is not None)
    if t is not None:
        assert tt == t


# ---- custom_refract, shader.comp:209-221 -------------------------------------------------

def test_refract_normal_incidence():
    r = orc.custom_refract((0, 0, -1), (0, 0, 1), 1.5)
    assert np.allclose(r, (0, 0, -1), atol=1e-7)


def test_refract_snell():
    s = 1 / math.sqrt(2)
    r = orc.custom_refract((s, 0, -s), (0, 0, 1), 1.5)  # entering glass at 45 degrees
    assert abs(math.hypot(*r) - 1) < 1e-6
    assert abs(r[0] - math.sin(math.pi / 4) / 1.5) < 1e-6 and r[2] < 0


def test_refract_total_internal_reflection():
    s = 1 / math.sqrt(2)
    # leaving glass (dot(I,N) > 0) at 45 degrees > critical angle 41.8: returns vec3(0)
    assert orc.custom_refract((s, 0, s), (0, 0, 1), 1.5) == (0.0, 0.0, 0.0)
    # below the critical angle it refracts, bending away from the normal
    r = orc.custom_refract((0.5, 0, math.sqrt(0.75)), (0, 0, 1), 1.5)
    assert r != (0.0, 0.0, 0.0) and abs(r[0] - 0.75) < 1e-6


# ---- direction_to_uv + sampler, shader.comp:410-416, main.cpp:1091-1106 ---------------------

@pytest.mark.parametrize("d,uv", [
    ((1, 0, 0), (0.5, 0.5)), ((0, 0, 1), (0.75, 0.5)), ((0, 0, -1), (0.25, 0.5)),
    ((0, 1, 0), (0.5, 0.0)), ((0, -1, 0), (0.5, 1.0)), ((-1, 0, 0), (1.0, 0.5)),
])
def test_direction_to_uv(d, uv):
    got = orc.direction_to_uv(d)
    assert abs(got[0] - uv[0]) < 1e-7 and abs(got[1] - uv[1]) < 1e-7


def test_bilinear_clamp_to_edge():
    env = np.zeros((2, 2, 4), np.uint8)
    env[0, 0, :3] = (0, 0, 0)
    env[0, 1, :3] = (255, 0, 0)
    env[1, 0, :3] = (0, 255, 0)
    env[1, 1, :3] = (0, 0, 255)
    env[..., 3] = 255
    c = orc.sample_env(env, (0.5, 0.5))  # centre: equal weights
    assert np.allclose(c, (0.25, 0.25, 0.25), atol=1e-7)
    assert orc.sample_env(env, (0.0, 0.0)) == (0.0, 0.0, 0.0)  # clamped to texel (0,0)
    assert orc.sample_env(env, (1.0, 1.0)) == (0.0, 0.0, 1.0)  # clamped to texel (1,1)
    assert np.allclose(orc.sample_env(env, (0.5, 0.0)), (0.5, 0.0, 0.0), atol=1e-7)  # top row only


# ---- primary rays, main.cpp:1496-1506 --------------------------------------------------

def _expected_dir(W, H, x, row, fov=1.05):
    dx = f32((x + 0.5) - W / 2.0)
    dy = f32(-(row + 0.5) + H / 2.0)
    dz = f32(-1.0 * (H / (2.0 * math.tan(float(f32(fov)) / 2.0))))
    v = np.array([dx, dy, dz], np.float32)
    for _ in range(2):  # glm::normalize on the host, normalize() in the shader
        s = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]
        v = v * (f32(1.0) / np.sqrt(s))
    return tuple(v)


@pytest.mark.parametrize("x,y,row", [(0, 0, 0), (511, 383, 383), (1022, 5, 5), (1023, 0, 1), (1023, 767, 768)])
def test_primary_ray_row_quirk(x, y, row):
    """The last column uses the next row's dy (pix++ before pix / WIDTH, main.cpp:1501-1502)."""
    p = T.make_params(flags=T.FLAGS_REFERENCE)
    assert orc.primary_dir(p, x, y) == _expected_dir(1024, 768, x, row)


def test_primary_ray_without_quirk():
    p = T.make_params(flags=T.FLAG_FLOOR)
    assert orc.primary_dir(p, 1023, 0) == _expected_dir(1024, 768, 1023, 0)


# ---- cast_ray, shader.comp:423-583 --------------------------------------------------------

def _floor_scene(checker: bool):
    flags = T.FLAG_FLOOR | (T.FLAG_CHECKER if checker else 0)
    return S.Scene("floor", S.make_ubo(), flags=flags, max_depth=4)


def test_constant_background():
    sc = S.Scene("empty", S.make_ubo(), flags=0, max_depth=4)
    c, st = orc.cast_ray(sc, sc.params(), (0, 0, 0), (0, 0, -1))
    assert c == tuple(np.float32([0.2, 0.7, 0.8]))  # BACKGROUND_COLOR, shader.comp:77
    assert (st["primary_rays"], st["secondary_rays"], st["shadow_rays"], st["misses"]) == (1, 0, 0, 1)


def test_floor_phong_known_answer():
    """Straight down onto the plain floor: diffuse = specular = l.y per light (v = n), floor
    albedo = (2, 0) so colour = 2 * kd * sum(l.y), clamped (shader.comp:302-320, 483-507)."""
    sc = _floor_scene(checker=True)
    o, d = (0.0, 0.0, -9.0), (0.0, -1.0, 0.0)  # p = (0,-4,-9): checker cell with kd (0.3,0.2,0.1)
    c, st = orc.cast_ray(sc, sc.params(), o, d)
    p = np.array([0, -4, -9], np.float64) + np.array([0, 1e-4, 0])
    ly = sum(((np.array(L) - p) / np.linalg.norm(np.array(L) - p))[1] for L in S.LIGHTS)
    exp = np.minimum(2 * np.array([0.3, 0.2, 0.1]) * ly, 1.0)
    assert np.allclose(c, exp, rtol=1e-5)
    assert c[0] == 1.0  # red saturates and is clamped (shader.comp:582)
    assert st["shadow_rays"] == 3 and st["secondary_rays"] == 0


def test_mirror_sphere_reflection_depth():
    """A ray hitting the mirror sphere spawns one reflection child (albedo.z = 0.8)."""
    sc = S.Scene("spheres", S.make_ubo(), flags=T.FLAG_SPHERES, max_depth=2)
    d = np.array([7, 5, -18], np.float32)
    d = tuple(d / np.linalg.norm(d))
    _, st = orc.cast_ray(sc, sc.params(), (0, 0, 0), d)
    assert (st["primary_rays"], st["secondary_rays"]) == (1, 1)
    sc.max_depth = 1
    _, st = orc.cast_ray(sc, sc.params(), (0, 0, 0), d)
    assert st["secondary_rays"] == 0


def test_glass_sphere_tree():
    """Glass (albedo.z = 0.1, albedo.w = 0.8): refraction + reflection children per hit, so a
    depth-2 tree traces 2 secondaries; throughput cut (|thr|^2 < 0.001) prunes deep ones."""
    sc = S.Scene("spheres", S.make_ubo(), flags=T.FLAG_SPHERES, max_depth=2)
    d = np.array([-1, -1.5, -12], np.float32)
    d = tuple(d / np.linalg.norm(d))
    _, st = orc.cast_ray(sc, sc.params(), (0, 0, 0), d)
    assert st["secondary_rays"] == 2
    sc.max_depth = 20
    _, st20 = orc.cast_ray(sc, sc.params(), (0, 0, 0), d)
    # reflection weight 0.1 -> 3*(0.1)^2 = 0.03 ok, 3*(0.01)^2 < 0.001 pruned: bounded tree
    assert 2 < st20["secondary_rays"] < 200


def test_literal_equals_fast_single_rays():
    sc = S.config_c2(32, 24, env_size=(256, 128))
    sc.max_depth = 20
    rng = np.random.default_rng(0)
    for _ in range(200):
        d = rng.normal(size=3).astype(np.float32)
        d[2] = -abs(d[2])
        d /= np.linalg.norm(d)
        a = orc.cast_ray(sc, sc.params(), (0, 0, 0), tuple(d), orc.MODE_FAST)
        b = orc.cast_ray(sc, sc.params(), (0, 0, 0), tuple(d), orc.MODE_LITERAL)
        assert a == b
