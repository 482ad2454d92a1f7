"""The kernel culls batches with an implicit 8-ary hierarchy of union AABBs in front of the
reference's per-batch test (shader.comp:338-339).  That is only exact if a ray that misses a
parent box can never pass the reference test of a box inside it.  With the same slab formula
and FP32 rounding this holds by monotonicity, except when 0*inf = NaN: the reference's
NaN-ignoring min/max drops a NaN axis of a flat child lying on the parent's face, while the
parent's other slab endpoint constrains.  The kernel's internal-node test therefore treats a
NaN axis as unconstrained (`node_hit` below, restated from trt_kernel.hip); leaves keep the
exact reference test.  Checked with random and adversarial rays: axis-parallel directions
(1/0 = +-inf), origins on box faces, flat boxes, touching boxes."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as orc


def node_hit(o, d, bmin, bmax) -> bool:
    """trt_kernel.hip node_hit(): slab test with NaN axes made unconstrained."""
    f32 = np.float32
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv = f32(1.0) / np.asarray(d, f32)
        t0 = (np.asarray(bmin, f32) - np.asarray(o, f32)) * inv
        t1 = (np.asarray(bmax, f32) - np.asarray(o, f32)) * inv
    nan = np.isnan(t0) | np.isnan(t1)
    tmin = np.where(nan, -np.inf, np.minimum(t0, t1))
    tmax = np.where(nan, np.inf, np.maximum(t0, t1))
    tnear, tfar = f32(tmin.max()), f32(tmax.min())
    return bool(tnear <= tfar and tfar > f32(1e-4))


def _boxes(rng, n):
    c = rng.uniform(-5, 5, size=(n, 3)).astype(np.float32)
    e = rng.uniform(0, 2, size=(n, 3)).astype(np.float32)
    e[rng.random((n, 3)) < 0.1] = 0  # flat boxes
    return c - e, c + e


@pytest.mark.parametrize("seed", range(4))
def test_parent_miss_implies_child_miss(seed):
    rng = np.random.default_rng(seed)
    lo, hi = _boxes(rng, 8)
    plo, phi = lo.min(0), hi.max(0)  # union, exact
    dirs = rng.normal(size=(400, 3)).astype(np.float32)
    dirs[rng.random((400, 3)) < 0.3] = 0  # axis-parallel components
    dirs[(dirs == 0).all(1)] = (0, 0, 1)
    signs = rng.random((400, 3)) < 0.5
    dirs = np.where((dirs == 0) & signs, np.float32(-0.0), dirs)
    origins = rng.uniform(-8, 8, size=(400, 3)).astype(np.float32)
    # adversarial: origins on faces / corners of the child and parent boxes
    pick = rng.integers(0, 8, 400)
    face = rng.integers(0, 4, (400, 3))
    cand = np.stack([lo[pick], hi[pick], np.broadcast_to(plo, lo[pick].shape), np.broadcast_to(phi, lo[pick].shape)])
    on = np.take_along_axis(cand.transpose(1, 2, 0), face[..., None], 2)[..., 0]
    use = rng.random((400, 3)) < 0.5
    origins = np.where(use, on, origins).astype(np.float32)
    bad = 0
    for o, d in zip(origins, dirs):
        if node_hit(o, d, plo, phi):
            continue
        for k in range(8):
            bad += orc.ray_aabb(o, d, lo[k], hi[k])
    assert bad == 0


def test_reference_test_alone_is_not_conservative():
    """Why node_hit needs the NaN rule: flat child on the parent's max-z face, origin on that
    plane, dz = +0 -> the reference test hits the child but misses the parent."""
    o, d = (5.79, 2.16, 4.0), (-0.96, -0.0, 0.0)
    child = ((-6.8, 1.76, 4.0), (-2.87, 4.5, 4.0))
    parent = ((-6.8, -6.44, -6.58), (5.8, 4.77, 4.0))
    assert orc.ray_aabb(o, d, *child) and not orc.ray_aabb(o, d, *parent)
    assert node_hit(o, d, *parent)
