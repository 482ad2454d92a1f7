"""Scenes: the reference's config.hpp / main.cpp scene description, the benchmark
configurations C1-C5 (BASELINE.json), and seeded synthetic inputs (envmaps, icospheres).

Reference sources mirrored here:
  * sphere materials, spheres and lights  main.cpp:125-143
  * UBO fill                              main.cpp:2165-2179 (bboxMin/Max sentinels :120-121)
  * mesh materials / transforms / list    config.hpp:10-101 (ModelInfo: geometry.hpp:48-70)
Meshes are turned into Triangle/Model records by the product's C++ scene builder
(libtrt: trt_scene_add_mesh / trt_scene_add_obj), i.e. the same code path a C++ host uses.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from . import types as T
from ._lib import TrtError, lib

FLT_MAX = np.float32(3.402823466e38)


def material(albedo, diffuse_specular, refractive) -> np.ndarray:
    m = np.zeros((), T.MATERIAL)
    m["albedo"] = albedo
    m["diffuse_specular"] = diffuse_specular
    m["refractive"] = refractive
    return m


# main.cpp:125-128
IVORY = material((0.9, 0.5, 0.1, 0.0), (0.4, 0.4, 0.3, 50.0), (1.0, 0.0, 0.0, 0.0))
GLASS = material((0.0, 0.9, 0.1, 0.8), (0.6, 0.7, 0.8, 125.0), (1.5, 0.0, 0.0, 0.0))
RED_RUBBER = material((1.4, 0.3, 0.0, 0.0), (0.3, 0.1, 0.1, 10.0), (1.0, 0.0, 0.0, 0.0))
MIRROR = material((0.0, 16.0, 0.8, 0.0), (1.0, 1.0, 1.0, 1425.0), (1.0, 0.0, 0.0, 0.0))

# main.cpp:132-137
SPHERES = (
    ((-3.0, 0.0, -16.0, 2.0), IVORY),
    ((-1.0, -1.5, -12.0, 2.0), GLASS),
    ((1.5, -0.5, -18.0, 3.0), RED_RUBBER),
    ((7.0, 5.0, -18.0, 4.0), MIRROR),
)
# main.cpp:139-143
LIGHTS = ((-20.0, 20.0, 20.0), (30.0, 50.0, -25.0), (30.0, 20.0, 30.0))

# config.hpp:10-81 mesh materials
DUCK_MAT = material((0.0, 0.5, 0.1, 0.8), (0.6, 0.7, 0.8, 125.0), (1.5, 0.0, 0.0, 0.0))
ASSCHERCUT_MAT = material((0.0, 0.5, 0.1, 0.8), (0.6, 0.7, 0.8, 125.0), (1.5, 0.0, 0.0, 0.0))
BUNNY_MAT = material((0.9, 0.5, 0.0, 0.0), (0.0522876, 0.156863, 0.117647, 10.0), (1.0, 0.0, 0.0, 0.0))
DRAGON_MAT = material((0.9, 0.1, 0.0, 0.0), (0.013072, 0.078431, 0.143791, 10.0), (1.0, 0.0, 0.0, 0.0))
VENUS_MAT = material((0.0, 10.0, 0.8, 0.0), (1.0, 1.0, 1.0, 1425.0), (1.0, 0.0, 0.0, 0.0))
FUDANLOGO_MAT = material((0.7, 0.7, 0.0, 0.0), (0.515625, 0.3984275, 0.32421875, 12.0), (1.0, 0.0, 0.0, 0.0))
GLASS_MESH_MAT = material((0.0, 0.3, 0.05, 0.9), (0.95, 0.95, 0.95, 80.0), (1.5, 0.0, 0.0, 0.0))
WHISKY_MAT = material((0.3, 0.4, 0.05, 0.7), (0.9, 0.6, 0.3, 20.0), (1.2, 0.0, 0.0, 0.0))
ICE_MAT = material((0.05, 0.4, 0.2, 0.8), (0.8, 0.85, 0.9, 20.0), (1.31, 0.0, 0.0, 0.0))


@dataclass(frozen=True)
class ModelInfo:
    """geometry.hpp:48-70 ModelInfo + Model(material, normalinterpolation)."""

    asset: str  # file name under VCSA/assets (reference) / key in the golden mesh bundle
    material: np.ndarray
    scale: tuple
    rotation: tuple  # degrees
    translation: tuple
    normal_interp: int


# config.hpp:10-93
MODEL_INFOS = {
    "duck": ModelInfo("duck.obj", DUCK_MAT, (1, 1, 1), (0, 0, 0), (0, 0, 0), 1),
    "asschercut": ModelInfo("asschercut-mesh.obj", ASSCHERCUT_MAT, (2, 2, 2), (45, 45, 0), (0.2, -2.0, -14.0), 0),
    "bunny": ModelInfo("bunny-mesh.obj", BUNNY_MAT, (1, 1, 1), (0, 0, 0), (2.5, -1.5, -5.5), 0),
    "dragon": ModelInfo("dragon-mesh.obj", DRAGON_MAT, (0.7, 0.7, 0.7), (0, 110, 0), (-2.5, -2.175, -4.45), 1),
    "venus": ModelInfo("venus-mesh.obj", VENUS_MAT, (5.5, 5.5, 5.5), (0, 0, 0), (-1.0, 2.0, -19.0), 1),
    "fudanlogo": ModelInfo("fudanlogo-mesh.obj", FUDANLOGO_MAT, (0.4, 0.4, 0.4), (90, 0, 0), (0.85, 1.95, -4.15), 0),
    "glass": ModelInfo("glass.obj", GLASS_MESH_MAT, (1, 1, 1), (0, 0, 0), (0.0, -2.0, -8.0), 1),
    "water": ModelInfo("water.obj", WHISKY_MAT, (1, 1, 1), (0, 0, 0), (0.0, -2.0, -8.0), 1),
    "ice": ModelInfo("ice.obj", ICE_MAT, (1, 1, 1), (0, 0, 0), (0.0, -2.0, -8.0), 1),
}
DEFAULT_MODEL_LIST = ("glass", "water", "ice")  # config.hpp:97-101
README_MODEL_LIST = ("asschercut", "bunny", "dragon", "venus", "fudanlogo")  # config.hpp:96


def make_ubo(cam=(0.0, 0.0, 0.0), spheres=SPHERES, lights=LIGHTS) -> np.ndarray:
    """updateUniformBuffer (main.cpp:2165-2179)."""
    u = np.zeros((), T.UBO)
    for i, (cr, mat) in enumerate(spheres):
        u[f"sphere{i}"]["center_radius"] = cr
        u[f"sphere{i}"]["material"] = mat
    for i, l in enumerate(lights):
        u[f"light{i}"] = (*l, 1.0)
    u["camPos"] = (*cam, 1.0)
    u["bboxMin"] = FLT_MAX
    u["bboxMax"] = -FLT_MAX
    return u


def camera_path(ubo: np.ndarray, n: int, speed: float = 0.02) -> np.ndarray:
    """n per-frame UBOs of the reference's interactive loop with W and D held: processInput
    (main.cpp:391-403) moves cameraPos by cameraSpeed along cameraFront (0, 0, -1) and along
    normalize(cross(cameraFront, cameraUp)) = (1, 0, 0) every frame, and updateUniformBuffer
    (main.cpp:2165-2179) writes it to the frame's UBO.  cameraSpeed = 5 / FPS in the reference;
    `speed` fixes it per frame."""
    out = np.repeat(ubo[None], n, axis=0).copy()
    base = np.array(ubo["camPos"][:3], np.float32)
    for k in range(n):
        out[k]["camPos"][:3] = base + np.float32(speed) * np.array([k, 0.0, -k], np.float32)
    return out


# ---- synthetic inputs --------------------------------------------------------------------


def _hash32(x: np.ndarray) -> np.ndarray:
    """PCG-style integer hash (uint32, vectorised)."""
    x = x.astype(np.uint32)
    state = x * np.uint32(747796405) + np.uint32(2891336453)
    word = ((state >> ((state >> np.uint32(28)) + np.uint32(4))) ^ state) * np.uint32(277803737)
    return (word >> np.uint32(22)) ^ word


def synthetic_envmap(width: int = 7616, height: int = 3808, seed: int = 0) -> np.ndarray:
    """Seeded procedural equirectangular RGBA8 envmap (H, W, 4), a stand-in with the shape of
    the reference's background.jpg (7616x3808, main.cpp:928-949): sky gradient over a darker
    ground, a longitude/latitude grid and per-texel hashed noise, so bilinear filtering sees
    texel-scale detail.  Deterministic for (width, height, seed)."""
    with np.errstate(over="ignore"):
        out = np.empty((height, width, 4), np.uint8)
        xs = np.arange(width, dtype=np.uint32)
        hx = _hash32(xs ^ np.uint32(seed * 0x9E3779B9 & 0xFFFFFFFF))
        grid_x = (xs % np.uint32(256)) < np.uint32(6)
        for y0 in range(0, height, 512):
            ys = np.arange(y0, min(height, y0 + 512), dtype=np.uint32)
            v = (ys.astype(np.float32) + 0.5) / np.float32(height)
            n = _hash32(hx[None, :] + ys[:, None] * np.uint32(0x85EBCA6B))
            noise = (n & np.uint32(31)).astype(np.int32) - 16
            sky = v[:, None] < 0.5
            t = np.abs(v - 0.5)[:, None] * 2.0
            r = np.where(sky, 120 + 100 * t, 90 - 40 * t)
            g = np.where(sky, 170 + 60 * t, 70 - 30 * t)
            b = np.where(sky, 230 - 20 * t, 50 - 20 * t)
            grid = grid_x[None, :] | ((ys % np.uint32(256)) < np.uint32(6))[:, None]
            r = np.where(grid, 250, r) + noise
            g = np.where(grid, 240, g) + ((noise * 3) >> 2)
            b = np.where(grid, 200, b) + (noise >> 1)
            sl = slice(y0, y0 + len(ys))
            out[sl, :, 0] = np.clip(r, 0, 255).astype(np.uint8)
            out[sl, :, 1] = np.clip(g, 0, 255).astype(np.uint8)
            out[sl, :, 2] = np.clip(b, 0, 255).astype(np.uint8)
            out[sl, :, 3] = 255
    return out


def icosphere(level: int) -> tuple[np.ndarray, np.ndarray]:
    """Unit icosphere: 20 * 4**level triangles (level 4 = 5,120).  Returns float32 (V,3)
    positions and uint32 (F,3) indices, deterministic."""
    t = (1.0 + 5.0**0.5) / 2.0
    verts = [
        (-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0),
        (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
        (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1),
    ]
    verts = [np.array(v, np.float64) / np.linalg.norm(v) for v in verts]
    faces = [
        (0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11),
        (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6), (7, 1, 8),
        (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9),
        (4, 9, 5), (2, 4, 11), (6, 2, 10), (8, 6, 7), (9, 8, 1),
    ]
    for _ in range(level):
        cache: dict = {}

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = verts[a] + verts[b]
                verts.append(m / np.linalg.norm(m))
                cache[key] = len(verts) - 1
            return cache[key]

        nf = []
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    return np.asarray(verts, np.float32), np.asarray(faces, np.uint32)


# ---- scene assembly ---------------------------------------------------------------------


class SceneBuilder:
    """The reference's per-model loop of createShaderStorageBuffers() (main.cpp:1533-1567),
    run by the product's C++ builder (trt_scene_*)."""

    def __init__(self, batch_size: int = 64):
        self._L = lib()
        h = ctypes.c_void_p()
        rc = self._L.trt_scene_create(ctypes.byref(h))
        if rc != 0:
            raise TrtError(rc, "trt_scene_create failed")
        self._h = h
        if batch_size != 64:
            self._check(self._L.trt_scene_set_batch_size(self._h, batch_size))

    def _check(self, rc: int):
        if rc != 0:
            raise TrtError(rc, self._L.trt_scene_last_error(self._h).decode())

    @staticmethod
    def _f3(v) -> ctypes.Array:
        return (ctypes.c_float * 3)(*[float(np.float32(x)) for x in v])

    def add_mesh(self, positions, indices, mat, scale=(1, 1, 1), rotation=(0, 0, 0),
                 translation=(0, 0, 0), normal_interp: int = 1) -> "SceneBuilder":
        pos = np.ascontiguousarray(positions, np.float32).reshape(-1, 3)
        idx = np.ascontiguousarray(indices, np.uint32).reshape(-1, 3)
        m = np.ascontiguousarray(np.asarray(mat, T.MATERIAL).reshape(()))
        self._check(self._L.trt_scene_add_mesh(
            self._h, pos.ctypes.data, pos.shape[0], idx.ctypes.data, idx.shape[0], m.ctypes.data,
            self._f3(scale), self._f3(rotation), self._f3(translation), int(normal_interp)))
        return self

    def add_obj(self, path, mat, scale=(1, 1, 1), rotation=(0, 0, 0), translation=(0, 0, 0),
                normal_interp: int = 1) -> "SceneBuilder":
        m = np.ascontiguousarray(np.asarray(mat, T.MATERIAL).reshape(()))
        self._check(self._L.trt_scene_add_obj(
            self._h, str(path).encode(), m.ctypes.data, self._f3(scale), self._f3(rotation),
            self._f3(translation), int(normal_interp)))
        return self

    def add_model(self, info: ModelInfo, positions, indices) -> "SceneBuilder":
        return self.add_mesh(positions, indices, info.material, info.scale, info.rotation,
                             info.translation, info.normal_interp)

    def arrays(self) -> tuple[np.ndarray, np.ndarray]:
        nt = self._L.trt_scene_triangle_count(self._h)
        nm = self._L.trt_scene_model_count(self._h)
        tris = np.zeros(nt, T.TRIANGLE)
        models = np.zeros(nm, T.MODEL)
        if nt:
            ctypes.memmove(tris.ctypes.data, self._L.trt_scene_triangles(self._h), nt * T.TRIANGLE.itemsize)
        if nm:
            ctypes.memmove(models.ctypes.data, self._L.trt_scene_models(self._h), nm * T.MODEL.itemsize)
        return tris, models

    def close(self):
        if self._h:
            self._L.trt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Scene:
    """Everything the reference binds for one frame (bindings 0, 4, 5, 6) plus the render
    settings of a configuration."""

    name: str
    ubo: np.ndarray
    tris: np.ndarray = field(default_factory=lambda: np.zeros(0, T.TRIANGLE))
    models: np.ndarray = field(default_factory=lambda: np.zeros(0, T.MODEL))
    env: np.ndarray | None = None  # (H, W, 4) uint8
    width: int = 1024
    height: int = 768
    max_depth: int = 20
    spp: int = 1
    flags: int = T.FLAGS_REFERENCE

    def params(self, **kw) -> T.Params:
        args = dict(width=self.width, height=self.height, max_depth=self.max_depth, spp=self.spp,
                    flags=self.flags)
        args.update(kw)
        return T.make_params(**args)


GOLDEN_MESHES = Path(__file__).resolve().parent.parent / "tests" / "golden" / "meshes.npz"


def load_golden_meshes(path: Path = GOLDEN_MESHES) -> dict:
    """Positions + triangulated indices of the reference assets as parsed by the reference's
    own tinyobjloader (tests/golden/make_goldens.py)."""
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def build_models(names, meshes: dict, batch_size: int = 64) -> tuple[np.ndarray, np.ndarray]:
    b = SceneBuilder(batch_size)
    for n in names:
        info = MODEL_INFOS[n]
        key = info.asset
        b.add_model(info, meshes[f"{key}:pos"], meshes[f"{key}:idx"])
    out = b.arrays()
    b.close()
    return out


_ENV_CACHE: dict = {}


def cached_envmap(width: int, height: int, seed: int = 0) -> np.ndarray:
    k = (width, height, seed)
    if k not in _ENV_CACHE:
        _ENV_CACHE[k] = synthetic_envmap(width, height, seed)
    return _ENV_CACHE[k]


def config_c1(width=1024, height=768) -> Scene:
    """C1: 4 spheres + checker floor, depth 1, no meshes, constant background (the CPU
    tinyraytracer reference case)."""
    return Scene("C1", make_ubo(), width=width, height=height, max_depth=1,
                 flags=T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_CHECKER | T.FLAG_ROW_QUIRK)


def config_c2(width=1024, height=768, env_size=(7616, 3808), seed=0) -> Scene:
    """C2 (headline): 4 spheres + plain floor + seeded envmap at the reference texture size,
    depth 4."""
    return Scene("C2", make_ubo(), env=cached_envmap(*env_size, seed), width=width, height=height,
                 max_depth=4, flags=T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)


def config_c3(width=1920, height=1080, env_size=(7616, 3808), level=4) -> Scene:
    """C3: spheres + one icosphere mesh (level 4 = 5,120 tris, 80 batches) in the reference's
    glass mesh material, depth 4."""
    pos, idx = icosphere(level)
    b = SceneBuilder()
    b.add_mesh(pos, idx, GLASS_MESH_MAT, scale=(1.5, 1.5, 1.5), translation=(2.5, -2.0, -10.0), normal_interp=1)
    tris, models = b.arrays()
    b.close()
    return Scene("C3", make_ubo(), tris, models, cached_envmap(*env_size), width, height, 4,
                 flags=T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)


C4_MATERIALS = (GLASS_MESH_MAT, WHISKY_MAT, ICE_MAT, BUNNY_MAT, DRAGON_MAT, FUDANLOGO_MAT, VENUS_MAT, DUCK_MAT)


def config_c4(width=3840, height=2160, env_size=(7616, 3808), n_objects=20, level=4, spp=1) -> Scene:
    """C4: ~100k triangles (20 level-4 icospheres = 102,400 tris / 1,600 batches) on a 5x4
    grid with the config.hpp mesh materials, spheres, floor, envmap, depth 4."""
    pos, idx = icosphere(level)
    b = SceneBuilder()
    for k in range(n_objects):
        gx, gz = k % 5, k // 5
        tr = (-6.0 + 3.0 * gx, -3.0 + 0.5 * (k % 3), -7.0 - 4.0 * gz)
        b.add_mesh(pos, idx, C4_MATERIALS[k % len(C4_MATERIALS)], scale=(1.0, 1.0, 1.0), translation=tr,
                   normal_interp=1 if k % 2 == 0 else 0)
    tris, models = b.arrays()
    b.close()
    return Scene("C4" if spp == 1 else "C5", make_ubo(), tris, models, cached_envmap(*env_size), width, height,
                 4, spp=spp, flags=T.FLAG_SPHERES | T.FLAG_FLOOR | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)


def config_c5(width=3840, height=2160, env_size=(7616, 3808)) -> Scene:
    """C5: C4 with 16 PCG-jittered samples per pixel (build extension)."""
    return config_c4(width, height, env_size, spp=16)


def config_reference_default(meshes: dict | None = None, env_size=(7616, 3808), width=1024, height=768) -> Scene:
    """The shipped reference frame: glass + water + ice (37,956 tris / 594 batches, config.hpp:97),
    floor on, spheres off (shader.comp:83-84), envmap background, MAX_DEPTH 20, host ray quirk."""
    meshes = meshes if meshes is not None else load_golden_meshes()
    tris, models = build_models(DEFAULT_MODEL_LIST, meshes)
    return Scene("reference", make_ubo(), tris, models, cached_envmap(*env_size), width, height, 20,
                 flags=T.FLAGS_REFERENCE)


def config_readme(meshes: dict | None = None, env_size=(7616, 3808), width=1024, height=768,
                  max_depth=20) -> Scene:
    """The README-era scene that carries the reference's only published frame rate (10-11 FPS
    on an RTX 4060 at 1024x768, README.md:334-340): asschercut + bunny + dragon + venus +
    fudanlogo (config.hpp:96; 53,877 tris / 844 batches, rotated and flat-shaded models),
    checker floor, spheres off, envmap background, MAX_DEPTH 20 (shader.comp:75).  The README
    screenshots come from an older shader state, so the published figure is context only."""
    meshes = meshes if meshes is not None else load_golden_meshes()
    tris, models = build_models(README_MODEL_LIST, meshes)
    return Scene("readme", make_ubo(), tris, models, cached_envmap(*env_size), width, height, max_depth,
                 flags=T.FLAG_FLOOR | T.FLAG_CHECKER | T.FLAG_ENVMAP | T.FLAG_ROW_QUIRK)


CONFIGS = {"C1": config_c1, "C2": config_c2, "C3": config_c3, "C4": config_c4, "C5": config_c5}
