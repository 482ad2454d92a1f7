"""The reference's own renders: lossless PNG screenshots of its Vulkan compute shader, read in
place from the read-only reference checkout (build container only; nothing is copied).

Each shot names the scene it shows (config.hpp modelList, shader.comp flags), the frame offset
(y, x) at which the screenshot registers with a 1024x768 frame, and the display transform:
the compute image holds pow(c, 2.2) (shader.comp:598) and is drawn into a B8G8R8A8_SRGB
swapchain (main.cpp:2341), so the displayed byte is sRGB-encode(pow(c, 2.2)) — the oracle's
TRT_FLAG_SRGB_OUT.  The envmap is background.jpg decoded by the reference's own stb_image
v2.22 (oracle/_ref/stb_decode, built in place by `make -C oracle ref`), as main.cpp:930 does.

Used by tests/test_reference_screens.py (the pin of the oracle to the running reference) and
tools/ref_screens.py (offset search)."""
from __future__ import annotations

import hashlib
import os
import subprocess
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
VCSA = REF / "VulkanComputeShaderApplication"
REPO = Path(__file__).resolve().parents[1]
STB_DECODE = REPO / "oracle" / "_ref" / "stb_decode"
# SHA-256 of the stb v2.22 RGBA decode of background.jpg (SURVEY §8c iv).
BACKGROUND_SHA256 = "f183e364ed4338676e426d5484da764979713ac38055d67c9bd29781199cf5b1"


@dataclass(frozen=True)
class Shot:
    name: str
    png: str  # path under /root/reference
    models: tuple  # config.hpp modelList entries (MODEL_INFOS keys)
    offset: tuple  # (y, x): frame pixel of the (cropped) screenshot's (0, 0)
    flags: int | None = None  # None = FLAGS_REFERENCE (floor + envmap + row quirk)
    screen_crop: tuple = (0, 0)  # (y, x): screenshot pixel where the compared region starts (window chrome)
    max_depth: int = 20
    source: str = ""
    # Agreement the test asserts (fraction of compared pixels within 1 LSB on every channel).
    min_within1: float = 0.999
    rows_below: int | None = None  # compare only frame rows < this (older-shader regions masked)
    direct_only: bool = False  # compare only pixels with no secondary-ray contribution (see below)
    notes: str = ""


SHOTS = (
    Shot("shipped", "new_feature.assets/image-20250703101716795.png", ("glass", "water", "ice"), (339, 249),
         source="new_feature.md:126-134 (fig. 6: glass + whisky + ice with the volume-stack shader)"),
    Shot("three_models", "new_feature.assets/image-20250701202425177.png", ("glass", "water", "ice"), (254, 187),
         source="new_feature.md:17-22 (fig. 1: glass + whisky + ice before the volume stack)"),
    Shot("glass", "new_feature.assets/image-20250701202456088.png", ("glass",), (305, 223),
         source="new_feature.md:25-30 (fig. 2: glass alone)"),
    Shot("water", "new_feature.assets/image-20250701202522993.png", ("water",), (315, 231),
         source="new_feature.md:32-37 (fig. 3: whisky alone)"),
    Shot("ice", "new_feature.assets/image-20250701202549180.png", ("ice",), (303, 228),
         source="new_feature.md:39-44 (fig. 4: ice alone)"),
    # The TA's BaseCode as shipped to the students (README.md:32-34): the four spheres on a
    # checker floor under the constant background, captured with the window chrome (title
    # bar 36 px, border 6 px).  It is an older shader: its glass and mirror spheres and its
    # floor window differ from shader.comp, so only pixels whose colour has no secondary-ray
    # term (oracle depth-1 frame == depth-4 frame: sky, the red sphere, the floor and their
    # shadows, i.e. sphere intersection, checker, Phong and shadow rays) above frame row 640
    # (where the older floor ended) are compared.
    Shot("basecode_spheres", "README.assets/image-20250608191118648.png", (), (0, 0),
         flags=(1 << 0) | (1 << 1) | (1 << 2) | (1 << 4),  # spheres, floor, checker, row quirk
         screen_crop=(36, 6), max_depth=4, rows_below=640, direct_only=True,
         source="README.md:32-34 (BaseCode: spheres, checker floor, constant background)"),
)


def have_reference() -> bool:
    return VCSA.exists()


_ENV = None


def background_rgba() -> np.ndarray:
    """background.jpg through the reference's own stb_image (main.cpp:930), (H, W, 4) uint8."""
    global _ENV
    if _ENV is None:
        if not STB_DECODE.exists():
            subprocess.run(["make", "-s", "-C", os.fspath(REPO / "oracle"), "ref"], check=True)
        with tempfile.TemporaryDirectory() as td:
            out = Path(td) / "bg.rgba"
            r = subprocess.run([os.fspath(STB_DECODE), os.fspath(VCSA / "assets" / "background.jpg"), os.fspath(out)],
                               check=True, capture_output=True, text=True)
            w, h, _ = (int(v) for v in r.stdout.split())
            raw = out.read_bytes()
        assert hashlib.sha256(raw).hexdigest() == BACKGROUND_SHA256
        _ENV = np.frombuffer(raw, np.uint8).reshape(h, w, 4).copy()
    return _ENV


def load_screen(shot: Shot) -> np.ndarray:
    from PIL import Image  # PNG is lossless; any decoder gives the same bytes

    with Image.open(REF / shot.png) as im:
        a = np.asarray(im.convert("RGB"), dtype=np.uint8)
    cy, cx = shot.screen_crop
    return a[cy:cy + 768, cx:cx + 1024].copy()


_FRAMES: dict = {}


def oracle_frame(shot: Shot, width: int = 1024, height: int = 768) -> np.ndarray:
    """The oracle's frame of the shot's scene as displayed: (768, 1024, 4) uint8 sRGB."""
    key = (shot.models, shot.flags, shot.max_depth, width, height)
    if key not in _FRAMES:
        from oracle import oracle as orc
        from vkcomputeshader_tinyraytracer_amd import scene as S
        from vkcomputeshader_tinyraytracer_amd import types as T

        if shot.models:
            tris, models = S.build_models(shot.models, S.load_golden_meshes())
        else:
            tris, models = np.zeros(0, T.TRIANGLE), np.zeros(0, T.MODEL)
        flags = T.FLAGS_REFERENCE if shot.flags is None else int(shot.flags)
        env = background_rgba() if flags & T.FLAG_ENVMAP else None
        sc = S.Scene(shot.name, S.make_ubo(), tris, models, env, width, height, shot.max_depth,
                     flags=flags)
        o8, _, _ = orc.render(sc, sc.params(flags=flags | T.FLAG_SRGB_OUT))
        _FRAMES[key] = o8
    return _FRAMES[key]


def compare_mask(shot: Shot, frame: np.ndarray) -> np.ndarray:
    """Frame pixels the shot is compared on (bool, frame-sized)."""
    m = np.ones(frame.shape[:2], bool)
    if shot.rows_below is not None:
        m[shot.rows_below:] = False
    if shot.direct_only:
        d1 = oracle_frame(Shot(shot.name + "_d1", shot.png, shot.models, shot.offset, flags=shot.flags,
                               screen_crop=shot.screen_crop, max_depth=1))
        m &= (d1[..., :3] == frame[..., :3]).all(axis=-1)
    return m


def pixel_diff(frame: np.ndarray, screen: np.ndarray, offset, shot: Shot | None = None):
    """(|frame - screen| max over RGB, mask) on the screenshot's footprint, or None if it
    does not fit at `offset` (frame pixel of screenshot (0, 0))."""
    y, x = offset
    h, w = screen.shape[:2]
    if y < 0 or x < 0 or y + h > frame.shape[0] or x + w > frame.shape[1]:
        return None
    f = frame[y:y + h, x:x + w, :3].astype(np.int16)
    d = np.abs(f - screen.astype(np.int16)).max(axis=-1)
    m = compare_mask(shot, frame)[y:y + h, x:x + w] if shot is not None else np.ones(d.shape, bool)
    return d, m


def register(frame: np.ndarray, screen: np.ndarray, offset, shot: Shot | None = None) -> dict | None:
    """Agreement of the screenshot with the frame at `offset` on the shot's compared pixels."""
    r = pixel_diff(frame, screen, offset, shot)
    if r is None:
        return None
    d = r[0][r[1]]
    return {
        "px": int(d.size),
        "within1": float((d <= 1).mean()),
        "exact": float((d == 0).mean()),
        "max": int(d.max()),
        "n_gt1": int((d > 1).sum()),
        "n_gt8": int((d > 8).sum()),
    }


def _display(c) -> np.ndarray:
    """shader.comp:598 pow(c, 2.2) then the sRGB swapchain encode, as 8-bit (float64 here:
    at most 1 LSB from the oracle's float32 path, far below the instability threshold)."""
    g = np.power(np.clip(np.asarray(c, np.float64), 0.0, 1.0), 2.2)
    e = np.where(g <= 0.0031308, 12.92 * g, 1.055 * np.power(g, 1 / 2.4) - 0.055)
    return np.floor(e * 255 + 0.5).astype(np.int64)


def _scene(shot: Shot):
    from vkcomputeshader_tinyraytracer_amd import scene as S
    from vkcomputeshader_tinyraytracer_amd import types as T

    if shot.models:
        tris, models = S.build_models(shot.models, S.load_golden_meshes())
    else:
        tris, models = np.zeros(0, T.TRIANGLE), np.zeros(0, T.MODEL)
    flags = T.FLAGS_REFERENCE if shot.flags is None else int(shot.flags)
    env = background_rgba() if flags & T.FLAG_ENVMAP else None
    return S.Scene(shot.name, S.make_ubo(), tris, models, env, 1024, 768, shot.max_depth, flags=flags)


def _nudge(v: np.float32, k: int) -> np.float32:
    to = np.float32(np.inf if k > 0 else -np.inf)
    for _ in range(abs(k)):
        v = np.nextafter(v, to)
    return v


def instability(shot: Shot, fy: int, fx: int, screen_rgb, radius1: int = 4, radius3: int = 6) -> dict:
    """Is frame pixel (fy, fx) chaotic in the oracle?  Its primary direction is moved by a few
    float32 ulps (first each component alone by up to `radius1` ulps, then every combination
    within `radius3` ulps per component) and the pixel re-traced with the oracle's cast_ray.
    Returns whether some perturbation moves the displayed value by more than 1 LSB, and the
    closest any perturbation comes to the screenshot's value."""
    from oracle import oracle as orc

    sc = _scene(shot)
    p = sc.params()
    cam = tuple(float(v) for v in sc.ubo["camPos"][:3])
    d0 = np.array(orc.primary_dir(p, fx, fy), np.float32)
    base = _display(orc.cast_ray(sc, p, cam, d0)[0])
    scr = np.asarray(screen_rgb, np.int64)
    out = {"unstable": False, "closest": int(np.abs(base - scr).max()), "tries": 0}

    def probe(ks) -> bool:
        d = d0.copy()
        for c, k in enumerate(ks):
            d[c] = _nudge(d[c], k)
        v = _display(orc.cast_ray(sc, p, cam, d)[0])
        out["tries"] += 1
        out["closest"] = min(out["closest"], int(np.abs(v - scr).max()))
        if int(np.abs(v - base).max()) > 1:
            out["unstable"] = True
        return out["unstable"] and out["closest"] <= 1

    for c in range(3):
        for k in range(1, radius1 + 1):
            for s in (k, -k):
                ks = [0, 0, 0]
                ks[c] = s
                if probe(ks):
                    return out
    if out["unstable"]:
        return out
    r = range(-radius3, radius3 + 1)
    for a in r:
        for b in r:
            for c in r:
                if probe((a, b, c)):
                    return out
    return out


def edge_match(frame: np.ndarray, fy: int, fx: int, screen_rgb) -> bool:
    """The screenshot's value is (within 1 LSB) the oracle's value of an 8-neighbour: an edge
    (silhouette, checker square, shadow boundary) placed a fraction of a pixel apart."""
    scr = np.asarray(screen_rgb, np.int64)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            y, x = fy + dy, fx + dx
            if (dy or dx) and 0 <= y < frame.shape[0] and 0 <= x < frame.shape[1]:
                if int(np.abs(frame[y, x, :3].astype(np.int64) - scr).max()) <= 1:
                    return True
    return False


def sphere_acne(shot: Shot, fy: int, fx: int, screen_rgb, tol: int = 2) -> bool:
    """Shadow acne of the older shader: the pixel's primary ray hits one of the UBO spheres
    (nearest of the four, main.cpp:132-137) and the screenshot equals (within `tol` LSB) the
    direct Phong term of shader.comp:483-507 with one or more lights dropped, i.e. a shadow
    ray that found its own sphere.  float64 restatement of the direct term only; it is used
    only to classify a screenshot pixel, never as a parity reference."""
    import itertools

    from oracle import oracle as orc
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = _scene(shot)
    d = np.array(orc.primary_dir(sc.params(), fx, fy), np.float64)
    o = np.array(sc.ubo["camPos"][:3], np.float64)
    best = None
    for cr, mat in S.SPHERES:
        c, r = np.array(cr[:3], np.float64), float(cr[3])
        L = c - o
        tca = L @ d
        d2 = L @ L - tca * tca
        if d2 > r * r:
            continue
        t = tca - np.sqrt(r * r - d2)
        if t > 1e-4 and (best is None or t < best[0]):
            best = (t, c, r, mat)
    if best is None:
        return False
    t, c, r, mat = best
    p = o + t * d
    n = (p - c) / r
    kd = np.array(mat["diffuse_specular"][:3], np.float64)
    ex = float(mat["diffuse_specular"][3])
    alb = np.array(mat["albedo"], np.float64)
    terms = []
    for lp in S.LIGHTS:
        l = np.array(lp, np.float64) - p
        l /= np.linalg.norm(l)
        refl = -l - 2 * (n @ -l) * n
        terms.append(max(0.0, n @ l) * kd * alb[0] + max(0.0, refl @ -d) ** ex * kd * alb[1])
    scr = np.asarray(screen_rgb, np.int64)
    for keep in itertools.product((0, 1), repeat=len(terms)):
        if all(keep):
            continue
        col = sum((tm for tm, k in zip(terms, keep) if k), np.zeros(3))
        if int(np.abs(_display(col) - scr).max()) <= tol:
            return True
    return False
