"""Envmap JPEG decode parity with the reference's stb_image v2.22.

Goldens (tests/golden/jpeg_goldens.json, made by tests/golden/make_jpeg_goldens.py) hold the
SHA-256 and sampled texels of the RGBA8 buffer the reference's own stb_image returns for
stbi_load(..., STBI_rgb_alpha) — for the committed synthetic JPEGs (baseline / progressive,
4:4:4 / 4:2:2 / 4:2:0, grayscale, CMYK, restart intervals, 1-pixel edges) and, by hash only,
for the reference's envmap asset itself.

CPU: the product's host entropy decoder (trt_jpeg_parse) + the oracle's numpy restatement of
stb's reconstruction (oracle/jpeg_ref.py) reproduce every golden bit for bit; the envmap asset
is read in place when the reference checkout is present.  GPU: the product's full path
(host entropy decode + HIP reconstruction, trt_jpeg_decode) reproduces every golden, a
reference-sized progressive JPEG matches the oracle, and trt_upload_envmap_jpeg feeds the
renderer the same binding 4 as an RGBA upload."""
from __future__ import annotations

import hashlib
import io
import json
from pathlib import Path

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd import TrtError
from vkcomputeshader_tinyraytracer_amd import types as T
from vkcomputeshader_tinyraytracer_amd.jpeg import JpegFile

GOLDEN = Path(__file__).resolve().parent / "golden"
META = json.loads((GOLDEN / "jpeg_goldens.json").read_text())
SYN = sorted(META["synthetic"])
REF_ROOT = Path("/root/reference")
REF_ASSETS = {
    "assets/background.jpg": REF_ROOT / "VulkanComputeShaderApplication" / "assets" / "background.jpg",
    "README.assets/output-result-v2-1024-768-our.jpg": REF_ROOT / "README.assets" / "output-result-v2-1024-768-our.jpg",
}


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _check_golden(img: np.ndarray, m: dict):
    assert img.shape == (m["height"], m["width"], 4)
    for y, x, px in m["texels"]:
        assert img[y, x].tolist() == px, (y, x)
    assert _sha(img) == m["rgba_sha256"]


def test_fixture_integrity():
    for name in SYN:
        data = (GOLDEN / "jpeg" / name).read_bytes()
        assert hashlib.sha256(data).hexdigest() == META["synthetic"][name]["jpeg_sha256"]


@pytest.mark.parametrize("name", SYN)
def test_entropy_decode_plus_oracle_matches_stb(name):
    from oracle import jpeg_ref

    m = META["synthetic"][name]
    jf = JpegFile(GOLDEN / "jpeg" / name)
    assert (jf.info.width, jf.info.height) == (m["width"], m["height"])
    assert jf.info.components == (4 if name.startswith("cmyk") else m["channels"])
    assert jf.info.progressive == (1 if name.startswith(("p", "gray_p", "edge_p")) else 0)
    _check_golden(jpeg_ref.reconstruct(jf), m)


@pytest.mark.reference
@pytest.mark.parametrize("rel", sorted(REF_ASSETS))
def test_reference_assets_match_stb(rel):
    """The reference's own envmap (and README render), read in place: product entropy decode
    + oracle reconstruction give the exact stbi_load bytes (SURVEY §8c (iv) texels)."""
    from oracle import jpeg_ref

    path = REF_ASSETS[rel]
    if not path.exists():
        pytest.skip("reference checkout absent")
    m = META["reference_assets"][rel]
    assert hashlib.sha256(path.read_bytes()).hexdigest() == m["jpeg_sha256"]
    _check_golden(jpeg_ref.reconstruct(JpegFile(path)), m)


def test_envmap_texels_of_survey():
    """the stb decode of background.jpg, pinned by texels."""
    m = META["reference_assets"]["assets/background.jpg"]
    assert (m["width"], m["height"]) == (7616, 3808)
    assert m["rgba_sha256"] == "f183e364ed4338676e426d5484da764979713ac38055d67c9bd29781199cf5b1"


@pytest.mark.parametrize("data,why", [
    (b"", "empty"),
    (b"\x89PNG\r\n\x1a\n" + b"\0" * 32, "not a JPEG"),
    (None, "truncated"),
    (None, "arithmetic"),
])
def test_parse_errors(data, why):
    src = (GOLDEN / "jpeg" / "b420_q75_37x23.jpg").read_bytes()
    if why == "truncated":
        data = src[:200]
    elif why == "arithmetic":  # SOF0 -> SOF9 (arithmetic coding), unsupported as in stb
        i = src.index(b"\xff\xc0")
        data = src[:i] + b"\xff\xc9" + src[i + 2:]
    with pytest.raises(TrtError):
        JpegFile(data)


def test_coefficient_planes_layout():
    jf = JpegFile(GOLDEN / "jpeg" / "p420_q80_61x45.jpg")
    i = jf.info
    assert (i.hmax, i.vmax) == (2, 2)
    y = jf.coefficients(0)
    assert y.shape == (i.blocks_h[0], i.blocks_w[0], 8, 8) == (6, 8, 8, 8)
    assert jf.coefficients(1).shape == (3, 4, 8, 8)
    assert jf.quant(0).shape == (8, 8) and (jf.quant(0) > 0).all()
    with pytest.raises(IndexError):
        jf.coefficients(3)


# ---- GPU: the product path (host entropy decode + HIP reconstruction) ------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", SYN)
def test_gpu_decode_matches_stb(gpu_renderer, name):
    img = gpu_renderer.decode_jpeg(GOLDEN / "jpeg" / name)
    _check_golden(img, META["synthetic"][name])


@pytest.mark.gpu
def test_gpu_decode_into_device_tensor(gpu_renderer):
    torch = pytest.importorskip("torch")
    name = "p420_q90_256x192.jpg"
    out = torch.zeros((192, 256, 4), dtype=torch.uint8, device="cuda")
    gpu_renderer.decode_jpeg(GOLDEN / "jpeg" / name, out=out)
    torch.cuda.synchronize()
    _check_golden(out.cpu().numpy(), META["synthetic"][name])


def _big_progressive_jpeg(w=7616, h=3808) -> bytes:
    """A reference-sized progressive 4:2:0 JPEG made here (Pillow/libjpeg), seeded."""
    from PIL import Image

    rng = np.random.default_rng(7)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([128 + 100 * np.sin(xx / 97.0), 128 + 100 * np.cos(yy / 53.0), (xx + yy) % 256], -1)
    img += rng.normal(0, 6, img.shape).astype(np.float32)
    buf = io.BytesIO()
    Image.fromarray(np.clip(img, 0, 255).astype(np.uint8), "RGB").save(buf, "JPEG", quality=92, progressive=True)
    return buf.getvalue()


@pytest.mark.gpu
def test_gpu_decode_reference_sized_envmap(gpu_renderer):
    """7616 x 3808 progressive (the envmap's size and process): GPU == oracle."""
    from oracle import jpeg_ref

    data = _big_progressive_jpeg()
    jf = JpegFile(data)
    gpu = gpu_renderer.decode_jpeg(jf)
    ref = jpeg_ref.reconstruct(jf)
    assert np.array_equal(gpu, ref)


@pytest.mark.gpu
def test_upload_envmap_jpeg_feeds_binding4(gpu_renderer):
    """trt_upload_envmap_jpeg == trt_upload_scene with the decoded RGBA as env: same frame."""
    from vkcomputeshader_tinyraytracer_amd import scene as S

    path = GOLDEN / "jpeg" / "p420_q90_256x192.jpg"
    rgba = gpu_renderer.decode_jpeg(path)
    sc = S.config_c2(160, 120, env_size=(256, 128))
    sc.env = rgba
    gpu_renderer.upload_scene(sc)
    want, _, _ = gpu_renderer.draw_frame(sc.params())
    sc2 = S.config_c2(160, 120, env_size=(256, 128))
    gpu_renderer.upload_scene(sc2)  # different (synthetic) env first
    gpu_renderer.upload_envmap_jpeg(path)
    got, _, _ = gpu_renderer.draw_frame(sc2.params())
    assert np.array_equal(got, want)
    with pytest.raises(TrtError):
        gpu_renderer.upload_envmap_jpeg(b"not a jpeg")
    p = sc2.params()
    p.flags |= T.FLAG_ENVMAP
    gpu_renderer.draw_frame(p)  # the envmap survived the failed upload
