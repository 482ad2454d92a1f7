"""Regenerates the JPEG decode fixtures (SURVEY §8 f2 — envmap input parity with the
reference's stb_image v2.22, main.cpp:928-949).  Run in the build container, where the
read-only reference checkout exists; the GPU box only reads the outputs.

  jpeg/*.jpg          small synthetic JPEGs encoded here with Pillow/libjpeg covering the
                      decoder's cases (baseline / progressive, 4:4:4 / 4:2:2 / 4:2:0,
                      grayscale, CMYK, restart intervals, optimised tables, 1-pixel edges)
  jpeg_goldens.json   "synthetic": per committed file, width, height, channels in file,
                      SHA-256 of the RGBA8 buffer stbi_load(..., STBI_rgb_alpha) returns and a
                      few sampled texels;
                      "reference_assets": the same derived values (no bytes) for the
                      reference's own JPEGs (assets/background.jpg — the envmap — and the
                      README render), which are read in place where the checkout exists and
                      are not copied into this repository

The expected outputs come from the reference's own vendored stb_image.h, compiled unmodified
by `make -C oracle ref` into oracle/_ref/stb_decode (SSE2 kernels on x86-64, as the
reference's x64 build).  Usage: python tests/golden/make_jpeg_goldens.py
"""
from __future__ import annotations

import hashlib
import json
import subprocess
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
OUT = REPO / "tests" / "golden" / "jpeg"
REF = Path("/root/reference")
STB = REPO / "oracle" / "_ref" / "stb_decode"
# read in place (never copied): the envmap stbi_load reads (main.cpp:930) and a baseline JPEG
REFERENCE_ASSETS = {
    "assets/background.jpg": REF / "VulkanComputeShaderApplication" / "assets" / "background.jpg",
    "README.assets/output-result-v2-1024-768-our.jpg": REF / "README.assets" / "output-result-v2-1024-768-our.jpg",
}


def synth(w: int, h: int, seed: int) -> np.ndarray:
    """Smooth colour gradients + a hard-edged disc + noise: exercises both DC and AC terms."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([255 * x / max(w - 1, 1), 255 * y / max(h - 1, 1),
                    127 + 120 * np.sin((x + 2 * y) / 5.0)], -1)
    disc = (x - w / 2) ** 2 + (y - h / 2) ** 2 < (min(w, h) / 3) ** 2
    img[disc] = [250, 30, 60]
    img += rng.normal(0, 12, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def cases():
    """name -> (Pillow image mode, size, save kwargs)."""
    return {
        "b444_q90_37x23.jpg": ("RGB", (37, 23), dict(quality=90, subsampling=0)),
        "b420_q75_37x23.jpg": ("RGB", (37, 23), dict(quality=75, subsampling=2)),
        "b422_q85_64x40.jpg": ("RGB", (64, 40), dict(quality=85, subsampling=1)),
        "b420_opt_q60_70x52.jpg": ("RGB", (70, 52), dict(quality=60, subsampling=2, optimize=True)),
        "b420_rst3_q80_45x37.jpg": ("RGB", (45, 37), dict(quality=80, subsampling=2, restart_marker_blocks=3)),
        "p420_q80_61x45.jpg": ("RGB", (61, 45), dict(quality=80, subsampling=2, progressive=True)),
        "p444_q95_50x33.jpg": ("RGB", (50, 33), dict(quality=95, subsampling=0, progressive=True)),
        "p422_rst2_q70_66x34.jpg": ("RGB", (66, 34), dict(quality=70, subsampling=1, progressive=True,
                                                          restart_marker_blocks=2)),
        "p420_q90_256x192.jpg": ("RGB", (256, 192), dict(quality=90, subsampling=2, progressive=True)),
        "gray_b_q90_29x31.jpg": ("L", (29, 31), dict(quality=90)),
        "gray_p_q70_33x17.jpg": ("L", (33, 17), dict(quality=70, progressive=True)),
        "cmyk_b_q90_24x18.jpg": ("CMYK", (24, 18), dict(quality=90)),
        "edge_b420_1x17.jpg": ("RGB", (1, 17), dict(quality=85, subsampling=2)),
        "edge_b420_17x1.jpg": ("RGB", (17, 1), dict(quality=85, subsampling=2)),
        "edge_p420_2x3.jpg": ("RGB", (2, 3), dict(quality=85, subsampling=2, progressive=True)),
    }


def make_inputs() -> list[Path]:
    from PIL import Image

    OUT.mkdir(parents=True, exist_ok=True)
    files = []
    for k, (name, (mode, (w, h), kw)) in enumerate(sorted(cases().items())):
        im = Image.fromarray(synth(w, h, seed=k), "RGB").convert(mode)
        im.save(OUT / name, "JPEG", **kw)
        files.append(OUT / name)
    return files


def stb_decode(path: Path, td: str) -> tuple[np.ndarray, int]:
    raw = Path(td) / "out.rgba"
    res = subprocess.run([str(STB), str(path), str(raw)], check=True, capture_output=True, text=True)
    w, h, n = map(int, res.stdout.split())
    return np.fromfile(raw, np.uint8).reshape(h, w, 4), n


def describe(path: Path, td: str) -> dict:
    px, n = stb_decode(path, td)
    h, w = px.shape[:2]
    pts = sorted({(0, 0), (h - 1, w - 1), (h // 2, w // 2), (h // 3, (2 * w) // 3)})
    return {
        "width": w, "height": h, "channels": n,
        "jpeg_sha256": hashlib.sha256(path.read_bytes()).hexdigest(),
        "rgba_sha256": hashlib.sha256(px.tobytes()).hexdigest(),
        "texels": [[y, x, px[y, x].tolist()] for y, x in pts],
    }


def main() -> None:
    subprocess.run(["make", "-s", "-C", str(REPO / "oracle"), "ref"], check=True)
    files = make_inputs()
    meta = {"synthetic": {}, "reference_assets": {}}
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            meta["synthetic"][f.name] = describe(f, td)
        for rel, f in REFERENCE_ASSETS.items():
            meta["reference_assets"][rel] = describe(f, td)
    (REPO / "tests" / "golden" / "jpeg_goldens.json").write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")
    for sec in meta.values():
        print(json.dumps({k: (v["width"], v["height"], v["channels"]) for k, v in sec.items()}))


if __name__ == "__main__":
    main()
