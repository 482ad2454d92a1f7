"""The C++ drop-in host (tests/native/drop_in_host.cpp) on the CPU: it is built, links libtrt.so
and the HIP runtime by RUNPATH (no Python loader involved), and its restatement of the synthetic
envmap equals the Python package's byte for byte (so its frames render the same inputs as the
GPU parity tests).  The GPU run is tests/test_gpu_dropin.py."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from vkcomputeshader_tinyraytracer_amd.scene import synthetic_envmap

REPO = Path(__file__).resolve().parents[1]
HOST = REPO / "tests" / "native" / "drop_in_host"


def test_host_is_built_and_links_by_runpath():
    assert HOST.exists(), "build it: make -C vkcomputeshader_tinyraytracer_amd/csrc"
    if not shutil.which("readelf"):
        pytest.skip("readelf absent")
    dyn = subprocess.run(["readelf", "-d", str(HOST)], check=True, capture_output=True, text=True).stdout
    assert "[libtrt.so]" in dyn and "libamdhip64.so" in dyn
    assert "libpython" not in dyn and "torch" not in dyn
    assert "$ORIGIN/../../vkcomputeshader_tinyraytracer_amd" in dyn and "/opt/rocm/lib" in dyn
    lib = subprocess.run(["readelf", "-d", str(REPO / "vkcomputeshader_tinyraytracer_amd" / "libtrt.so")],
                         check=True, capture_output=True, text=True).stdout
    assert "Library soname: [libtrt.so]" in lib


@pytest.mark.parametrize("w,h", [(1000, 600), (7616, 3808)])
def test_host_envmap_equals_package(tmp_path, w, h):
    out = tmp_path / "env.raw"
    subprocess.run([str(HOST), "--envmap", str(w), str(h), str(out)], check=True, timeout=120)
    got = np.fromfile(out, np.uint8).reshape(h, w, 4)
    assert np.array_equal(got, synthetic_envmap(w, h))


def test_mesh_dump_matches_golden_meshes():
    """tests/golden/dropin_meshes.bin is the shipped scene's slice of tests/golden/meshes.npz."""
    import struct

    raw = (REPO / "tests" / "golden" / "dropin_meshes.bin").read_bytes()
    assert raw[:8] == b"TRTMESH1"
    (n,) = struct.unpack_from("<I", raw, 8)
    off = 12
    with np.load(REPO / "tests" / "golden" / "meshes.npz", allow_pickle=False) as z:
        for _ in range(n):
            (ln,) = struct.unpack_from("<I", raw, off)
            name = raw[off + 4:off + 4 + ln].decode()
            off += 4 + ln
            nv, nt = struct.unpack_from("<II", raw, off)
            off += 8
            pos = np.frombuffer(raw, "<f4", nv * 3, off).reshape(nv, 3)
            off += nv * 12
            idx = np.frombuffer(raw, "<u4", nt * 3, off).reshape(nt, 3)
            off += nt * 12
            assert np.array_equal(pos, z[f"{name}:pos"]) and np.array_equal(idx, z[f"{name}:idx"])
    assert off == len(raw)
