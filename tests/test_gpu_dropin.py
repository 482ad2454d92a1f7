"""The C-ABI's real caller on the GPU: tests/native/drop_in_host, a plain C++ program built from
INTEGRATION.md §2 (the reference's createShaderStorageBuffers + drawFrame with the Vulkan
compute objects replaced by libtrt; main.cpp:1494-1664, 2165-2205), run as a fresh process with
no Python or torch in it.  It builds the shipped scene with trt_scene_add_mesh from the committed
mesh dump, uploads, and renders through trt_render (host output), trt_render_frames (device
outputs, the camera walk) and trt_render_multi (one-device communicator).  Its HIP runtime and
RCCL are the ones libtrt's RUNPATH names (/opt/rocm/lib), not torch's copies.

Every frame must equal, bit for bit, the same frame rendered in this pytest process through the
Python package (same kernel, the other runtime), and the committed golden hashes
(tests/golden/frame_hashes.json, "dropin:<frame>"); the shipped frame is also checked against the
CPU oracle under the parity bar."""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from tests.helpers import assert_rgba8_close
from vkcomputeshader_tinyraytracer_amd import scene as S
from vkcomputeshader_tinyraytracer_amd import types as T

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parents[1]
HOST = REPO / "tests" / "native" / "drop_in_host"
DUMP = REPO / "tests" / "golden" / "dropin_meshes.bin"
HASHES = REPO / "tests" / "golden" / "frame_hashes.json"
W, H = 1024, 768


@pytest.fixture(scope="module")
def host_run(tmp_path_factory):
    out = tmp_path_factory.mktemp("dropin")
    env = {k: v for k, v in os.environ.items() if k != "LD_LIBRARY_PATH"}  # resolve by RUNPATH only
    r = subprocess.run([str(HOST), str(DUMP), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    frames = {d["frame"]: np.fromfile(out / f"{d['frame']}.rgba", np.uint8).reshape(H, W, 4)
              for d in lines if "frame" in d}
    info = {k: v for d in lines for k, v in d.items() if k != "frame" and k != "bytes"}
    rec = os.environ.get("TRT_DROPIN_RECORD")
    if rec:  # write the frames' hashes for committing (the first run of a new frame set)
        Path(rec).write_text(json.dumps({f"dropin:{k}": hashlib.sha256(v.tobytes()).hexdigest()
                                         for k, v in sorted(frames.items())}, indent=1) + "\n")
    return frames, info


def test_host_runs_on_the_rocm_runtime(host_run):
    frames, info = host_run
    assert info.get("done") is True
    assert "/opt/rocm" in info["libamdhip64"] and "torch" not in info["libamdhip64"], info
    assert "/opt/rocm" in info["librccl"] and "torch" not in info["librccl"], info
    assert info["scene_triangles"] == 37956 and info["scene_batches"] == 594
    assert len(frames) == 1 + 4 + 8 + 1


def _python_frames(meshes):
    """The same frames through the Python package (torch's runtime in this process)."""
    import vkcomputeshader_tinyraytracer_amd as trt

    out = {}
    ref = S.config_reference_default(meshes)
    c2 = S.config_c2()
    with trt.Renderer(0) as r:
        r.upload_scene(ref)
        out["shipped"], _, _ = r.draw_frame(ref.params())
        for k, u in enumerate(S.camera_path(ref.ubo, 4)):
            r.update_ubo(u)
            out[f"shipped_walk_{k}"], _, _ = r.draw_frame(ref.params())
        r.upload_scene(c2)
        for k, u in enumerate(S.camera_path(c2.ubo, 8)):
            r.update_ubo(u)
            out[f"c2_walk_{k}"], _, _ = r.draw_frame(c2.params())
    out["multi_c2"] = out["c2_walk_0"]
    return out


def test_host_frames_equal_python_path(host_run, golden_meshes):
    frames, _ = host_run
    want = _python_frames(golden_meshes)
    assert sorted(frames) == sorted(want)
    for k in frames:
        assert np.array_equal(frames[k], want[k]), k


def test_host_frames_equal_committed_hashes(host_run):
    frames, _ = host_run
    committed = json.loads(HASHES.read_text())
    keys = [f"dropin:{k}" for k in frames]
    missing = [k for k in keys if k not in committed]
    if len(missing) == len(keys):
        pytest.skip("no committed drop-in hashes yet (record with TRT_DROPIN_RECORD)")
    assert not missing, missing
    for k, v in frames.items():
        assert hashlib.sha256(v.tobytes()).hexdigest() == committed[f"dropin:{k}"], k


def test_host_shipped_frame_vs_oracle(host_run, golden_meshes):
    from oracle import oracle as orc

    frames, _ = host_run
    sc = S.config_reference_default(golden_meshes)
    o8, _, _ = orc.render(sc, sc.params())
    assert_rgba8_close(frames["shipped"], o8)
    assert T.FLAGS_REFERENCE == sc.flags
