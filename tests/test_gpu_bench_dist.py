"""The N > 1 bench process shape at one rank (bench.py --force-dist): torch.distributed's nccl
(RCCL) process group and libtrt's own RCCL rank communicator (trt_multi_create_rank, id passed
through the process group) in ONE process, the tiled weak headline with rotating roots, the
strong form, the single-root (rank 0) forms and the frame-per-GPU leg — the code the driver's
8-GPU scaling run executes, here on the one-GPU box."""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parents[1]


def test_bench_dist_branch_at_one_rank():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(random.randint(20000, 40000)))
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--force-dist", "--steps", "8", "--warmup", "2",
                        "--no-cpu", "--tiled-frames", "2", "--extra-frames", "0", "--traffic", "off",
                        "--camera-period", "4"], capture_output=True, text=True, timeout=400, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["path"].startswith("trt_render_multi_frames")
    assert line["config"]["last_frame_matches_trt_render"] is True
    assert line["config"]["value_form"].startswith("weak")
    assert line["frame_per_gpu"]["last_frame_ok"] is True
    assert line["strong_scaling"]["last_frames_match_trt_render"] is True
    fr = line["fixed_root"]
    assert fr["weak"]["last_frames_match_trt_render"] is True and fr["strong"]["last_frames_match_trt_render"] is True
    assert fr["weak"]["value"] > 0 and fr["strong"]["value"] > 0
    assert line["tiled_frame"]["matches_1gpu_frame"] is True
