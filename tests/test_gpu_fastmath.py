"""GPU proof that the kernel's shortened correctly-rounded fp32 sequences (csrc/trt_math.h)
return exactly the IEEE results hipcc's general sequences (and the CPU oracle) produce:
exhaustive for the reciprocal and the square root over their fast domains, 2^32 sampled pairs
for the division (tools/dbg/fastmath_check.hip)."""
from __future__ import annotations

import json
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

BIN = Path(__file__).resolve().parents[1] / "vkcomputeshader_tinyraytracer_amd" / "fastmath_check"


def test_fastmath_sequences_are_correctly_rounded():
    assert BIN.exists(), "build with __graft_entry__.build() (csrc Makefile target ../fastmath_check)"
    p = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=300)
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["tested"]["rcp"] > 2 * 2_000_000_000 and res["tested"]["sqrt"] > 1_800_000_000, res
    assert res["tested"]["div"] == 1 << 32, res
    assert (res["rcp"], res["sqrt"], res["div"], res["rsqrt"]) == (0, 0, 0, 0), res
    assert p.returncode == 0
