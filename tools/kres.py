#!/usr/bin/env python3
"""Kernel resources (VGPRs, SGPRs, scratch bytes per lane, LDS) of the built trace kernels, read
from the gfx950 code object inside build/csrc/trt_kernel.o (llvm-objdump --offloading + the
AMDGPU metadata notes): `make resources` without a recompile.

    python tools/kres.py [regex]     (default: every trace/defer kernel)
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
LLVM = Path("/opt/rocm/lib/llvm/bin")


def main() -> None:
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else r"trace_|defer_")
    obj = REPO / "build" / "csrc" / "trt_kernel.o"
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td) / "k.o"
        tmp.write_bytes(obj.read_bytes())
        subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(tmp)], check=True, capture_output=True)
        co = next(Path(td).glob("k.o.*gfx950*"))
        notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
    for blk in re.split(r"\n  - \.agpr_count", notes)[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", blk)
            return m.group(1) if m else "?"
        name = g("name")
        if not pat.search(name):
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"{dem:70s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} scratch {g('private_segment_fixed_size'):>5} "
              f"lds {g('group_segment_fixed_size'):>6} spill_v {g('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
