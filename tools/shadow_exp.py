#!/usr/bin/env python3
"""Prices coherent (deferred) shadow tracing against the in-frame shadow queries.

With a TRT_DIAG_DUMP_SHADOW build (tools/build_variants.sh dumpshadow; TRT_LIB=...), one
counting pass of a frame appends every shadow query (origin, max distance, direction) to a
device buffer instead of tracing it, in the order the waves issue them (per wave: light 0 of
its hit lanes, then light 1, ...).  The same queries are then traced by shadow_batch_kernel
(64 consecutive queries per wave, one per lane) and timed with HIP events; optionally sorted
by light first.  Prints one JSON line.

  TRT_LIB=variants/libtrt_dumpshadow.so python tools/shadow_exp.py --config C4
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import lib, types as T
    from vkcomputeshader_tinyraytracer_amd import scene as S

    L = lib()
    L.trt_diag_set_buffer.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.trt_diag_counter.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.trt_diag_counter.restype = ctypes.c_ulonglong
    L.trt_diag_shadow_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(T.Params), ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_void_p]
    sc = S.config_reference_default() if a.config == "ref" else (
        S.config_readme() if a.config == "readme" else S.CONFIGS[a.config]())
    p = sc.params()
    r = trt.Renderer(0)
    r.upload_scene(sc)
    _, _, st = r.draw_frame(p, count=True)
    nsh = st["shadow_rays"]
    buf = torch.empty((2 * nsh + 64, 4), dtype=torch.float32, device="cuda")
    L.trt_diag_set_buffer(r._h, buf.data_ptr())
    r.draw_frame(p, count=True)
    torch.cuda.synchronize()
    n = int(L.trt_diag_counter(r._h, 31))
    L.trt_diag_set_buffer(r._h, None)
    assert n == nsh, (n, nsh)
    occ = torch.empty(n, dtype=torch.int32, device="cuda")
    pd = T.Params.from_buffer_copy(p)
    pd.flags |= T.FLAG_DEVICE_PTRS
    res = {"config": a.config, "shadow_rays": n}

    def run(rays, tag):
        s = torch.cuda.Stream()
        r.set_stream(s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            L.trt_diag_shadow_batch(r._h, ctypes.byref(pd), rays.data_ptr(), n, occ.data_ptr())
        e0.record(s)
        for _ in range(a.reps):
            L.trt_diag_shadow_batch(r._h, ctypes.byref(pd), rays.data_ptr(), n, occ.data_ptr())
        e1.record(s)
        s.synchronize()
        r.set_stream(None)
        ms = e0.elapsed_time(e1) / a.reps
        res[tag] = {"ms": round(ms, 4), "Mquery_s": round(n / ms / 1e3, 1),
                    "occluded_frac": round(float(occ.float().mean().item()), 4)}

    rays = buf[: 2 * n].contiguous()
    run(rays, "issue_order")
    # sorted by light (key: the direction's light = nearest of the three light directions is
    # not stored; sort by max distance bucket instead is meaningless) -> sort by direction octant
    d = rays.view(n, 2, 4)[:, 1, :3]
    key = ((d[:, 0] >= 0).int() * 4 + (d[:, 1] >= 0).int() * 2 + (d[:, 2] >= 0).int())
    order = torch.argsort(key, stable=True)
    run(rays.view(n, 2, 4)[order].reshape(2 * n, 4).contiguous(), "octant_sorted")
    print(json.dumps(res), flush=True)
    r.close()


if __name__ == "__main__":
    main()
