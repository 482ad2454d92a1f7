#!/usr/bin/env python3
"""Benchmark of the hot path: Mray/s (primary + secondary) at 1024x768, depth 4 (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5] [--no-cpu]

One step = one frame of the configuration rendered by the HIP kernel through the C-ABI
(trt_render, device output pointers, inputs resident in HBM).  At N > 1 (one process per GPU
under torch.distributed.run) every rank renders its own frame of a camera path, so per-GPU
work is fixed and there is no data-path collective ("scaling": "weak"); the barrier and the
max-over-ranks timing are the only cross-rank operations in the timed region.

Rank 0 prints ONE JSON line.  `roofline` is the algorithmic-byte rate of the trace kernel
(SURVEY.md §8d units x counts from a counting pass, / the kernel's average duration measured
with HIP events on its stream in the timed loop); `cpu_baseline` is the CPU oracle
(oracle/, fast mode) timed on this host on the same workload.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 157.3  # FP32 vector spec
TIME_EVERY = 16  # one timed (event-bracketed) launch per 16 frames


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5", "ref"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU oracle baseline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--inflight", type=int, default=2,
                    help="frames in flight (trt_set_frames_in_flight; the reference's MAX_FRAMES_IN_FLIGHT = 2)")
    ap.add_argument("--split", type=int, default=0, help="subtree split window (trt_set_subtree_split: 0 auto, 1 off)")
    ap.add_argument("--pmc", default=None, help="PMC summary json (tools/pmc_traffic.py) for roofline.traffic")
    ap.add_argument("--tiled-frames", type=int, default=20,
                    help="frames of the tiled-frame leg (C4 row-tiled over the ranks + RCCL gather); 0 skips it")
    return ap.parse_args()


WORKLOADS = {
    "C2": "1024x768, 4 spheres + floor + 7616x3808 seeded envmap, depth 4, 1 spp",
    "C3": "1920x1080, spheres + icosphere mesh (5,120 tris / 80 batches), depth 4",
    "C4": "3840x2160, 20 icospheres (102,400 tris / 1,600 batches), depth 4",
    "C5": "3840x2160, C4 scene, 16 jittered spp, depth 4",
    "ref": "1024x768, the shipped frame: glass + water + ice (37,956 tris / 594 batches), floor, "
           "7616x3808 seeded envmap, depth 20 (config.hpp:97-101, shader.comp:75-84)",
}


def algorithmic_bytes(st: dict, pixels: int, envmap: bool) -> int:
    """SURVEY.md §8(d) units: 24 B per batch (or hierarchy-node) bbox tested (+8 B start/count
    when a batch passes),
    36 B per triangle tested (v0, e1, e2), 16 B per sphere tested, 16 B per envmap sample
    (4 RGBA8 texels), 48 B material per closest hit (+36 B vertex normals for a triangle),
    4 B written per pixel."""
    hits = st["primary_rays"] + st["secondary_rays"] - st["misses"]
    return (24 * (st["batch_tests"] + st.get("node_tests", 0)) + 8 * st["batch_hits"] + 36 * st["tri_tests"]
            + 16 * st["sphere_tests"] + (16 * st["misses"] if envmap else 0)
            + 48 * hits + 36 * st["tri_nearest"] + 4 * pixels)


def cpu_baseline(scene, params, rays_per_frame: int, budget_s: float) -> dict:
    """CPU oracle (fast mode) on this host: whole frames, 1 warm-up, median of >= 3 frames
    within the time budget."""
    from oracle import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    orc.render(scene, params, threads=threads)  # warm-up (also loads/builds the library)
    times = []
    t_start = time.perf_counter()
    while len(times) < 3 or (time.perf_counter() - t_start < budget_s and len(times) < 50):
        t0 = time.perf_counter()
        _, _, st = orc.render(scene, params, threads=threads)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    cpu_rays = st["primary_rays"] + st["secondary_rays"]
    return {
        "value": round(cpu_rays / med / 1e6, 3),
        "unit": "Mray/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(times)} whole frames of the same workload after 1 warm-up, median "
                  f"{med * 1e3:.1f} ms/frame; oracle/trt_oracle.c fast mode, -O3, rows over {threads} threads",
        "rays_match_gpu": bool(cpu_rays == rays_per_frame),
    }


def tiled_frame(frames: int, rank: int, world: int, dist, dev: int) -> dict:
    """BASELINE configs[3]: a 3840x2160 C4 frame row-tiled across the ranks (interleaved
    8-row bands, dist.TiledFrame) and gathered to rank 0 as RGBA8 over RCCL (xGMI), then
    re-interleaved there.  Strong scaling: the frame is fixed, each rank renders 1/N of it.
    Two frames in flight (dist.PipelinedTiles, main.cpp:45): frame i's gather and render
    overlap frame i+1's render.  The timed region (barrier + synchronize on both sides, max over ranks)
    covers `frames` frames end to end.  `frame_sha256` (rank 0's last assembled frame) is the
    same at every world size: the tiled frame is bit-identical to the 1-GPU frame."""
    import hashlib

    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import dist as D, scene as S

    band = 8
    sc = S.config_c4()
    p = sc.params()
    r = trt.Renderer(dev)
    r.upload_scene(sc)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    r.set_stream(streams[0])
    pipe = D.PipelinedTiles(p.width, p.height, band, torch.device("cuda", dev), streams)
    bp = D.band_params(p, band, world, rank)
    _, _, st = r.draw_frame(bp, out8=pipe.tf[0].local, count=True)
    torch.cuda.synchronize()
    rays = st["primary_rays"] + st["secondary_rays"]

    def render(out, stream):  # frames alternate between two streams: consecutive renders overlap
        r.set_stream(stream)
        r.draw_frame(bp, out8=out)

    for _ in range(4):
        pipe.submit(render)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        img = pipe.submit(render)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed, float(rays)], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, rays = float(mx[0].item()), int(t[1].item())
    out = None
    if rank == 0:
        sha = hashlib.sha256(img.contiguous().cpu().numpy().tobytes()).hexdigest()
        out = {
            "workload": "C4: 3840x2160, 20 icospheres (102,400 tris), depth 4, one frame row-tiled "
                        f"over {world} GPU(s) in interleaved {band}-row bands",
            "scaling": "strong",
            "collective": "dist.gather of padded RGBA8 band buffers to rank 0 (RCCL over xGMI), "
                          "overlapped with the next frame's render (2 frames in flight on 2 render streams)"
                          if world > 1 else "none (1 GPU)",
            "frames": frames,
            "ms_per_frame": round(elapsed / frames * 1e3, 4),
            "frames_per_s": round(frames / elapsed, 3),
            "mray_s": round(rays * frames / elapsed / 1e6, 3),
            "rays_per_frame": rays,
            "gather_bytes_per_frame": int(pipe.tf[0].local.numel() * world) if world > 1 else 0,
            "frame_sha256": sha,
        }
    r.close()
    return out


def main():
    args = parse()
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S, types as T

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    scene = S.config_reference_default() if args.config == "ref" else S.CONFIGS[args.config]()
    # Weak scaling: rank r renders frame r of a short camera path (camPos drifts along x).
    scene.ubo = S.make_ubo(cam=(0.05 * rank, 0.0, 0.0))
    params = scene.params()
    rows = params.height
    pixels = rows * params.width
    envmap = bool(params.flags & T.FLAG_ENVMAP)

    r = trt.Renderer(dev)
    r.upload_scene(scene)
    out8 = torch.empty((rows, params.width, 4), dtype=torch.uint8, device="cuda")

    # Counting pass (excluded from timing): rays and per-stage work of this rank's frame.
    _, _, st = r.draw_frame(params, count=True)
    rays_per_frame = st["primary_rays"] + st["secondary_rays"]
    alg_bytes = algorithmic_bytes(st, pixels, envmap)

    # Frames are enqueued by the native frame loop (trt_render_frames: one kernel launch per
    # frame).  A HIP event pair on the kernel's own stream brackets every TIME_EVERY-th launch:
    # the kernel duration is measured live while the timed region stays nearly event-free
    # (an event pair adds ~7 us of queue time to a ~40 us frame).
    # Frames in flight (main.cpp:45, MAX_FRAMES_IN_FLIGHT = 2): frame i runs on slot
    # i % inflight, so frame i+1's tiles fill the GPU while frame i's slowest tiles finish;
    # render_frames joins every slot back into `stream` before it returns.  Every step renders
    # the same frame, so the frames share one image (the reference's single storage image,
    # main.cpp:865-926; concurrent frames write identical bytes).
    nfl = max(1, args.inflight)
    stream = torch.cuda.Stream()
    r.set_stream(stream)
    r.set_frames_in_flight(nfl)
    r.set_subtree_split(args.split)
    r.render_frames(params, out8, args.warmup)
    torch.cuda.synchronize()

    K = args.steps
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ntimed = r.render_frames(params, out8, K, timing=True, time_every=TIME_EVERY)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = r.frame_times(ntimed)
    kern_avg_ms = float(kern_ms.mean())

    total_rays = rays_per_frame
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        rr = torch.tensor([rays_per_frame], dtype=torch.float64, device="cuda")
        dist.all_reduce(rr, op=dist.ReduceOp.SUM)
        total_rays = int(rr.item())
        kk = torch.tensor([kern_avg_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(kk, op=dist.ReduceOp.MAX)
        kern_avg_ms = float(kk.item())

    value = total_rays * K / elapsed / 1e6
    ms_per_step = elapsed / K * 1e3
    tiled = None
    if args.tiled_frames > 0:
        try:
            tiled = tiled_frame(args.tiled_frames, rank, world, dist, dev)
        except Exception as e:  # the headline line is still printed; the failure is reported in it
            tiled = {"error": f"{type(e).__name__}: {e}"} if rank == 0 else None

    if rank == 0:
        achieved = alg_bytes / (kern_avg_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = Path(args.pmc) if args.pmc else REPO / "profiles" / f"pmc_{args.config}.json"
        if pmc_path.exists():
            try:
                traffic = json.loads(pmc_path.read_text()).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        result = {
            "metric": "Mray/s (primary+secondary) at 1024\u00d7768 depth4; 1/2/4/8-GPU scaling",
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded procedural envmap; reference spheres/lights/materials, main.cpp:125-143)",
            "config": {
                "workload": f"{args.config}: {WORKLOADS[args.config]}",
                "width": params.width,
                "height": params.height,
                "max_depth": params.max_depth,
                "spp": params.spp,
                "rays_per_frame": rays_per_frame,
                "shadow_rays_per_frame": st["shadow_rays"],
                "parallelism": f"frame-per-GPU x{world}" if world > 1 else "1 GPU",
                "frames_in_flight": nfl,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "trace_kernel",
                "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
                "algorithmic_bytes_per_launch": alg_bytes,
                "per_frame_rate": round(alg_bytes / (ms_per_step * 1e-3) / 1e9, 2),
                "note": "achieved = algorithmic SoA bytes (SURVEY §8d) per launch / HIP-event kernel "
                        "time on the launch's stream (with frames in flight the span includes the "
                        "overlapping frame); per_frame_rate = the same bytes / wall time per frame. "
                        "An efficiency index, not physical traffic (wave-uniform scalar/L2 reuse); "
                        "physical HBM bytes per launch = traffic (PMC FETCH_SIZE + WRITE_SIZE)",
            },
        }
        if tiled is not None:
            result["tiled_frame"] = tiled
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(scene, params, rays_per_frame, args.cpu_seconds)
        print(json.dumps(result), flush=True)

    r.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
