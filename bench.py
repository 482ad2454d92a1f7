#!/usr/bin/env python3
"""Benchmark of the hot path: Mray/s (primary + secondary) at 1024x768, depth 4 (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5|ref|readme] [--no-cpu]

One step = one frame of the configuration (C2 by default), inputs resident in HBM.

* N = 1: the frame loop of the C-ABI (trt_render_frames, 2 frames in flight) on one GPU.
* N > 1 (one process per GPU under torch.distributed.run): every frame is row-tiled over the
  N GPUs and gathered over RCCL by the native multi-GPU path (trt_render_multi_frames,
  csrc/trt_multi.cpp): strong scaling, the frame is fixed and each GPU renders 1/N of it.
  Frames are gathered in batches of --frames-per-gather on a rotating root (batch j on rank
  j % N).  The frame-per-GPU weak-scaling number is reported beside it (`weak_scaling`).

Rank 0 prints ONE JSON line.  Extra keys: `tiled_frame` (BASELINE configs[3]: a 3840x2160
~100k-triangle frame row-tiled over the N GPUs and gathered on rank 0 over RCCL, with its
SHA-256 checked against the 1-GPU frame and the committed hash), `shipped_frame` (the
reference's own default frame, config.hpp:97-101 at MAX_DEPTH 20), `readme_frame` (the scene
of the reference's only published frame rate, README.md:334-340), `roofline` (FP32 VALU:
SURVEY §8d flop units x this frame's counted work / the kernel's HIP-event launch time),
`cpu_baseline` (the CPU oracle timed on this host on the same workload).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
# frames in flight are HIP streams: 32 hardware queues (HIP's default, 4, is what the box's
# environment sets) before any HIP init in this process
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) <= 4:
    os.environ["GPU_MAX_HW_QUEUES"] = "32"

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 157.3  # MI355X FP32 vector, FMA = 2 flops (AMD spec)
TIME_EVERY = 16  # one timed (event-bracketed) launch per 16 frames
FRAME_HASHES = REPO / "tests" / "golden" / "frame_hashes.json"
METRIC = "Mray/s (primary+secondary) at 1024×768 depth4; 1/2/4/8-GPU scaling"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5", "ref", "readme"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU oracle baseline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight (trt_set_frames_in_flight: 0 = auto = 4, or 8 for deferred-shadow "
                         "frames; the reference's MAX_FRAMES_IN_FLIGHT is 2)")
    ap.add_argument("--split", type=int, default=0, help="subtree split window (trt_set_subtree_split: 0 auto, 1 off)")
    ap.add_argument("--band-rows", type=int, default=8, help="rows per band of the tiled frames")
    ap.add_argument("--frames-per-gather", type=int, default=64,
                    help="frames whose bands move in one RCCL gather (N > 1 headline)")
    ap.add_argument("--tiled-frames", type=int, default=20,
                    help="frames of the tiled 3840x2160 leg (C4 row-tiled + RCCL gather on rank 0); 0 skips it")
    ap.add_argument("--extra-frames", type=int, default=40,
                    help="frames of the shipped / README-scene legs; 0 skips them")
    return ap.parse_args()


WORKLOADS = {
    "C2": "1024x768, 4 spheres + floor + 7616x3808 seeded envmap, depth 4, 1 spp",
    "C3": "1920x1080, spheres + icosphere mesh (5,120 tris / 80 batches), depth 4",
    "C4": "3840x2160, 20 icospheres (102,400 tris / 1,600 batches), depth 4",
    "C5": "3840x2160, C4 scene, 16 jittered spp, depth 4",
    "ref": "1024x768, the shipped frame: glass + water + ice (37,956 tris / 594 batches), floor, "
           "7616x3808 seeded envmap, depth 20 (config.hpp:97-101, shader.comp:75-84)",
    "readme": "1024x768, the README-era scene: asschercut + bunny + dragon + venus + fudanlogo "
              "(53,877 tris / 844 batches, config.hpp:96), checker floor, envmap, depth 20",
}


def make_scene(name: str):
    from vkcomputeshader_tinyraytracer_amd import scene as S

    if name == "ref":
        return S.config_reference_default()
    if name == "readme":
        return S.config_readme()
    return S.CONFIGS[name]()


# ---- roofline units ---------------------------------------------------------

def algorithmic_flops(st: dict, pixels: int, envmap: bool, mesh: bool) -> int:
    """FP32 flops of the work the frame executes, in SURVEY §8(d) units: slab test 24 per box
    (BVH / hierarchy node or the reference's batch gate), Moller-Trumbore 22 / 34 / 52 / 59 by
    the stage it exits at (+27 for the hit's interpolated normal), sphere test 21, floor test 8,
    invDir 3 per mesh query, Phong 60 per light (3 lights per hit segment), background uv +
    bilinear 40 per envmap miss.  Child-ray construction and gamma are not counted; the work
    of the shadow queries the frame skips (zero contribution, counted by the counting pass) is
    subtracted."""
    queries = st["primary_rays"] + st["secondary_rays"] + st["shadow_rays"]
    scene_queries = st["primary_rays"] + st["secondary_rays"]
    hits = scene_queries - st["misses"]
    mt = (22 * st["tri_tests"] + 12 * st["tri_past_a"] + 18 * st["tri_past_u"] + 7 * st["tri_past_v"])
    total = (24 * (st["node_tests"] + st["batch_tests"]) + mt + 27 * st["tri_nearest"]
             + 21 * st["sphere_tests"] + 8 * scene_queries + (3 * queries if mesh else 0)
             + 180 * hits + (40 * st["misses"] if envmap else 0))
    # the counting pass traces the shadow queries the frame skips (zero contribution): not executed
    skipped = (24 * st["skipped_box_tests"] + 22 * st["skipped_tri_tests"] + 12 * st["skipped_tri_past_a"]
               + 18 * st["skipped_tri_past_u"] + 7 * st["skipped_tri_past_v"] + 21 * st["skipped_sphere_tests"]
               + (3 * st["shadow_skipped"] if mesh else 0))
    return int(total - skipped)


def algorithmic_bytes(st: dict, pixels: int, envmap: bool) -> int:
    """SURVEY §8(d) byte units for the data that lives in memory (sphere records and the floor /
    sphere materials are kernel arguments in SGPRs and are excluded): 24 B per box tested,
    +8 B start/count per batch passed, 36 B per triangle tested, 16 B per envmap sample,
    48 B material + 36 B vertex normals per triangle hit, 4 B written per pixel."""
    return int(24 * (st["batch_tests"] + st["node_tests"] - st["skipped_box_tests"]) + 8 * st["batch_hits"]
               + 36 * (st["tri_tests"] - st["skipped_tri_tests"])
               + (16 * st["misses"] if envmap else 0) + 84 * st["tri_nearest"] + 4 * pixels)


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


class Group:
    """torch.distributed helpers (no-ops at N = 1)."""

    def __init__(self, world: int, rank: int):
        self.world, self.rank = world, rank
        self.dist = None
        if world > 1:
            import torch
            import torch.distributed as dist

            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def sum(self, x: float) -> float:
        return self._reduce(x, "SUM")

    def _reduce(self, x: float, op: str) -> float:
        if not self.dist:
            return x
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64, device="cuda")
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return float(t.item())

    def unique_id(self) -> bytes:
        from vkcomputeshader_tinyraytracer_amd.multi import unique_id

        obj = [unique_id() if self.rank == 0 else None]
        if self.dist:
            self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def timed(g: Group, fn) -> float:
    """Barrier + synchronize on both sides; the max over ranks of the wall time."""
    import torch

    torch.cuda.synchronize()
    g.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    g.barrier()
    return g.max(time.perf_counter() - t0)


def frame_loop(dev: int, scene, frames: int, warmup: int, inflight: int, split: int, time_every: int = TIME_EVERY,
               g: Group | None = None):
    """trt_render_frames of `scene` on one GPU: (elapsed s, kernel ms per sampled launch, stats of
    a counting pass, params)."""
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt

    p = scene.params()
    r = trt.Renderer(dev)
    try:
        r.upload_scene(scene)
        r.set_subtree_split(split)
        _, _, st = r.draw_frame(p, count=True)  # counting pass, excluded from timing
        out8 = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        stream = torch.cuda.Stream()
        r.set_stream(stream)
        r.set_frames_in_flight(inflight)
        r.render_frames(p, out8, warmup)
        box = {}
        elapsed = timed(g or Group(1, 0), lambda: box.update(n=r.render_frames(p, out8, frames, timing=True,
                                                                                 time_every=time_every)))
        kern_ms = r.frame_times(box["n"])
        return elapsed, kern_ms, st, p
    finally:
        r.close()


def resolved_inflight(inflight: int, scene) -> int:
    """The library's frames in flight for this scene: the explicit count, or its auto rule (8
    for deferred-shadow frames: meshes at max_depth >= 8 and spp 1, else 4)."""
    if inflight:
        return inflight
    return 8 if (len(scene.models) > 0 and scene.max_depth >= 8 and scene.spp <= 1) else 4


def extra_frame(dev: int, name: str, frames: int, args) -> dict:
    import vkcomputeshader_tinyraytracer_amd  # noqa: F401  (lib load)

    sc = make_scene(name)
    elapsed, kern_ms, st, p = frame_loop(dev, sc, frames, 4, args.inflight, args.split, time_every=4)
    rays = st["primary_rays"] + st["secondary_rays"]
    ms = elapsed / frames * 1e3
    out = {
        "workload": f"{name}: {WORKLOADS[name]}",
        "frames": frames,
        "frames_in_flight": resolved_inflight(args.inflight, sc),
        "ms_per_frame": round(ms, 4),
        "fps": round(1e3 / ms, 2),
        "mray_s": round(rays / (ms * 1e-3) / 1e6, 3),
        "rays_per_frame": rays,
        "shadow_rays_per_frame": st["shadow_rays"],
        "shadow_rays_traced_per_frame": st["shadow_rays"] - st["shadow_skipped"],
        "kernel_span_ms": round(float(kern_ms.mean()), 4),
    }
    if name == "readme":
        out["published_context"] = {
            "fps": "10-11 (dips to 7)", "hardware": "NVIDIA GeForce RTX 4060", "source": "README.md:334-340",
            "note": "same scene and size, but an older shader state of the reference: a different-hardware "
                    "context bar, not a like-for-like baseline",
            "ratio_vs_10.5_fps": round(1e3 / ms / 10.5, 1),
        }
    return out


def tiled_stream(g: Group, dev: int, multi, scene, frames: int, warmup: int, band_rows: int, root: int,
                 per_gather: int):
    """trt_render_multi_frames of `scene` over all ranks: (elapsed s, whole-frame stats, output)."""
    import torch

    p = scene.params()
    multi.upload_scene(scene if g.rank == 0 else None)
    st = multi.draw_frame(p, band_rows=band_rows, root=0, count=True)  # counting pass (all ranks)
    out = torch.zeros((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    multi.set_stream(0, stream)
    # warmup: at least one batch of the timed batches' size, so the gather buffers are sized
    # before timing (the timed batches never allocate)
    multi.render_frames(p, max(warmup, min(frames, per_gather)), band_rows, root, per_gather, outs=[out])
    elapsed = timed(g, lambda: multi.render_frames(p, frames, band_rows, root, per_gather, outs=[out]))
    multi.set_stream(0, None)
    return elapsed, st, out, p


def tiled_frame(g: Group, dev: int, multi, frames: int, band_rows: int) -> dict:
    """BASELINE configs[3]: a 3840x2160 C4 frame row-tiled across the ranks (interleaved
    band_rows-row bands) and gathered to rank 0 as RGBA8 over RCCL (xGMI) by the native path,
    one gather per frame (the display case), two frames in flight."""
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = S.config_c4()
    elapsed, st, out, p = tiled_stream(g, dev, multi, sc, frames, 2, band_rows, 0, 1)
    rays = st["primary_rays"] + st["secondary_rays"]
    res = None
    if g.rank == 0:
        sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
        with trt.Renderer(dev) as r:  # the 1-GPU frame (trt_render of the whole frame)
            r.upload_scene(sc)
            one, _, _ = r.draw_frame(p)
        sha1 = hashlib.sha256(one.tobytes()).hexdigest()
        committed = json.loads(FRAME_HASHES.read_text()).get("C4_3840x2160") if FRAME_HASHES.exists() else None
        res = {
            "workload": "C4: 3840x2160, 20 icospheres (102,400 tris), depth 4, one frame row-tiled "
                        f"over {g.world} GPU(s) in interleaved {band_rows}-row bands, gathered on rank 0",
            "scaling": "strong",
            "collective": "RCCL grouped ncclSend/ncclRecv of the compact RGBA8 band buffers to rank 0 "
                          "(csrc/trt_multi.cpp)" + (" — 1 rank: sent to itself" if g.world == 1 else ""),
            "frames": frames,
            "ms_per_frame": round(elapsed / frames * 1e3, 4),
            "frames_per_s": round(frames / elapsed, 3),
            "mray_s": round(rays * frames / elapsed / 1e6, 3),
            "rays_per_frame": rays,
            "gather_bytes_per_frame": int(p.width * p.height * 4 * (g.world - 1) / g.world),
            "frame_sha256": sha,
            "matches_1gpu_frame": sha == sha1,
            "matches_committed_hash": (sha == committed) if committed else None,
        }
    torch.cuda.synchronize()
    return res


def main():
    args = parse()
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local if world > 1 else 0)
    dev = torch.cuda.current_device()
    g = Group(world, rank)

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import types as T
    from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, MultiRenderer

    scene = make_scene(args.config)
    K = args.steps
    envmap = bool(scene.flags & T.FLAG_ENVMAP)
    mesh = len(scene.models) > 0

    # Frame per GPU (the N = 1 headline; the weak-scaling extra at N > 1): also the live kernel
    # timing of the roofline.
    elapsed1, kern_ms, st, params = frame_loop(dev, scene, K, args.warmup, args.inflight, args.split, g=g)
    rays_per_frame = st["primary_rays"] + st["secondary_rays"]
    pixels = params.width * params.height
    kern_avg_ms = g.max(float(kern_ms.mean()))
    weak_value = g.sum(rays_per_frame) * K / elapsed1 / 1e6

    multi = MultiRenderer.for_rank(dev, world, rank, g.unique_id())
    if world == 1:
        value, ms_per_step = weak_value, elapsed1 / K * 1e3
        scaling, parallelism = "weak", "1 GPU"
        # the N > 1 headline's path (trt_render_multi_frames) at one rank: the base of its
        # strong-scaling curve, so the driver's per-N values can be read against it
        elapsed_t, mst, _, _ = tiled_stream(g, dev, multi, scene, K, args.warmup, args.band_rows, ROOT_ROTATE,
                                            args.frames_per_gather)
        rays_whole = mst["primary_rays"] + mst["secondary_rays"]
        headline_extra = {"tiled_headline_1gpu": {
            "value": round(rays_whole * K / elapsed_t / 1e6, 3), "unit": "Mray/s",
            "ms_per_step": round(elapsed_t / K * 1e3, 5),
            "workload": f"the N > 1 headline's path at 1 rank: {args.config} through trt_render_multi_frames "
                        f"({args.band_rows}-row bands, RCCL gather of {args.frames_per_gather} frames per op)"}}
    else:
        # the frame row-tiled over all GPUs, RCCL gathers of --frames-per-gather frames on a rotating root
        elapsed, mst, _, _ = tiled_stream(g, dev, multi, scene, K, args.warmup, args.band_rows, ROOT_ROTATE,
                                          args.frames_per_gather)
        rays_whole = mst["primary_rays"] + mst["secondary_rays"]
        value, ms_per_step = rays_whole * K / elapsed / 1e6, elapsed / K * 1e3
        scaling = "strong"
        parallelism = (f"row-tiled x{world} ({args.band_rows}-row interleaved bands), RCCL gather of "
                       f"{args.frames_per_gather} frames per op on a rotating root")
        headline_extra = {"weak_scaling": {
            "value": round(weak_value, 3), "unit": "Mray/s",
            "workload": f"frame per GPU: every rank renders its own whole {args.config} frame, no data-path collective",
            "ms_per_step": round(elapsed1 / K * 1e3, 5)}}

    tiled = tiled_frame(g, dev, multi, args.tiled_frames, args.band_rows) if args.tiled_frames > 0 else None
    multi.close()

    extras = {}
    if args.extra_frames > 0:
        for key, name in (("shipped_frame", "ref"), ("readme_frame", "readme")):
            if rank == 0:
                if world == 1:
                    try:
                        extras[key] = extra_frame(dev, name, args.extra_frames, args)
                    except Exception as e:  # N = 1: report the failure in the line
                        extras[key] = {"error": f"{type(e).__name__}: {e}"}
                else:  # N > 1: fail fast (the launcher tears the job down)
                    extras[key] = extra_frame(dev, name, args.extra_frames, args)
            g.barrier()

    if rank == 0:
        flops = algorithmic_flops(st, pixels, envmap, mesh)
        tflops = flops / (kern_avg_ms * 1e-3) / 1e12
        abytes = algorithmic_bytes(st, pixels, envmap)
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": scaling,
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
                "shadow_rays_traced_per_frame": st["shadow_rays"] - st["shadow_skipped"],
                "parallelism": parallelism,
                "frames_in_flight": resolved_inflight(args.inflight, scene),
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(tflops, 3),
                "peak": VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(tflops / VALU_PEAK_TFLOPS, 4),
                "traffic": None,
                "kernel": "trace_kernel",
                "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
                "flops_per_launch": flops,
                "achieved_per_frame": round(flops / (elapsed1 / K) / 1e12, 3),
                "frac_per_frame": round(flops / (elapsed1 / K) / 1e12 / VALU_PEAK_TFLOPS, 4),
                "note": "FP32 flops of the executed work in SURVEY §8d units (counting pass of this frame) / "
                        "the trace kernel's launch time (HIP events on its stream, every 16th launch of the "
                        "timed loop; with several frames in flight a launch's span includes the overlapping "
                        "frames, so *_per_frame divides by the wall time per frame instead); "
                        "peak counts an FMA as 2 flops, the kernel has no FMA contraction (-ffp-contract=off). "
                        "traffic: no PMC pass in this run (profiles/ holds the PMC summaries of this build)",
                "hbm_index": {
                    "algorithmic_bytes_per_launch": abytes,
                    "gb_s_per_launch": round(abytes / (kern_avg_ms * 1e-3) / 1e9, 2),
                    "gb_s_per_frame": round(abytes / (elapsed1 / K) / 1e9, 2),
                    "peak": HBM_PEAK_GBS,
                    "note": "SURVEY §8d bytes excluding SGPR-resident sphere records and constant materials; "
                            "an index, not measured traffic",
                },
            },
        }
        if headline_extra:
            result.update(headline_extra)
        if tiled is not None:
            result["tiled_frame"] = tiled
        result.update(extras)
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(scene, params, rays_per_frame, args.cpu_seconds)
        print(json.dumps(result), flush=True)
    g.close()


if __name__ == "__main__":
    main()
