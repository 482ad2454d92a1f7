#!/usr/bin/env python3
"""Benchmark of the hot path: Mray/s (primary + secondary) at 1024x768, depth 4 (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5|ref|readme] [--no-cpu]

Every frame has its own UBO: the camera walks like the reference's interactive loop with W and
D held (processInput + updateUniformBuffer, main.cpp:391-403, 2165-2179), cycling through
--camera-period positions whose ray counts come from one counting pass each (excluded from
timing).  Inputs are resident in HBM; the timed region only enqueues and runs frames.  Before
it, untimed frames of the same loop run for --settle-ms (default 50): the MI355X raises its
clocks over the first ~30 ms of sustained load, and a 20-step region (0.3 ms) timed from an idle
GPU measured the ramp (C2 13.7 us per frame of kernel time cold, 12.2 settled,
profiles/r04l_settle.jsonl).  The timed region itself holds exactly K full steps.

* N = 1: one step = one frame.  The value is the native frame loop (trt_render_frames: plain
  frames go out as multi-frame launches) — `path` in the line says which path produced it; the
  N > 1 path at one rank is reported beside it (`tiled_1gpu`) as the base of the scaling curve.
* N > 1 (one process per GPU under torch.distributed.run): one step = N frames, EACH row-tiled
  over all N GPUs (interleaved 8-row bands) and gathered over RCCL to its own root, rank i % N
  (trt_render_multi_frames: per-frame rotating roots, so every device's xGMI links ingest at
  once).  Per-GPU work per step is one frame's worth at every N ("scaling": "weak"); the strong
  form (one frame per step over all N GPUs) and the frame-per-GPU form (no collective) are
  reported beside it.

Rank 0 prints ONE JSON line.  Extra keys: `tiled_frame` (BASELINE configs[3]: a 3840x2160
~100k-triangle frame row-tiled over the N GPUs and gathered on rank 0 over RCCL, hash-checked
against the 1-GPU frame and the committed hash), `shipped_frame` (the reference's own default
frame, config.hpp:97-101 at MAX_DEPTH 20), `readme_frame` (the scene of the reference's only
published frame rate, README.md:334-340), `roofline` (FP32 VALU: SURVEY §8d flop units x the
counted work / wall time per frame), `cpu_baseline` (the CPU oracle on this host).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
# frames in flight are HIP streams: 32 hardware queues (HIP's default, 4, is what the box's
# environment sets) before any HIP init in this process (TRT_KEEP_HW_QUEUES=1 opts out)
from vkcomputeshader_tinyraytracer_amd._lib import raise_hw_queues  # noqa: E402

raise_hw_queues()

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 157.3  # MI355X FP32 vector, FMA = 2 flops (AMD spec)
FRAME_HASHES = REPO / "tests" / "golden" / "frame_hashes.json"
METRIC = "Mray/s (primary+secondary) at 1024×768 depth4; 1/2/4/8-GPU scaling"
RING = 256  # output images of a timed loop (frame i -> image i % RING)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5", "ref", "readme"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU oracle baseline")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget per thread count")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight (trt_set_frames_in_flight: 0 = auto; the reference's is 2)")
    ap.add_argument("--frame-batch", type=int, default=0,
                    help="frames per launch (trt_set_frame_batch: 0 = auto, 1 = one launch per frame)")
    ap.add_argument("--split", type=int, default=0, help="subtree split window (trt_set_subtree_split: 0 auto, 1 off)")
    ap.add_argument("--band-rows", type=int, default=8, help="rows per band of the tiled frames")
    ap.add_argument("--frames-per-gather", type=int, default=0,
                    help="frames per RCCL exchange of the tiled loop (0 = auto: a quarter of the frames, <= 64)")
    ap.add_argument("--camera-period", type=int, default=64,
                    help="distinct camera positions of the walk (>= the 64 frames of a launch, so no launch "
                         "traces the same frame twice: the reference's camera never revisits a position)")
    ap.add_argument("--tiled-frames", type=int, default=20,
                    help="frames of the tiled 3840x2160 leg (C4 row-tiled + RCCL gather on rank 0); 0 skips it")
    ap.add_argument("--extra-frames", type=int, default=160,
                    help="frames of the shipped / README-scene legs (16 run in flight: 160 keeps the pipeline's "
                         "fill and drain to a few per cent); 0 skips them")
    ap.add_argument("--legs", default="c3,c5,c2pf,cabi",
                    help="extra legs (comma list; '' = none): c3 = BASELINE configs[2] (1920x1080 mesh), c5 = "
                         "configs[4] (4K, 16 spp), c2pf = C2 at one launch per frame, 2 in flight (drawFrame)")
    ap.add_argument("--legs-frames", type=int, default=200, help="frames of the C3 and per-frame-launch C2 legs")
    ap.add_argument("--c5-frames", type=int, default=6, help="frames of the C5 leg (~80 ms each)")
    ap.add_argument("--traffic", default="live", choices=["live", "table", "off"],
                    help="roofline.traffic: live = two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over a "
                         "child run of the same frame loop (N = 1); table = the committed measurement")
    ap.add_argument("--settle-ms", type=float, default=50.0,
                    help="untimed frames of the timed loop's own shape for this long before the timed "
                         "region (clocks at their steady state)")
    ap.add_argument("--traffic-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N > 1 process shape (torch.distributed nccl group + trt_multi rank "
                         "communicator in one process, tiled headline) even at one rank (tests)")
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

def algorithmic_flops(st: dict, envmap: bool, mesh: bool) -> int:
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


def roofline(st_frame: dict, s_per_frame: float, envmap: bool, mesh: bool, pixels: int,
             kernel_ms_per_frame: float | None = None) -> dict:
    """FP32-VALU roofline of one frame's counted work over the wall time per frame (the wall
    clock of the timed loop / frames — never more than the time the frames took)."""
    flops = algorithmic_flops(st_frame, envmap, mesh)
    tf = flops / s_per_frame / 1e12
    out = {
        "bound": "valu", "achieved": round(tf, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": round(tf / VALU_PEAK_TFLOPS, 4), "traffic": None,
        "flops_per_frame": flops, "us_per_frame": round(s_per_frame * 1e6, 3),
    }
    if kernel_ms_per_frame is not None:
        if kernel_ms_per_frame * 1e-3 <= s_per_frame * 1.0001:
            out["kernel_us_per_frame"] = round(kernel_ms_per_frame * 1e3, 3)
            out["kernel_frac"] = round(flops / (kernel_ms_per_frame * 1e-3) / 1e12 / VALU_PEAK_TFLOPS, 4)
        else:
            # frames overlap (several in flight): a launch's span per frame is the frame's
            # latency, longer than the wall time per frame, so it prices no rate
            out["frame_span_us"] = round(kernel_ms_per_frame * 1e3, 3)
    ab = algorithmic_bytes(st_frame, pixels, envmap)
    # bytes the algorithm asks of the memory hierarchy, not HBM bytes: on mesh scenes nodes and
    # triangles are served from L1 / L2 (97 % L1 hits on C4), so this rate can exceed the HBM
    # peak; the HBM bytes are the PMC FETCH figures under profiles/
    out["request_bytes"] = {"per_frame": ab, "gb_s": round(ab / s_per_frame / 1e9, 2),
                            "note": "SURVEY 8(d) byte units requested per frame; mostly cache hits, not an HBM figure"}
    return out


def cpu_info() -> dict:
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "cgroup_cpu_quota": quota,
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def cpu_baseline(scene, params, rays_per_frame: int, budget_s: float) -> dict:
    """CPU oracle (fast mode, -O3, rows dynamically scheduled over pthreads) on this host, on
    whole frames of the same workload (camera at the walk's start): at
    std::thread::hardware_concurrency() threads and at the process's CPU share."""
    from oracle import oracle as orc

    info = cpu_info()
    hw = min(os.cpu_count() or 1, 256)  # the oracle caps its pool at 256 threads
    share = info["affinity_cpus"] or hw
    if info["cgroup_cpu_quota"]:
        share = min(share, max(1, int(info["cgroup_cpu_quota"])))

    def run(threads):
        orc.render(scene, params, threads=threads)  # warm-up (also loads/builds the library)
        times = []
        t_start = time.perf_counter()
        while len(times) < 3 or (time.perf_counter() - t_start < budget_s and len(times) < 50):
            t0 = time.perf_counter()
            _, _, st = orc.render(scene, params, threads=threads)
            times.append(time.perf_counter() - t0)
        med = statistics.median(times)
        return st["primary_rays"] + st["secondary_rays"], med, len(times)

    rays, med, n = run(hw)
    # `cores`: the CPUs the threads could actually run on — the job's cgroup quota (16 on the GPU
    # box) caps the 256 hardware threads of the host, so the thread count overstates the CPU
    cores = min(hw, share)
    out = {
        "value": round(rays / med / 1e6, 3), "unit": "Mray/s", "cores": cores, "threads": hw, "kind": "port",
        "sample": f"{n} whole frames of the same workload after 1 warm-up, median {med * 1e3:.1f} ms/frame; "
                  f"oracle/trt_oracle.c fast mode, -O3, pixel spans over {hw} threads (hardware_concurrency) "
                  f"on {cores} CPUs (min of the cgroup quota {info['cgroup_cpu_quota']} and the affinity mask) of "
                  f"a {info['model']}",
        "host": info, "rays_match_gpu": bool(rays == rays_per_frame),
    }
    if share != hw:
        r2, med2, n2 = run(share)
        out["at_cpu_share"] = {"threads": share, "value": round(r2 / med2 / 1e6, 3), "frames": n2,
                               "ms_per_frame": round(med2 * 1e3, 2)}
    return out


class Group:
    """torch.distributed helpers (no-ops at N = 1)."""

    def __init__(self, world: int, rank: int, force: bool = False):
        self.world, self.rank = world, rank
        self.dist = None
        if world > 1 or force:
            import torch
            import torch.distributed as dist

            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def min(self, x: float) -> float:
        return self._reduce(x, "MIN")

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


def settle(args, fn) -> None:
    """Runs fn (one untimed pass of the timed loop's first chunk) until args.settle_ms have passed."""
    import torch

    t_end = time.perf_counter() + max(0.0, getattr(args, "settle_ms", 0.0)) / 1e3
    while time.perf_counter() < t_end:
        fn()
        torch.cuda.synchronize()


def walk(scene, period: int):
    from vkcomputeshader_tinyraytracer_amd import camera_path

    return camera_path(scene.ubo, period)


def count_walk(r, p, walk_ubos) -> tuple[list[dict], dict]:
    """Counting pass of every camera position of the walk: (per-position stats, their mean)."""
    per = []
    for u in walk_ubos:
        r.update_ubo(u)
        _, _, st = r.draw_frame(p, count=True)
        per.append(st)
    mean = {k: sum(s[k] for s in per) / len(per) for k in per[0] if k != "kernel_ms"}
    return per, mean


def rays_of(st: dict) -> int:
    return int(st["primary_rays"] + st["secondary_rays"])


def frame_loop(dev: int, scene, frames: int, warmup: int, args, g: Group | None = None, check_last: bool = True):
    """trt_render_frames of `scene` on one GPU over the camera walk: wall time, per-frame launch
    times, the walk's counts, and whether the last timed frame equals trt_render of its UBO."""
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt

    p = scene.params()
    wk = walk(scene, args.camera_period)
    r = trt.Renderer(dev)
    try:
        r.upload_scene(scene)
        r.set_subtree_split(args.split)
        per, mean = count_walk(r, p, wk)
        rays_total = sum(rays_of(per[i % len(wk)]) for i in range(frames))
        ring = min(frames, RING)
        ubos = np.stack([wk[i % len(wk)] for i in range(frames)])
        out8 = torch.empty((ring, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
        fb = p.height * p.width * 4
        stream = torch.cuda.Stream()
        r.set_stream(stream)
        r.set_frames_in_flight(args.inflight)
        r.set_frame_batch(args.frame_batch)
        r.render_frames(p, out8, max(1, min(warmup, ring)), ubos=ubos, frame_stride=fb)
        chunks = [(i0, min(ring, frames - i0)) for i0 in range(0, frames, ring)]
        ubo_chunks = [np.ascontiguousarray(ubos[i0:i0 + n]) for i0, n in chunks]
        settle(args, lambda: r.render_frames(p, out8, chunks[0][1], ubos=ubo_chunks[0], frame_stride=fb))

        # the frame lists prepared outside the region: one native call per chunk inside it
        calls = [r.frames_call(p, out8, n, ubos=u, frame_stride=fb) for (_, n), u in zip(chunks, ubo_chunks)]

        def run():
            for call in calls:
                call()

        elapsed = timed(g or Group(1, 0), run)
        # the same loop again with HIP events around every launch (outside the timed region):
        # the device time per frame of the launches
        ms, nf = [], []
        for (_, n), u in zip(chunks, ubo_chunks):
            nt = r.render_frames(p, out8, n, ubos=u, frame_stride=fb, timing=True)
            ms.append(r.frame_times(nt))
            nf.append(r.launch_frames())
        ms = np.concatenate(ms)
        nf = np.concatenate(nf).astype(np.float64)
        kernel_ms_per_frame = float((ms * nf).sum() / nf.sum())  # launch spans / frames
        launches = int(len(nf))
        torch.cuda.synchronize()
        ok = None
        if check_last:
            last = frames - 1
            got = out8[last % ring].cpu().numpy()
            r.set_stream(None)
            r.update_ubo(ubos[last])
            want, _, _ = r.draw_frame(p)
            ok = bool(np.array_equal(got, want))
        return {"elapsed": elapsed, "rays_total": rays_total, "mean": mean, "p": p,
                "kernel_ms_per_frame": kernel_ms_per_frame, "launches": launches, "last_frame_ok": ok}
    finally:
        r.close()


def auto_per_gather(total: int, world: int, arg: int) -> int:
    if arg > 0:
        return arg
    if world == 1:  # nothing travels at one rank: one batch of multi-frame launches
        return max(1, min(64, total))
    return max(1, min(64, -(-total // 4)))  # >= 4 exchanges pipeline in the timed region


def tiled_loop(g: Group, dev: int, multi, scene, frames: int, warmup: int, args, per_gather: int, root: int):
    """trt_render_multi_frames over all ranks along the camera walk: frame i row-tiled over the
    ranks and assembled on rank frame_root(i): (elapsed s, rays of all frames, walk mean stats,
    last-frame check on every rank that rooted frames)."""
    import numpy as np
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd.multi import frame_root

    p = scene.params()
    wk = walk(scene, args.camera_period)
    multi.upload_scene(scene if g.rank == 0 else None)
    per = []
    for u in wk:  # counting passes (all ranks), excluded from timing
        multi.update_ubo(u)
        per.append(multi.draw_frame(p, band_rows=args.band_rows, root=0, count=True))
    mean = {k: sum(s[k] for s in per) / len(per) for k in per[0] if k != "kernel_ms"}
    rays_total = sum(rays_of(per[i % len(wk)]) for i in range(frames))
    ring = min(frames, RING - RING % g.world)  # a multiple of the ranks: frame i keeps root i % N
    ubos = np.stack([wk[i % len(wk)] for i in range(frames)])
    fb = p.height * p.width * 4
    out = torch.zeros((ring, p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill ran on the default stream: order it before the frames
    stream = torch.cuda.Stream()
    multi.set_stream(0, stream)
    # warmup: one exchange of the timed size, so the timed batches never allocate
    multi.render_frames(p, max(min(warmup, ring), min(per_gather, ring)), args.band_rows, root, per_gather,
                        outs=[out], frame_stride=fb, ubos=ubos)

    chunks = [(i0, min(ring, frames - i0)) for i0 in range(0, frames, ring)]
    ubo_chunks = [np.ascontiguousarray(ubos[i0:i0 + n]) for i0, n in chunks]

    # the frame lists prepared once: one native call per chunk in the timed region
    calls = [multi.frames_call(p, n, args.band_rows, root, per_gather, outs=[out], frame_stride=fb, ubos=u)
             for (_, n), u in zip(chunks, ubo_chunks)]
    chunk0 = calls[0]

    # settle: the same number of untimed passes on every rank (they exchange), sized from the
    # slowest rank's time for one pass (after the allocating warmup above)
    if args.settle_ms > 0:
        t0 = time.perf_counter()
        chunk0()
        torch.cuda.synchronize()
        t_chunk = max(g.max(time.perf_counter() - t0), 1e-4)
        for _ in range(int(np.ceil(args.settle_ms / 1e3 / t_chunk))):
            chunk0()
        torch.cuda.synchronize()

    def run():
        for call in calls:
            call()

    elapsed = timed(g, run)
    multi.set_stream(0, None)
    # the last frame this rank assembled vs trt_render of its UBO on this GPU
    mine = [i for i in range(frames) if frame_root(i % ring, g.world, root) == g.rank]
    ok = 1.0
    if mine:
        last = mine[-1]
        got = out[last % ring].cpu().numpy()
        with trt.Renderer(dev) as r:
            r.upload_scene(scene)
            r.update_ubo(ubos[last])
            want, _, _ = r.draw_frame(p)
        ok = 1.0 if np.array_equal(got, want) else 0.0
    ok = g.min(ok)
    return elapsed, rays_total, mean, bool(ok > 0.5)


def extra_frame(dev: int, name: str, frames: int, args) -> dict:
    sc = make_scene(name)
    res = frame_loop(dev, sc, frames, 4, args)
    ms = res["elapsed"] / frames * 1e3
    mean = res["mean"]
    p = res["p"]
    out = {
        "workload": f"{name}: {WORKLOADS[name]}; camera walk of {args.camera_period} positions",
        "frames": frames,
        "ms_per_frame": round(ms, 4),
        "fps": round(1e3 / ms, 2),
        "mray_s": round(res["rays_total"] / res["elapsed"] / 1e6, 3),
        "rays_per_frame": round(res["rays_total"] / frames, 1),
        "shadow_rays_per_frame": round(mean["shadow_rays"], 1),
        "shadow_rays_traced_per_frame": round(mean["shadow_rays"] - mean["shadow_skipped"], 1),
        "launches": res["launches"],
        "last_frame_matches_trt_render": res["last_frame_ok"],
        "roofline": roofline(mean, ms * 1e-3, True, True, p.width * p.height, res["kernel_ms_per_frame"]),
    }
    if args.inflight == 0:
        # the reference's frame pacing: MAX_FRAMES_IN_FLIGHT = 2 (main.cpp:45)
        a2 = argparse.Namespace(**vars(args))
        a2.inflight = 2
        r2 = frame_loop(dev, sc, frames, 4, a2)
        ms2 = r2["elapsed"] / frames * 1e3
        out["at_2_in_flight"] = {
            "note": "MAX_FRAMES_IN_FLIGHT = 2 (main.cpp:45), the reference's pacing; the leg above runs the "
                    "library's auto shape (deferred-shadow frames: 8 slots x 3-frame groups with 32 hardware queues)",
            "ms_per_frame": round(ms2, 4), "fps": round(1e3 / ms2, 2),
            "mray_s": round(r2["rays_total"] / r2["elapsed"] / 1e6, 3),
            "latency_ms": round(r2["kernel_ms_per_frame"], 4),
            "last_frame_matches_trt_render": r2["last_frame_ok"],
        }
        out["latency_ms"] = round(res["kernel_ms_per_frame"], 4)
    if name == "readme":
        out["published_context"] = {
            "fps": "10-11 (dips to 7)", "hardware": "NVIDIA GeForce RTX 4060", "source": "README.md:334-340",
            "note": "same scene and size, but an older shader state of the reference: a different-hardware "
                    "context bar, not a like-for-like baseline",
            "ratio_vs_10.5_fps": round(1e3 / ms / 10.5, 1),
        }
    return out


def tiled_frame(g: Group, dev: int, multi, frames: int, args) -> dict | None:
    """BASELINE configs[3]: a 3840x2160 C4 frame row-tiled across the ranks (interleaved
    band_rows-row bands) and gathered to rank 0 as RGBA8 over RCCL (xGMI) by the native path,
    one exchange per frame (the display case)."""
    import torch

    import vkcomputeshader_tinyraytracer_amd as trt
    from vkcomputeshader_tinyraytracer_amd import scene as S

    sc = S.config_c4()
    p = sc.params()
    multi.upload_scene(sc if g.rank == 0 else None)
    st = multi.draw_frame(p, band_rows=args.band_rows, root=0, count=True)
    out = torch.zeros((p.height, p.width, 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    multi.set_stream(0, stream)
    t0 = time.perf_counter()
    multi.render_frames(p, 2, args.band_rows, 0, 1, outs=[out])
    torch.cuda.synchronize()
    t_frame = max(g.max(time.perf_counter() - t0) / 2, 1e-4)
    if args.settle_ms > 0:  # the same untimed frame count on every rank (they exchange)
        multi.render_frames(p, int(min(1000, -(-args.settle_ms / 1e3 // t_frame))), args.band_rows, 0, 1, outs=[out])
        torch.cuda.synchronize()
    elapsed = timed(g, lambda: multi.render_frames(p, frames, args.band_rows, 0, 1, outs=[out]))
    multi.set_stream(0, None)
    rays = rays_of(st)
    res = None
    if g.rank == 0:
        sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
        with trt.Renderer(dev) as r:  # the 1-GPU frame (trt_render of the whole frame)
            r.upload_scene(sc)
            one, _, _ = r.draw_frame(p)
        sha1 = hashlib.sha256(one.tobytes()).hexdigest()
        committed = json.loads(FRAME_HASHES.read_text()).get("C4_3840x2160") if FRAME_HASHES.exists() else None
        ms = elapsed / frames * 1e3
        res = {
            "workload": "C4: 3840x2160, 20 icospheres (102,400 tris), depth 4, one frame row-tiled "
                        f"over {g.world} GPU(s) in interleaved {args.band_rows}-row bands, gathered on rank 0",
            "scaling": "strong",
            "collective": ("RCCL grouped ncclSend/ncclRecv of the compact RGBA8 band buffers to rank 0 "
                           "(csrc/trt_multi.cpp, plan csrc/band_plan.cpp)") if g.world > 1 else
                          "none at 1 rank: rank 0 traces every band in place, nothing travels",
            "frames": frames,
            "ms_per_frame": round(ms, 4),
            "frames_per_s": round(frames / elapsed, 3),
            "mray_s": round(rays * frames / elapsed / 1e6, 3),
            "rays_per_frame": rays,
            "gather_bytes_per_frame": int(p.width * p.height * 4 * (g.world - 1) / g.world),
            "frame_sha256": sha,
            "matches_1gpu_frame": sha == sha1,
            "matches_committed_hash": (sha == committed) if committed else None,
            "committed_hash_note": "regression check: the committed hash is this kernel's own earlier output, "
                                   "not an independent reference (C4 parity vs the oracle: tests/test_gpu_fullres.py)",
            "roofline": roofline(st, ms * 1e-3, True, True, p.width * p.height),
        }
    torch.cuda.synchronize()
    return res


def count_first(dev: int, scene) -> dict:
    """Counting pass of the scene's own UBO (the camera the CPU baseline renders)."""
    import vkcomputeshader_tinyraytracer_amd as trt

    with trt.Renderer(dev) as r:
        r.upload_scene(scene)
        _, _, st = r.draw_frame(scene.params(), count=True)
    return st

# ---- physical HBM traffic (roofline.traffic) --------------------------------------------------

TRAFFIC_TABLE = REPO / "profiles" / "r04_traffic_table.json"


def traffic_probe(args) -> None:
    """Child of measure_traffic, run under rocprofv3 --pmc: the N = 1 frame loop of the line
    (same scene, camera walk, frames per launch) and nothing else."""
    import torch

    torch.cuda.set_device(0)
    scene = make_scene(args.config)
    res = frame_loop(0, scene, args.steps, args.warmup, args, check_last=False)
    print(json.dumps({"probe_frames": args.steps, "launches": res["launches"]}), flush=True)


def probe_steps(args) -> int:
    """Frames of the probe: one timed-size launch (the auto frame batch caps a launch at 64)."""
    return max(1, min(args.steps, 64))


def _pmc_pass(counter: str, args, outdir: Path) -> list[dict]:
    """One rocprofv3 PMC pass (one counter, --kernel-trace only) over the probe; returns the
    per-dispatch records of the non-counting trace_kernel launches."""
    import csv
    import re
    import subprocess

    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", str(outdir),
           "-o", "run", "--", sys.executable, str(REPO / "bench.py"), "--traffic-probe", "--config", args.config,
           "--steps", str(probe_steps(args)), "--warmup", str(args.warmup), "--inflight", str(args.inflight),
           "--frame-batch", str(args.frame_batch), "--camera-period", str(args.camera_period), "--settle-ms", "0"]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    subprocess.run(cmd, check=True, timeout=240, env=env, cwd="/tmp", stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)
    rows: dict = {}
    for f in outdir.rglob("run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "trace_kernel" not in name or re.search(r"trace_kernel<\d+, true", name):
                continue  # counting passes are not the timed kernel
            d = rows.setdefault(r["Dispatch_Id"], {"grid": int(r["Grid_Size"]), "dur_ns":
                                                  int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "value": 0.0})
            if r["Counter_Name"] == counter:
                d["value"] += float(r["Counter_Value"])
    return list(rows.values())


def probe_args(args, **over) -> argparse.Namespace:
    """The traffic probe's arguments: the line's own, with a leg's overrides (config, steps,
    inflight, frame_batch, camera_period)."""
    a = argparse.Namespace(**vars(args))
    for k, v in over.items():
        setattr(a, k, v)
    return a


def measure_traffic(args, kernel_us_per_frame: float | None, table_key: str | None = None) -> dict | None:
    """Memory-side bytes per frame of the dominant kernel, from two separate PMC passes
    (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md §HBM: the two cannot share a pass) over a child
    run of the line's own frame loop; the launches of the timed size (the largest grid) are kept.
    FETCH_SIZE and WRITE_SIZE are KiB.  The guide's gfx950 note (FETCH_SIZE counts half the bytes
    of a wide coalesced streaming read) holds for this tracer's gathers too: calibrated with
    tools/calib/fetch_calib.hip (profiles/r05j_fetch_calibration_aligned.log), every 128-B line a
    dispatch touches is ONE request counted as 64 B, whether one 16-B lane, both 64-B halves or
    all 128 B of it are read.  So traffic = 2 x FETCH + WRITE (the raw figures are kept beside it)."""
    import shutil
    import tempfile

    if args.traffic == "off":
        return None
    if args.traffic == "live" and shutil.which("rocprofv3"):
        try:
            with tempfile.TemporaryDirectory(prefix="trt_pmc_") as td:
                fetch = _pmc_pass("FETCH_SIZE", args, Path(td) / "fetch")
                write = _pmc_pass("WRITE_SIZE", args, Path(td) / "write")
            gmax = max(d["grid"] for d in fetch)
            f_sel = [d["value"] for d in fetch if d["grid"] == gmax]
            w_sel = [d["value"] for d in write if d["grid"] == gmax]
            dur = [d["dur_ns"] for d in fetch + write if d["grid"] == gmax]
            frames = probe_steps(args) if args.frame_batch == 0 else min(probe_steps(args), args.frame_batch)
            fetch_b = statistics.median(f_sel) * 1024 / frames
            write_b = statistics.median(w_sel) * 1024 / frames
            out = {"source": f"live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over a child run of "
                             f"this frame loop ({args.config}, frame batch {args.frame_batch or 'auto'}, "
                             f"{args.inflight or 'auto'} in flight), {len(f_sel)}+{len(w_sel)} launches of {frames} "
                             f"frame(s)",
                   "fetch_bytes_raw": round(fetch_b), "write_bytes": round(write_b),
                   "launch_us_under_pmc": round(statistics.median(dur) / 1e3, 3)}
        except Exception as e:  # the committed table stands in
            out = {"live_error": f"{type(e).__name__}: {e}"}
    else:
        out = {}
    if "fetch_bytes_raw" not in out:
        if not TRAFFIC_TABLE.exists():
            return out or None
        t = json.loads(TRAFFIC_TABLE.read_text()).get(table_key or args.config)
        if not t:
            return out or None
        out.update({"source": f"table: {TRAFFIC_TABLE.relative_to(REPO)} ({t.get('measured', '')})",
                    "fetch_bytes_raw": t["fetch_bytes_raw"], "write_bytes": t["write_bytes"]})
    out["bytes_per_frame"] = 2 * out["fetch_bytes_raw"] + out["write_bytes"]
    out["fetch_correction"] = ("x2: each 128-B line read is one request counted as 64 B, for streams and for this "
                               "kernel's gathers alike (tools/calib/fetch_calib.hip)")
    if kernel_us_per_frame:
        gbs = out["bytes_per_frame"] / (kernel_us_per_frame * 1e-6) / 1e9
        out["hbm_gb_s"] = round(gbs, 1)
        out["hbm_frac"] = round(gbs / HBM_PEAK_GBS, 4)
    return out


def attach_traffic(rl: dict, td: dict | None) -> None:
    """roofline.traffic (+ traffic_detail) of a leg from measure_traffic."""
    if td and "hbm_gb_s" in td:
        td["time_basis"] = "kernel" if rl.get("kernel_us_per_frame") else "wall"
    if td and "bytes_per_frame" in td:
        rl["traffic"] = td["bytes_per_frame"]
    rl["traffic_detail"] = td


# ---- the shipped frame through the C++ host at the reference host's defaults -----------------

DROPIN_HOST = REPO / "tests" / "native" / "drop_in_host"
DROPIN_DUMP = REPO / "tests" / "golden" / "dropin_meshes.bin"


def c_abi_leg(frames: int) -> dict:
    """The shipped frame (depth 20) through the C-ABI from a plain C++ process
    (tests/native/drop_in_host --bench: the INTEGRATION.md §2 binding, no Python in the process),
    once with the environment the reference's own host would start with — GPU_MAX_HW_QUEUES
    unset, i.e. HIP's default of 4 hardware queues, the library's automatic in-flight count — and
    once with 32 queues (what the Python package and this bench export)."""
    out = {"note": "tests/native/drop_in_host --bench: trt_render_frames of the camera walk (auto in-flight "
                   "count) and trt_render per frame into host memory (drawFrame pacing)"}
    for key, queues, inflight in (("default_env", None, 0), ("queues_32", "32", 0)):
        env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "LD_LIBRARY_PATH")}
        if queues:
            env["GPU_MAX_HW_QUEUES"] = queues
        r = subprocess.run([str(DROPIN_HOST), "--bench", str(DROPIN_DUMP), str(frames), str(inflight)],
                           capture_output=True, text=True, timeout=600, env=env)
        if r.returncode != 0:
            out[key] = {"error": r.stderr[-500:]}
            continue
        line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and "bench" in x][-1]
        out[key] = {k: line[k] for k in ("gpu_max_hw_queues", "in_flight_setting", "ms_per_frame", "fps",
                                         "draw_frame_ms", "frames")}
    return out


# ---- the BASELINE configs[2] / configs[4] legs and the drawFrame-paced C2 leg -----------------

def config_leg(dev: int, name: str, frames: int, args, period: int) -> dict:
    """C3 or C5 on one GPU: the plain frame loop over a camera walk of `period` positions, with
    its roofline and live PMC traffic (BASELINE configs[2] / configs[4]; C5 is the config BASELINE
    names for the HBM-roofline report)."""
    a = probe_args(args, camera_period=period, inflight=0, frame_batch=0)
    sc = make_scene(name)
    res = frame_loop(dev, sc, frames, 2, a)
    ms = res["elapsed"] / frames * 1e3
    p = res["p"]
    rl = roofline(res["mean"], ms * 1e-3, True, True, p.width * p.height, res["kernel_ms_per_frame"])
    rl["kernel"] = "trace_kernel"
    attach_traffic(rl, measure_traffic(probe_args(a, config=name, steps=min(frames, 64), warmup=1),
                                       rl.get("kernel_us_per_frame") or rl["us_per_frame"]))
    return {
        "workload": f"{name}: {WORKLOADS[name]}; camera walk of {period} positions",
        "frames": frames, "ms_per_frame": round(ms, 4), "fps": round(1e3 / ms, 3),
        "mray_s": round(res["rays_total"] / res["elapsed"] / 1e6, 3),
        "rays_per_frame": round(res["rays_total"] / frames, 1),
        "shadow_rays_traced_per_frame": round(res["mean"]["shadow_rays"] - res["mean"]["shadow_skipped"], 1),
        "launches": res["launches"], "last_frame_matches_trt_render": res["last_frame_ok"],
        "roofline": rl,
    }


def c2_per_frame_leg(dev: int, frames: int, args) -> dict:
    """C2 at the reference's pacing: one launch per frame (drawFrame records one vkCmdDispatch per
    frame, main.cpp:2108-2131, 2181-2205) with MAX_FRAMES_IN_FLIGHT = 2 (main.cpp:45), beside the
    headline's multi-frame launches."""
    a = probe_args(args, frame_batch=1, inflight=2)
    sc = make_scene("C2")
    res = frame_loop(dev, sc, frames, 4, a)
    ms = res["elapsed"] / frames * 1e3
    p = res["p"]
    rl = roofline(res["mean"], ms * 1e-3, True, False, p.width * p.height, res["kernel_ms_per_frame"])
    rl["kernel"] = "trace_kernel"
    attach_traffic(rl, measure_traffic(probe_args(a, config="C2", steps=min(frames, 64), warmup=4),
                                       rl.get("kernel_us_per_frame") or rl["us_per_frame"], "C2_per_frame"))
    return {
        "workload": f"C2: {WORKLOADS['C2']}; one launch per frame, 2 frames in flight (main.cpp:45, 2181-2205)",
        "frames": frames, "ms_per_frame": round(ms, 5), "us_per_frame": round(ms * 1e3, 3),
        "mray_s": round(res["rays_total"] / res["elapsed"] / 1e6, 3),
        "launches": res["launches"], "last_frame_matches_trt_render": res["last_frame_ok"],
        "launch_span_us": round(res["kernel_ms_per_frame"] * 1e3, 3),
        "roofline": rl,
    }


def main():
    args = parse()
    if args.traffic_probe:
        traffic_probe(args)
        return
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_mode = world > 1 or args.force_dist  # the N > 1 process shape (also at one rank: tests)
    torch.cuda.set_device(local if world > 1 else 0)
    dev = torch.cuda.current_device()
    g = Group(world, rank, args.force_dist)

    from vkcomputeshader_tinyraytracer_amd import types as T
    from vkcomputeshader_tinyraytracer_amd.multi import ROOT_ROTATE, MultiRenderer

    scene = make_scene(args.config)
    K = args.steps
    envmap = bool(scene.flags & T.FLAG_ENVMAP)
    mesh = len(scene.models) > 0
    pixels = scene.width * scene.height

    # Frame per GPU: the plain frame loop on every rank, no data-path collective (the N = 1
    # value; at N > 1 the frame-per-GPU extra).  Also the live launch timing.
    fl = frame_loop(dev, scene, K, args.warmup, args, g=g)
    plain_value = g.sum(fl["rays_total"]) / fl["elapsed"] / 1e6
    plain_ok = g.min(1.0 if fl["last_frame_ok"] else 0.0) > 0.5

    multi = MultiRenderer.for_rank(dev, world, rank, g.unique_id())
    # the tiled loop: N frames per step (weak), each row-tiled over all N GPUs, rotating roots
    t_frames = K * world
    fpg = auto_per_gather(t_frames, world, args.frames_per_gather)
    el_t, rays_t, mean_t, tiled_ok = tiled_loop(g, dev, multi, scene, t_frames, args.warmup, args, fpg, ROOT_ROTATE)
    tiled_value = rays_t / el_t / 1e6
    tiled = {
        "value": round(tiled_value, 3), "unit": "Mray/s", "ms_per_step": round(el_t / K * 1e3, 5),
        "frames": t_frames, "frames_per_gather": fpg, "last_frames_match_trt_render": tiled_ok,
        "path": "trt_render_multi_frames: every frame row-tiled over all ranks in interleaved "
                f"{args.band_rows}-row bands, RCCL exchange of {fpg} frames per op to per-frame rotating roots "
                "(frame i -> rank i % N)" + (" — 1 rank: every band traced in place, nothing travels"
                                             if world == 1 else ""),
    }
    extra = {}
    if not dist_mode:
        value, ms_per_step, scaling = plain_value, fl["elapsed"] / K * 1e3, "weak"
        path = "trt_render_frames (plain frame loop, multi-frame launches)"
        parallelism = "1 GPU"
        extra["tiled_1gpu"] = dict(tiled, note="the N > 1 headline's path at one rank: the base of the scaling curve")
        st_frame, s_frame = fl["mean"], fl["elapsed"] / K
    else:
        value, ms_per_step, scaling = tiled_value, el_t / K * 1e3, "weak"
        path = tiled["path"]
        parallelism = (f"{world} frames per step, each row-tiled x{world} ({args.band_rows}-row interleaved bands), "
                       "RCCL exchange to per-frame rotating roots")
        extra["frame_per_gpu"] = {
            "value": round(plain_value, 3), "unit": "Mray/s", "ms_per_step": round(fl["elapsed"] / K * 1e3, 5),
            "workload": f"every rank renders its own whole {args.config} frames, no data-path collective",
            "last_frame_ok": plain_ok}
        # strong form: one frame per step over all N GPUs
        fpg1 = auto_per_gather(K, world, args.frames_per_gather)
        el_s, rays_s, _, ok_s = tiled_loop(g, dev, multi, scene, K, args.warmup, args, fpg1, ROOT_ROTATE)
        extra["strong_scaling"] = {
            "value": round(rays_s / el_s / 1e6, 3), "unit": "Mray/s", "ms_per_step": round(el_s / K * 1e3, 5),
            "frames": K, "frames_per_gather": fpg1, "last_frames_match_trt_render": ok_s,
            "workload": "one frame per step, row-tiled over all ranks (total work fixed as N grows)"}
        # single-root forms: every frame assembled on rank 0, as the reference presents every frame
        # from one queue (main.cpp:2207-2272); weak (N frames per step) and strong (one)
        el_f, rays_f, _, ok_f = tiled_loop(g, dev, multi, scene, t_frames, args.warmup, args, fpg, 0)
        el_fs, rays_fs, _, ok_fs = tiled_loop(g, dev, multi, scene, K, args.warmup, args, fpg1, 0)
        extra["fixed_root"] = {
            "weak": {"value": round(rays_f / el_f / 1e6, 3), "unit": "Mray/s", "ms_per_step": round(el_f / K * 1e3, 5),
                     "frames": t_frames, "frames_per_gather": fpg, "last_frames_match_trt_render": ok_f},
            "strong": {"value": round(rays_fs / el_fs / 1e6, 3), "unit": "Mray/s",
                       "ms_per_step": round(el_fs / K * 1e3, 5), "frames": K, "frames_per_gather": fpg1,
                       "last_frames_match_trt_render": ok_fs},
            "workload": "every frame row-tiled over all ranks and gathered on rank 0 (the display GPU)"}
        st_frame, s_frame = mean_t, el_t / t_frames * world  # per-GPU wall time per frame of work

    tiled_c4 = tiled_frame(g, dev, multi, args.tiled_frames, args) if args.tiled_frames > 0 else None
    multi.close()

    extras = {}
    if args.extra_frames > 0:
        for key, name in (("shipped_frame", "ref"), ("readme_frame", "readme")):
            if rank == 0:
                if not dist_mode:
                    try:
                        extras[key] = extra_frame(dev, name, args.extra_frames, args)
                    except Exception as e:  # N = 1: report the failure in the line
                        extras[key] = {"error": f"{type(e).__name__}: {e}"}
                else:  # N > 1: fail fast (the launcher tears the job down)
                    extras[key] = extra_frame(dev, name, args.extra_frames, args)
            g.barrier()

    legs = [x for x in args.legs.split(",") if x] if (rank == 0 and not dist_mode) else []
    for leg in legs:
        key = {"c3": "c3_frame", "c5": "c5_frame", "c2pf": "c2_per_frame_launch", "cabi": "shipped_frame_c_abi"}.get(leg)
        if key is None:
            continue
        try:
            if leg == "c3":
                extras[key] = config_leg(dev, "C3", args.legs_frames, args, min(args.camera_period, 64))
            elif leg == "c5":
                extras[key] = config_leg(dev, "C5", args.c5_frames, args, max(1, args.c5_frames))
            elif leg == "cabi":
                extras[key] = c_abi_leg(args.extra_frames)
            else:
                extras[key] = c2_per_frame_leg(dev, args.legs_frames, args)
        except Exception as e:  # N = 1: report the failure in the line
            extras[key] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        rl = roofline(st_frame, s_frame, envmap, mesh, pixels, fl["kernel_ms_per_frame"] if not dist_mode else None)
        rl["kernel"] = "trace_kernel"
        rl["note"] = ("FP32 flops of one frame's executed work in SURVEY §8d units (counting passes of the camera "
                      "walk, mean per frame) / the wall time per frame of the timed loop (at N > 1: per GPU); "
                      "kernel_us_per_frame = HIP-event span of every launch / the frames it traced (one launch "
                      "traces many frames), from a second, untimed pass of the same loop.  Peak counts an FMA "
                      "as 2 flops; the kernel has no FMA contraction "
                      "(-ffp-contract=off).  traffic: memory-side bytes per frame of trace_kernel from PMC "
                      "(2 x FETCH_SIZE + WRITE_SIZE: a 128-B line read is one request counted as 64 B, calibrated "
                      "for this kernel's gathers in tools/calib/fetch_calib.hip; see traffic_detail)")
        if not dist_mode:
            # over the kernel time per frame, or the wall time per frame when the event pass's
            # span is not the shorter one (then the rate is a lower bound)
            attach_traffic(rl, measure_traffic(args, rl.get("kernel_us_per_frame") or rl["us_per_frame"]))
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
            "data": "synthetic (seeded procedural envmap; reference spheres/lights/materials, main.cpp:125-143; "
                    f"camera walk of {args.camera_period} positions, main.cpp:391-403)",
            "path": path,
            "config": {
                "workload": f"{args.config}: {WORKLOADS[args.config]}",
                "width": scene.width,
                "height": scene.height,
                "max_depth": scene.max_depth,
                "spp": scene.spp,
                "rays_per_frame": round(fl["rays_total"] / K, 1),
                "shadow_rays_per_frame": round(fl["mean"]["shadow_rays"], 1),
                "shadow_rays_traced_per_frame": round(fl["mean"]["shadow_rays"] - fl["mean"]["shadow_skipped"], 1),
                "parallelism": parallelism,
                "frames_per_step": world,
                "launches": fl["launches"],
                "settle_ms": args.settle_ms,
                "last_frame_matches_trt_render": plain_ok if not dist_mode else tiled_ok,
                "value_form": "frame per GPU, plain loop" if not dist_mode else
                              "weak: N frames per step, each row-tiled over all ranks, rotating roots",
            },
            "roofline": rl,
        }
        result.update(extra)
        if tiled_c4 is not None:
            result["tiled_frame"] = tiled_c4
        result.update(extras)
        if not dist_mode and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(scene, scene.params(), rays_of(count_first(dev, scene)),
                                                  args.cpu_seconds)
        print(json.dumps(result), flush=True)
    g.close()


if __name__ == "__main__":
    main()
