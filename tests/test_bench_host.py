"""bench.py's host logic (no GPU): the roofline units and the physical-traffic fallback."""
from __future__ import annotations

import argparse
import importlib.util
import json
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_traffic_table_fallback():
    """--traffic table: memory-side bytes per frame = 2 x FETCH_SIZE + WRITE_SIZE of the committed
    PMC measurement (a 128-B line read is one request counted as 64 B, for the kernel's gathers as
    for streams: tools/calib/fetch_calib.hip), and the fraction of the 8 TB/s peak."""
    b = _bench()
    t = json.loads((REPO / "profiles" / "r04_traffic_table.json").read_text())["C2"]
    args = argparse.Namespace(traffic="table", config="C2", steps=20, frame_batch=0)
    out = b.measure_traffic(args, 14.0)
    # a 128-B line read is one request counted as 64 B (tools/calib/fetch_calib.hip)
    assert out["bytes_per_frame"] == 2 * t["fetch_bytes_raw"] + t["write_bytes"]
    assert out["source"].startswith("table: profiles/r04_traffic_table.json")
    assert abs(out["hbm_gb_s"] - out["bytes_per_frame"] / 14.0e-6 / 1e9) < 0.1
    assert 0.0 < out["hbm_frac"] < 1.0
    assert b.measure_traffic(argparse.Namespace(traffic="off"), 14.0) is None


def test_probe_is_one_timed_size_launch():
    b = _bench()
    assert b.probe_steps(argparse.Namespace(steps=20)) == 20
    assert b.probe_steps(argparse.Namespace(steps=1000)) == 64


def test_roofline_units():
    """SURVEY 8(d) flop units on a hand-made counter set."""
    b = _bench()
    st = {k: 0 for k in ("primary_rays", "secondary_rays", "shadow_rays", "misses", "tri_tests", "tri_past_a",
                         "tri_past_u", "tri_past_v", "node_tests", "batch_tests", "tri_nearest", "sphere_tests",
                         "skipped_box_tests", "skipped_tri_tests", "skipped_tri_past_a", "skipped_tri_past_u",
                         "skipped_tri_past_v", "skipped_sphere_tests", "shadow_skipped", "batch_hits")}
    st.update(primary_rays=10, misses=4, sphere_tests=40)
    # 10 queries: 8 (floor) each, 21 per sphere test, 180 (3 lights x 60) per hit, 40 per envmap miss
    assert b.algorithmic_flops(st, envmap=True, mesh=False) == 10 * 8 + 40 * 21 + 6 * 180 + 4 * 40
    rl = b.roofline(st, 1e-6, True, False, 100)
    assert rl["bound"] == "valu" and rl["peak"] == b.VALU_PEAK_TFLOPS and rl["traffic"] is None
