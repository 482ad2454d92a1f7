#!/usr/bin/env bash
# A/B of multi-frame launches x frames in flight on the plain C2 loop and the tiled path at one
# rank, at the driver's 20 steps and at 1000 (one bench process per point; prints value, wall
# per frame and kernel span per frame).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for steps in 20 1000; do
  for fl in ${INFLIGHTS:-1 2 3 4}; do
    for fb in ${BATCHES:-0 1 8}; do
      out=$(timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu --extra-frames 0 --tiled-frames 0 \
            --inflight $fl --frame-batch $fb 2>/dev/null | tail -1)
      rc=$?
      [ $rc -ge 124 ] && { echo "timeout/crash rc=$rc"; exit $rc; }
      python3 - "$steps" "$fl" "$fb" "$out" <<'PY'
import json, sys
steps, fl, fb, line = sys.argv[1:5]
d = json.loads(line)
r = d["roofline"]
t = d.get("tiled_1gpu", {})
print(f"steps={steps:>4} inflight={fl} batch={fb:>2} launches={d['config']['launches']:>4} "
      f"plain={d['value']:>9.0f} Mray/s {r['us_per_frame']:>7.2f} us/f kspan={r.get('kernel_us_per_frame', 0):>7.2f} | "
      f"tiled1={t.get('value', 0):>9.0f} ({t.get('ms_per_step', 0) * 1e3:.2f} us/f) ok={d['config']['last_frame_matches_trt_render']}")
PY
    done
  done
done
