#!/usr/bin/env bash
# Per-launch fixed cost of multi-frame launches: C2 at F frames per launch (one launch per
# timed batch), kernel time per frame from HIP events.  Fitting t(F) = s * F + X gives the
# steady per-frame cost s and the per-launch ramp + tail X.
#   CFG=C2 FRAMES="1 2 4 8 16 20 32 64" ROUNDS=2 tools/launch_tail_probe.sh
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for f in ${FRAMES:-1 2 4 8 16 20 32 64}; do
    out=$(TRT_LIB=${LIB:-} timeout -k 10 120 python tools/kbench.py --config "${CFG:-C2}" --frames "$((f * 4))" --frame-batch "$f" \
          --inflight 1 --tag "F$f" 2>/dev/null | tail -1)
    rc=$?
    [ $rc -ge 124 ] && { echo "timeout/crash rc=$rc (F=$f)"; exit $rc; }
    python3 -c "
import json,sys
d=json.loads(sys.argv[1]); f=int(sys.argv[2])
print(f\"round=$r F={f:3d} kernel_us_per_frame={d['med_us']:8.2f} launch_us={d['med_us']*f:9.1f} wall_us_per_frame={d['wall_us_no_events']:8.2f}\")" "$out" "$f"
  done
done
