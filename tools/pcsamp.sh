#!/usr/bin/env bash
# PC sampling (rocprofv3, stochastic hardware sampling on gfx950) of the C2 frame loop and of the
# shipped frame: which instructions the waves sit on.  Output: gpurun_out/<tag>/pcs_<cfg>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-pcs}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CFGS:-C2 ref}; do
  fb=""; [ "$cfg" = C2 ] && fb="--frame-batch 20"
  (cd /tmp && timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} \
      --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-1048576} --output-format csv \
      -d "$OUT/pcs_$cfg" -o run -- python3 "$ROOT/tools/kbench.py" --config $cfg --frames 60 $fb > "$OUT/pcs_$cfg.log" 2>&1)
  rc=$?
  echo "$cfg rc=$rc"
  tail -3 "$OUT/pcs_$cfg.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
