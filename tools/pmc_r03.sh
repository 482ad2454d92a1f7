#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over tools/kbench.py
# with one launch per frame, for C2, C4 (4-wave quantized BVH walk) and the shipped frame
# (deferred shadows: pass A trace_kernel<..., DEFER>, pass B defer_shadows, pass C
# defer_resolve).  Output: gpurun_out/pmc_r03/<cfg>_<pass>/.  Summarise with
# tools/pmc_summary_r03.py.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="${PMC_OUT:-$ROOT/gpurun_out/pmc_r03}"
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES"
P2="tatd GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum"
P3="fetch FETCH_SIZE"
P4="write WRITE_SIZE"
P5="tcc TCC_HIT_sum TCC_MISS_sum"
P6="tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
for cfg in ${CFGS:-C2 C4 ref}; do
  frames=6
  [ "$cfg" = C2 ] && frames=20
  for P in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
    name=${P%% *}; cnts=${P#* }
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $cnts --kernel-trace --output-format csv -d "$OUT/${cfg}_$name" -o run \
       -- python3 "$ROOT/tools/kbench.py" --config $cfg --frames $frames --inflight 1 --frame-batch 1 > "$OUT/${cfg}_$name.log" 2>&1)
    rc=$?
    echo "$cfg $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${cfg}_$name.log"; exit $rc; fi
  done
done
