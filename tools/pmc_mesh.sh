#!/usr/bin/env bash
# PMC passes over tools/kbench.py (one config, a few frames, 1 frame in flight) for the
# memory pipeline of the mesh kernels: texture-address / data (TA/TD) and vector L1 (TCP)
# busy and stall counters.  One counter group per rocprofv3 run, --kernel-trace only.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
LOG="$ROOT/gpurun_out/pmc_mesh"
mkdir -p "$LOG"
export TMPDIR=/tmp
cd /tmp
CFG=${CFG:-C4}
KB=("$ROOT/tools/kbench.py" --config "$CFG" --frames ${FRAMES:-6} --inflight 1 ${KB_EXTRA:-})
run() { # name counters...
    local name=$1
    shift
    echo "== pmc $name: $*"
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$LOG/$name" -o run \
        -- python3 "${KB[@]}" > "$LOG/$name.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    tail -n 2 "$LOG/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
if [ ! -s "$LOG/counters_list.txt" ]; then
    timeout -s KILL 120 rocprofv3 -L > "$LOG/counters_list.txt" 2>&1 || true
fi
for pass in ${PASSES:-"ta GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum"}; do
    # shellcheck disable=SC2086
    run $pass
done
