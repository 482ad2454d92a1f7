#!/usr/bin/env bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, --kernel-trace
# only, never combined with sys/runtime traces).  Outputs under gpurun_out/pmc/<pass>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
LOG="$ROOT/gpurun_out/pmc"
mkdir -p "$LOG"
export TMPDIR=/tmp
cd /tmp
CFG=${CFG:-C2}
BENCH=("$ROOT/bench.py" --config "$CFG" --steps ${STEPS:-20} --warmup 2 --no-cpu --tiled-frames 0 ${BENCH_EXTRA:-})
run() { # name counters...
    local name=$1
    shift
    echo "== pmc $name: $*"
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$LOG/$name" -o run \
        -- python3 "${BENCH[@]}" > "$LOG/$name.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    tail -n 3 "$LOG/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
timeout -k 10 120 rocprofv3 -L > "$LOG/counters_list.txt" 2>&1 || true
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH
run sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
run valu SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM
