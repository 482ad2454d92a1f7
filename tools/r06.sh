#!/usr/bin/env bash
# Round-6 GPU runner: one script, one stage per argument (run on the box through gpurun), e.g.
#   gpurun -- 'bash tools/r06.sh hotrepro prof'
# Every GPU step has its own time limit; the script stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${R06_TAG:-r06}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
PYT="python -u -m pytest -x -v --timeout 150 --timeout-method thread"

step() { # step <name> <seconds> <command...>: runs, logs to $OUT/<name>.log, stops on failure
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; exit $rc; fi
}

for stage in "$@"; do
  case $stage in
  tests) # the whole GPU suite
    TRT_PARITY_LOG="$OUT/parity_log.jsonl" step pytest_gpu 1000 $PYT -m gpu tests ;;
  smoke)
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench) # the driver's command
    step bench20 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
  prof) # rocprofv3 kernel trace of the bench command, split per (kernel, grid)
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu --traffic off > "$OUT/prof_bench.log" 2>&1) \
      || { tail -20 "$OUT/prof_bench.log"; exit 1; }
    db=$(find "$OUT/prof" -name '*.db' | head -1)
    python tools/rocpd_stats.py --split-grid "$db" "$OUT/kernel_stats_by_grid.csv"
    python tools/rocpd_stats.py "$db" "$OUT/kernel_stats.csv"
    grep '^{' "$OUT/prof_bench.log" | tail -1 > "$OUT/prof_bench_line.json"
    rm -rf "$OUT/prof"
    head -6 "$OUT/kernel_stats_by_grid.csv" | cut -c1-200 ;;
  kbench) # kbench legs named in KB (e.g. KB="C2:--frame-batch 20;shipped:--inflight 16")
    IFS=';' read -ra legs <<< "${KB:-}"
    for leg in "${legs[@]}"; do
      cfg=${leg%%:*}; args=${leg#*:}
      step "kb_${cfg}" 300 python tools/kbench.py --config "$cfg" $args --tag "$leg"
      grep '^{' "$OUT/kb_${cfg}.log" >> "$OUT/kb.jsonl"
    done ;;
  pytest) # the test files named in TESTS
    step "pytest_${TESTS_TAG:-sel}" 900 $PYT $TESTS ;;
  ab) # interleaved A/B of library builds: AB_LIBS="name:path ..." (empty path = the product),
      # AB_LEGS="config|args;config|args" (kbench), AB_ROUNDS rounds
    IFS=';' read -ra legs <<< "${AB_LEGS:-C2|--frames 200 --frame-batch 20}"
    for round in $(seq 1 "${AB_ROUNDS:-2}"); do
      for lib in ${AB_LIBS:-cur:}; do
        name=${lib%%:*}; path=${lib#*:}
        for leg in "${legs[@]}"; do
          cfg=${leg%%|*}; args=${leg#*|}
          TRT_LIB=$path timeout -k 10 300 python tools/kbench.py --config "$cfg" $args --tag "$name:$cfg:$args" \
            >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
        done
      done
    done
    python tools/ab_summary.py "$OUT/ab.jsonl" ;;
  envab) # interleaved A/B of runtime knobs: AB_ENVS="name:VAR=val,VAR=val name2:VAR=val", AB_LEGS as ab
    IFS=';' read -ra legs <<< "${AB_LEGS:-C2|--frames 200 --frame-batch 1 --inflight 2}"
    for round in $(seq 1 "${AB_ROUNDS:-2}"); do
      for spec in ${AB_ENVS:-cur:}; do
        name=${spec%%:*}; kv=${spec#*:}
        for leg in "${legs[@]}"; do
          cfg=${leg%%|*}; args=${leg#*|}
          env ${kv//,/ } timeout -k 10 300 python tools/kbench.py --config "$cfg" $args --tag "$name:$cfg:$args" \
            >> "$OUT/envab.jsonl" 2>> "$OUT/envab.err" || { tail -5 "$OUT/envab.err"; exit 1; }
        done
      done
    done
    python tools/ab_summary.py "$OUT/envab.jsonl" ;;
  groups) # deferred frame groups (TRT_DEFER_GROUP = G frames per launch, N groups in flight)
    for round in 1 2; do
      for gn in "1 16" "2 8" "4 4" "8 2" "16 1"; do
        set -- $gn
        for cfg in ref readme; do
          TRT_DEFER_GROUP=$1 timeout -k 10 300 python tools/kbench.py --config $cfg --frames 192 --inflight $2 \
            --tag "g$1n$2:$cfg" >> "$OUT/groups.jsonl" 2>> "$OUT/groups.err" || { tail -5 "$OUT/groups.err"; exit 1; }
        done
      done
    done
    python tools/ab_summary.py "$OUT/groups.jsonl"
    for gn in "1 0" "4 4" "8 2" "16 1"; do # the C++ host at HIP's default queue count
      set -- $gn
      env -u GPU_MAX_HW_QUEUES TRT_DEFER_GROUP=$1 timeout -k 10 200 tests/native/drop_in_host --bench \
        tests/golden/dropin_meshes.bin 192 "$2" >> "$OUT/groups_cabi.log" 2>&1 || exit 1
    done
    grep bench "$OUT/groups_cabi.log" ;;
  pmc) # PMC passes (one counter group per rocprofv3 run) over PMC_CMD, summarised per kernel
    CMD=${PMC_CMD:-python3 tools/kbench.py --config ref --frames 48 --inflight 16}
    i=0
    IFS=';' read -ra sets <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE;TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE}"
    for set_ in "${sets[@]}"; do
      i=$((i + 1))
      (export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $set_ --kernel-trace --output-format csv \
        -d "$OUT/pmc/p$i" -o run -- $CMD > "$OUT/pmc_p$i.log" 2>&1) || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc_p$i.log"; exit 1; }
    done
    python tools/pmc_kernels.py "$OUT/pmc" > "$OUT/pmc_kernels.jsonl"
    find "$OUT/pmc" -name '*kernel_trace.csv' -delete
    cut -c1-400 "$OUT/pmc_kernels.jsonl" | head -8 ;;
  cabi) # the shipped frame through the C++ host: HIP's default queues (auto / 4 in flight), 32 queues
    for cf in "unset 0" "unset 4" "unset 2" "32 0"; do
      set -- $cf
      if [ "$1" = unset ]; then
        env -u GPU_MAX_HW_QUEUES timeout -k 10 200 tests/native/drop_in_host --bench tests/golden/dropin_meshes.bin 160 "$2" >> "$OUT/cabi.log" 2>&1 || exit 1
      else
        GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 tests/native/drop_in_host --bench tests/golden/dropin_meshes.bin 160 "$2" >> "$OUT/cabi.log" 2>&1 || exit 1
      fi
    done
    grep bench "$OUT/cabi.log" ;;
  *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
