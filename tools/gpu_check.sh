#!/usr/bin/env bash
# One GPU-box session: smoke, GPU parity tests, a short bench, optionally a rocprofv3 kernel
# trace of the bench.  Every GPU step has its own time limit; a crash, abort or timeout
# (exit >= 124, or 134/139) ends the script, ordinary test failures (pytest exit 1) do not.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
LOG="$ROOT/gpurun_out"
mkdir -p "$LOG"
step() { # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$LOG/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "$LOG/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"
        exit $rc
    fi
    return 0
}
rocm-smi --showproductname > "$LOG/gpu_info.log" 2>&1 || true
lscpu > "$LOG/lscpu.log" 2>&1 || true
if [ -z "${SKIP_TESTS:-}" ]; then
    step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 900 python -m pytest tests -m gpu -q --timeout 300 ${PYTEST_ARGS:-}
fi
step bench 400 python bench.py ${BENCH_ARGS:-}
if [ -n "${PROFILE:-}" ]; then
    export TMPDIR=/tmp
    cd /tmp
    step rocprof_stats 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$LOG/prof" -o run -- python3 "$ROOT/bench.py" --steps 200 --warmup 10 --no-cpu
    cd "$ROOT"
fi
