#!/usr/bin/env bash
# Sourced by GPU-box commands: `source tools/gpu_lib.sh && step NAME SECONDS CMD... && step ...`.
# Each step runs under its own time limit with its log in gpurun_out/NAME.log; a crash, abort or
# timeout (exit >= 124, 134, 139) stops the chain (returns non-zero), ordinary test failures
# (pytest exit 1) do not.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
LOG="$ROOT/gpurun_out"
mkdir -p "$LOG"
step() { # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$LOG/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 30 "$LOG/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"
        return $rc
    fi
    return 0
}
pytest_gpu() { # name seconds pytest-args...
    local name=$1 secs=$2
    shift 2
    step "$name" "$secs" python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu "$@"
}
