#!/usr/bin/env bash
# One GPU-box session: smoke, GPU parity tests, a short bench.  Every GPU step has its own
# time limit; a crash, abort or timeout (exit >= 124, or 134/139) ends the script, ordinary
# test failures (pytest exit 1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "fatal rc=$rc in $name: stopping"
        exit $rc
    fi
    return 0
}
rocm-smi --showproductname > gpurun_out/gpu_info.log 2>&1 || true
lscpu > gpurun_out/lscpu.log 2>&1 || true
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -p pytest_timeout --timeout 300 ${PYTEST_ARGS:-}
step bench 400 python bench.py ${BENCH_ARGS:-}
