#!/usr/bin/env bash
# Round 5: the frames-in-flight parity test with a native backtrace on SIGABRT (diagnosing an
# abort seen with hot-first dealing).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05v}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32 LIBC_FATAL_STDERR_=1
timeout -k 10 300 python -u -c "
import ctypes, sys
ctypes.CDLL('$ROOT/tools/dbg/abort_bt.so')
import pytest
sys.exit(pytest.main(['-p', 'no:faulthandler', '-x', '-v', '--timeout', '150', '--timeout-method', 'thread', 'tests/test_gpu_parity.py']))
" > "$OUT/pytest.log" 2>&1
rc=$?
grep -v "^  File\|PASSED" "$OUT/pytest.log" | tail -60
exit $rc
