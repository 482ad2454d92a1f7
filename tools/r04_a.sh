#!/usr/bin/env bash
# Round 4, first GPU session: GPU suite, the driver's bench line (now with live PMC traffic and
# the 2-in-flight legs), PMC of the shipped frame's deferred passes (pass A / B / C), kernel
# stats of the bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r04a"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
step() { echo "== $1 $(date +%T)"; }
step pytest
TRT_PARITY_LOG="$OUT/parity_log.jsonl" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
step bench20
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench20.log" 2>&1 || { tail -30 "$OUT/bench20.log"; exit 1; }
tail -c 600 "$OUT/bench20.log"
step stats
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_bench20" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --traffic off > "$OUT/stats_bench20.log" 2>&1) || { tail -30 "$OUT/stats_bench20.log"; exit 1; }
step pmc_ref
PMC_OUT="$OUT/pmc" CFGS=ref bash "$ROOT/tools/pmc_r03.sh" || exit 1
step done
