#!/usr/bin/env bash
# Round 4, pass-A rewrite (wave-shared segment pool + tree events): GPU suite, kbench of the
# deep frames at 2 and 8 in flight, PMC of the shipped frame's passes, the driver's bench line.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04b}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
step() { echo "== $1 $(date +%T)"; }
step pytest
TRT_PARITY_LOG="$OUT/parity_log.jsonl" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
step kbench
for cfg in ref readme; do
  for inf in 2 8; do
    timeout -k 10 300 python tools/kbench.py --config $cfg --frames 40 --inflight $inf > "$OUT/kbench_${cfg}_if$inf.log" 2>&1 || { tail -20 "$OUT/kbench_${cfg}_if$inf.log"; exit 1; }
    tail -1 "$OUT/kbench_${cfg}_if$inf.log"
  done
done
step pmc_ref
PMC_OUT="$OUT/pmc" CFGS=ref bash "$ROOT/tools/pmc_r03.sh" || exit 1
step bench20
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench20.log" 2>&1 || { tail -30 "$OUT/bench20.log"; exit 1; }
tail -c 400 "$OUT/bench20.log"
step done
