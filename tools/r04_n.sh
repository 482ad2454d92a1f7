#!/usr/bin/env bash
# Round 4 closing validation: full GPU suite (parity log), smoke, the default bench line, the 20-step
# line, rocprofv3 kernel stats of the bench, PMC of the shipped frame's passes.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04n}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
echo "== pytest $(date +%T)"
TRT_PARITY_LOG="$OUT/parity_log.jsonl" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log" | cut -c1-200
echo "== bench default $(date +%T)"
timeout -k 10 900 python bench.py > "$OUT/bench_default.log" 2>&1 || { tail -30 "$OUT/bench_default.log"; exit 1; }
tail -c 300 "$OUT/bench_default.log"
echo "== bench20 $(date +%T)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench20.log" 2>&1 || { tail -30 "$OUT/bench20.log"; exit 1; }
tail -c 300 "$OUT/bench20.log"
echo "== stats $(date +%T)"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_bench20" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --traffic off > "$OUT/stats_bench20.log" 2>&1) || { tail -30 "$OUT/stats_bench20.log"; exit 1; }
echo "== pmc $(date +%T)"
PMC_OUT="$OUT/pmc" CFGS="${PMC_CFGS:-ref C4}" bash "$ROOT/tools/pmc_r03.sh" || exit 1
echo "== done $(date +%T)"
