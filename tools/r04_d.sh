#!/usr/bin/env bash
# Round 4: refill-style pass A (defer_walk_q) — deferred parity tests, A/B of the walk variants
# on the deep frames (2 and 8 in flight), PMC of the product's passes.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R04_TAG:-r04d}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-defer or dropin or multi_deep or reference or fullres}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
echo "== ab $(date +%T)"
for round in 1 2; do
  for v in ${VARIANTS:-prod norefill t16 t48}; do
    lib=""; [ "$v" != prod ] && lib="variants/libtrt_$v.so"
    for cfg in ref readme; do
      for inf in 2 8; do
        TRT_LIB=$lib timeout -k 10 200 python tools/kbench.py --config $cfg --frames 40 --inflight $inf --tag "$v" >> "$OUT/ab_deep.jsonl" 2>> "$OUT/ab_deep.err" || { tail -5 "$OUT/ab_deep.err"; exit 1; }
      done
    done
  done
done
python - "$OUT/ab_deep.jsonl" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[(r['tag'], r['config'], r['inflight'])].append(r['wall_us_no_events'])
for k in sorted(d): print(k, [round(x, 1) for x in d[k]], 'median', round(statistics.median(d[k]), 1))
PY
echo "== pmc $(date +%T)"
PMC_OUT="$OUT/pmc" CFGS=ref bash "$ROOT/tools/pmc_r03.sh" || exit 1
echo "== done $(date +%T)"
