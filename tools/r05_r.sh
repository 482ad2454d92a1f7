#!/usr/bin/env bash
# Round 5: the top nodes of the quantized BVH4 in each wave's LDS (TRT_TOP_LDS = 21, product) vs
# none (top0) and the top two levels (top5): GPU parity subset, then kbench C4 / C3 / C5 and the
# deep frames at the auto in-flight count, interleaved rounds; PMC FETCH / WRITE on C4.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05r}"
mkdir -p "$OUT"
cd "$ROOT"
export GPU_MAX_HW_QUEUES=32
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_fullres.py tests/test_golden_renders.py tests/test_gpu_parity.py tests/test_gpu_defer.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for round in 1 2; do
  for lib in prod top0 top5; do
    L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
    for cf in "C4 20" "C3 200" "C5 3" "ref 160" "readme 160"; do
      set -- $cf
      TRT_LIB=$L timeout -k 10 200 python tools/kbench.py --config $1 --frames $2 --tag "$lib:$1" >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err" || { tail -5 "$OUT/kb.err"; exit 1; }
    done
  done
done
python - "$OUT/kb.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r = json.loads(l); d[r['tag']].append((r['wall_us_no_events'], r['med_us']))
for k in sorted(d): print(k, 'wall us/frame', [x[0] for x in d[k]], 'span us', [x[1] for x in d[k]])
PY
cd /tmp && export TMPDIR=/tmp
for lib in prod top0; do
  L=""; [ $lib != prod ] && L="$ROOT/variants/libtrt_$lib.so"
  for c in WRITE_SIZE FETCH_SIZE; do
    TRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_${lib}_$c" -o run -- python "$ROOT/tools/kbench.py" --config C4 --frames 4 --settle-ms 0 --inflight 1 > "$OUT/pmc_${lib}_$c.log" 2>&1 || { tail -5 "$OUT/pmc_${lib}_$c.log"; exit 1; }
    python "$ROOT/tools/pmc_fetch.py" "$OUT/pmc_${lib}_$c" 4 "$lib"
  done
done
echo done
