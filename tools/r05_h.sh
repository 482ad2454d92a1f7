#!/usr/bin/env bash
# Round 5: where C2's FETCH comes from — FETCH_SIZE per frame of the 20-frame launches (kbench:
# one UBO, identical frames) with and without the envmap, and per dealing variant.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${R05_TAG:-r05h}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "env 0x1b 1 1" "noenv 0x13 1 1" "fmfixed 0x1b 0 0" "inter2 0x1b 2 1"; do
  set -- $v
  TRT_XCD_INTER=$3 TRT_XCD_ROT=$4 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/p_$1" -o run -- python "$ROOT/tools/kbench.py" --config C2 --frames 20 --flags $2 --settle-ms 0 > "$OUT/p_$1.log" 2>&1 || { tail -5 "$OUT/p_$1.log"; exit 1; }
  python "$ROOT/tools/pmc_fetch.py" "$OUT/p_$1" 20 "$1"
done
