#!/usr/bin/env bash
# (1) deep deferred frames with the 4-wave BVH build (TRT_BVH_WAVES4=1) vs the default 3-wave;
# (2) depth-4 mesh frames deferred vs the per-pixel loop at the default frames in flight.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for rep in 1 2; do
  for cfg in ref readme; do
    timeout -k 10 120 python tools/kbench.py --config $cfg --frames 80 --tag waves3
    TRT_BVH_WAVES4=1 timeout -k 10 120 python tools/kbench.py --config $cfg --frames 80 --tag waves4
  done
done
for cfg in C3 C4; do
  for d in 1 2; do
    timeout -k 10 120 python tools/kbench.py --config $cfg --frames 40 --defer $d --tag "defer$d"
  done
done
