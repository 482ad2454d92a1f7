#!/usr/bin/env bash
# C4: per-lane BVH vs the wave-uniform batch walk, by depth (primary rays are the coherent part).
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for d in 1 2 4; do
  timeout -k 10 120 python tools/kbench.py --config C4 --frames 20 --inflight 1 --depth $d --tag "bvh_d$d"
  timeout -k 10 120 python tools/kbench.py --config C4 --frames 20 --inflight 1 --depth $d --flags 283 --tag "walk_d$d"
done
