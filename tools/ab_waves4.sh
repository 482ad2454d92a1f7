#!/usr/bin/env bash
# A/B of the BVH walk's 3-wave (GEOM 2) and 4-wave (GEOM 3) builds, forced by TRT_BVH_WAVES4,
# over the mesh configurations; interleaved rounds in one box session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
for cfg in ${CFGS:-C3 C4 ref}; do
  for w in 0 1; do
    fr=30
    case $cfg in C4|ref) fr=10 ;; C5) fr=3 ;; esac
    TRT_BVH_WAVES4=$w timeout -k 10 200 python tools/kbench.py --config $cfg --frames $fr --inflight 2 --tag ${cfg}_w4=$w || exit $?
  done
done
done
