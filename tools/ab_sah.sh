#!/usr/bin/env bash
# A/B of the BVH builder's SAH knobs (TRT_BVH_CT node-visit cost, TRT_BVH_LEAF_MIN/MAX) over
# the mesh configurations; interleaved rounds in one box session.  SETTINGS: "ct:min:max ...".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
for cfg in ${CFGS:-C3 C4 ref}; do
  for s in ${SETTINGS:-0:4:8 1:4:8 2:4:8 1:4:16 4:4:16 0:2:4}; do
    IFS=: read ct lmin lmax <<< "$s"
    fr=30
    case $cfg in C4|ref) fr=10 ;; C5) fr=3 ;; esac
    TRT_BVH_CT=$ct TRT_BVH_LEAF_MIN=$lmin TRT_BVH_LEAF_MAX=$lmax timeout -k 10 200 \
        python tools/kbench.py --config $cfg --frames $fr --inflight 2 --tag ${cfg}_sah=$s || exit $?
  done
done
done
