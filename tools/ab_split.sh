#!/usr/bin/env bash
# Subtree-split windows x frames in flight on the mesh configurations (product library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in ${CFGS:-ref C3 C4}; do
  for w in ${WINDOWS:-1 2 3 4}; do
    for n in ${INFLIGHT:-1 2}; do
      fr=10; [ $cfg = C3 ] && fr=30
      timeout -k 10 300 python tools/kbench.py --config $cfg --frames $fr --inflight $n --split $w --tag ${cfg}_w${w}_if$n || exit $?
    done
  done
done
