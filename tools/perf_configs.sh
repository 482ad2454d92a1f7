#!/usr/bin/env bash
# Kernel-time probe across the benchmark configurations (one process per config), frames in
# flight 1 and 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in ${CFGS:-C1 C2 C3 C4 C5 ref}; do
  for n in ${INFLIGHT:-1 2}; do
    fr=${FRAMES:-50}
    [ "$cfg" = C5 ] && fr=6
    timeout -k 10 300 python tools/kbench.py --config $cfg --frames $fr --inflight $n --tag ${cfg}_if$n || exit $?
  done
done
