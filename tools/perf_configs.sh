#!/usr/bin/env bash
# Kernel-time probe across the benchmark configurations (one process per config).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in ${CFGS:-C2 C3 C4 ref}; do
  timeout -k 10 300 python tools/kbench.py --config $cfg --frames ${FRAMES:-50} --tag $cfg || exit $?
done
