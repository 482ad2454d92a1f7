#!/usr/bin/env bash
# Deferred-shadow feasibility: product vs no-shadow frame time, and the dumped shadow queries
# traced coherently by shadow_batch_kernel (tools/shadow_exp.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in ${CONFIGS:-C4 ref C3}; do
  timeout -k 10 200 python tools/kbench.py --config $cfg --frames 60 --inflight 1 --tag product || exit $?
  TRT_LIB=variants/libtrt_noshadow.so timeout -k 10 200 python tools/kbench.py --config $cfg --frames 60 --inflight 1 --tag noshadow || exit $?
  TRT_LIB=variants/libtrt_dumpshadow.so timeout -k 10 200 python tools/shadow_exp.py --config $cfg || exit $?
done
