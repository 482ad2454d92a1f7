#!/usr/bin/env bash
# A/B the in-tree product library against diag/ variants: interleaved kbench rounds.
#   VARIANTS="base" CONFIGS="C2 C3" bash tools/ab_product.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for cfg in ${CONFIGS:-C2}; do
    timeout -k 10 200 python tools/kbench.py --config $cfg --frames ${FRAMES:-200} --tag product || exit $?
    for v in ${VARIANTS:-base}; do
      TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $cfg --frames ${FRAMES:-200} --tag $v || exit $?
    done
  done
done
