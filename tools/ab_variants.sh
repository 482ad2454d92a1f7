#!/usr/bin/env bash
# A/B the diag/ library variants on one box: kbench per variant, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=${CFG:-C2}
for round in 1 2; do
for v in ${VARIANTS:-base nslp noshadow nopow fastdiv}; do
  TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $CFG --frames 200 --tag $v ${KB_ARGS:-} || exit $?
  if [ -n "${EMPTY:-}" ]; then
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $CFG --frames 200 --tag ${v}_empty --depth 1 --flags 0 || exit $?
  fi
done; done
