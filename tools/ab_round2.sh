#!/usr/bin/env bash
# A/B of variants/ builds (tools/build_variants.sh) and frames in flight, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-C2}
for round in 1 2; do
for v in ${VARIANTS:-base w5}; do
  for n in ${INFLIGHT:-1 2}; do
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $CFG --frames 400 --inflight $n --tag ${v}_if$n || exit $?
  done
done
done
