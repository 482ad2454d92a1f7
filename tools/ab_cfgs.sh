#!/usr/bin/env bash
# A/B of variants/ builds over several configurations and frames-in-flight settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
for cfg in ${CFGS:-C2 C3 ref}; do
for v in ${VARIANTS:-base prev}; do
  for n in ${INFLIGHT:-1 2}; do
    fr=${FRAMES:-100}
    case $cfg in C3) fr=30 ;; C4|ref) fr=10 ;; C5) fr=3 ;; esac
    TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config $cfg --frames $fr --inflight $n --tag ${cfg}_${v}_if$n || exit $?
  done
done
done
done
