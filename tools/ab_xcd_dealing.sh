#!/usr/bin/env bash
# A/B of the multi-frame tile dealing knobs (TRT_XCD_ROT / TRT_XCD_SKEW) on C2 at the driver's
# 20-frame launch and at 64-frame launches; entries interleaved per round.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for fr in ${FRAMESET:-20 64}; do
  LIBS="${LIBS:-prod prod+TRT_XCD_ROT=1 prod+TRT_XCD_ROT=2 prod+TRT_XCD_ROT=3 prod+TRT_XCD_SKEW=3 prod+TRT_XCD_SKEW=1 prod+TRT_XCD_ROT=1+TRT_XCD_SKEW=3}" \
    CFGS="${CFGS:-C2}" ROUNDS="${ROUNDS:-3}" FRAMES=$fr tools/ab_libs.sh || exit $?
done
