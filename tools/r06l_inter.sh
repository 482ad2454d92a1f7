# Round-6 A/B of frame-interleaved dealing in deferred frame groups (TRT_DEFER_INTER: 1 = pass A,
# 2 = passes A, B and C), parity first.  Run on the box: bash tools/r06l_inter.sh <tag> <modes...>
set -e
TAG=${1:-r06l}; shift
MODES=${*:-"0 1"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for m in $MODES; do
  [ "$m" = 0 ] && continue
  TRT_DEFER_INTER=$m R06_TAG=$TAG TESTS="tests/test_gpu_defer.py" TESTS_TAG=defer_inter$m bash tools/r06.sh pytest
done
ENVS=""
for m in $MODES; do ENVS="$ENVS g8i$m:TRT_DEFER_GROUP=8,TRT_DEFER_INTER=$m g4i$m:TRT_DEFER_GROUP=4,TRT_DEFER_INTER=$m"; done
R06_TAG=$TAG AB_ROUNDS=2 AB_ENVS="$ENVS" AB_LEGS="ref|--frames 192 --inflight 2;readme|--frames 192 --inflight 2" bash tools/r06.sh envab
for r in 1 2; do for m in $MODES; do
  env -u GPU_MAX_HW_QUEUES TRT_DEFER_INTER=$m timeout -k 10 200 tests/native/drop_in_host --bench tests/golden/dropin_meshes.bin 160 0 >> $OUT/cabi_inter.log 2>&1
  echo "inter=$m" >> $OUT/cabi_inter.log
done; done
grep "bench\|inter=" $OUT/cabi_inter.log
