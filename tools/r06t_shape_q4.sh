# Deferred launch shapes through the C++ host at HIP's default queues: "G:n ..." (G frames per
# group, n groups in flight).  Run on the box: bash tools/r06t_shape_q4.sh <tag> "8:2 12:2"
set -e
TAG=${1:-r06t}; SHAPES=${2:-"8:2 12:2"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2; do for gn in $SHAPES; do
  env -u GPU_MAX_HW_QUEUES TRT_DEFER_GROUP=${gn%%:*} timeout -k 10 200 tests/native/drop_in_host --bench \
    tests/golden/dropin_meshes.bin 192 ${gn#*:} >> $OUT/shape_q4.log 2>&1
  echo "shape=$gn" >> $OUT/shape_q4.log
done; done
grep "bench\|shape=" $OUT/shape_q4.log
