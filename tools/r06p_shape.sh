# Round-6 sweep of the deferred launch shape at 32 queues: G frames per group x n groups in flight
# (interleaved dealing).  Run on the box: bash tools/r06p_shape.sh <tag> "G:n G:n ..."
set -e
TAG=${1:-r06p}; SHAPES=${2:-"1:16 3:6 3:8 4:6 4:8 6:4 5:5"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export GPU_MAX_HW_QUEUES=32
for round in 1 2; do for gn in $SHAPES; do for cfg in ref readme; do
  TRT_DEFER_GROUP=${gn%%:*} timeout -k 10 300 python tools/kbench.py --config $cfg --frames 192 --inflight ${gn#*:} \
    --tag "g${gn%%:*}n${gn#*:}:$cfg" >> $OUT/shape.jsonl 2>> $OUT/shape.err
done; done; done
python tools/ab_summary.py $OUT/shape.jsonl
