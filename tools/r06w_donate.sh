# Round-6 pass-A donation (TRT_DEFER_DONATE): deferred parity under donation, then kbench A/B at
# the reference's 2 in flight and 16 single-frame slots.  bash tools/r06w_donate.sh <tag> "0 64 96"
set -e
TAG=${1:-r06w}; LEVELS=${2:-"0 64 96"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export GPU_MAX_HW_QUEUES=32
TRT_DEFER_DONATE=64 R06_TAG=$TAG TESTS="tests/test_gpu_defer.py" TESTS_TAG=defer_donate bash tools/r06.sh pytest
for round in 1 2; do for d in $LEVELS; do for leg in "ref 2" "readme 2" "ref 16" "readme 16"; do
  set -- $leg
  TRT_DEFER_DONATE=$d timeout -k 10 300 python tools/kbench.py --config $1 --frames 96 --inflight $2 \
    --tag "d$d:$1:if$2" >> $OUT/donate.jsonl 2>> $OUT/donate.err
done; done; done
python tools/ab_summary.py $OUT/donate.jsonl
