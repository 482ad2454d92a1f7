cd $GRAFT_REPO_ROOT
for v in trivial nopow; do
for sz in "1024 768" "512 384" "256 192" "2048 1536"; do
  set -- $sz
  TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag ${v}_$1 --depth 1 --flags 0 --width $1 --height $2 || exit $?
done; done
