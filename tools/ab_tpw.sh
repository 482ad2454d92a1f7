cd $GRAFT_REPO_ROOT
for v in base tpw2 tpw4; do
  TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag $v || exit $?
  TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag ${v}_empty --depth 1 --flags 0 || exit $?
  TRT_LIB=variants/libtrt_$v.so timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag ${v}_env_only --depth 1 --flags 8 || exit $?
done
