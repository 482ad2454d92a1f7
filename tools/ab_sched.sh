cd $GRAFT_REPO_ROOT
TRT_SCHED=static timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag static || exit $?
for w in 4 8 12 16 24 48; do
  TRT_WPC=$w TRT_SCHED=grid timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag grid_wpc$w || exit $?
  TRT_WPC=$w TRT_SCHED=persistent timeout -k 10 200 python tools/kbench.py --config C2 --frames 200 --tag atomic_wpc$w || exit $?
done
