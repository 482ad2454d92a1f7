set -u
P1="sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES"
P2="ta GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
P3="ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum"
P4="td TD_TD_BUSY_sum TD_TC_STALL_sum"
P5="tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
P6="tcp2 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
for cfg in C4 ref; do
  for P in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
    name=${P%% *}; cnts=${P#* }
    CFG=$cfg KB_EXTRA="--split 1" PASSES="x" bash -c "true"
    mkdir -p gpurun_out/pmc_mesh
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $cnts --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_mesh/${cfg}_$name" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kbench.py" --config $cfg --frames 6 --inflight 1 --split 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_mesh/${cfg}_$name.log" 2>&1)
    rc=$?
    echo "$cfg $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmc_mesh/${cfg}_$name.log"; exit $rc; fi
  done
done
