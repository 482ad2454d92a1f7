#!/usr/bin/env bash
# Same-box A/B of library builds and environment knobs on the kbench wall time per frame;
# entries interleaved per round to cancel drift.  An entry is a variant name
# (variants/libtrt_<name>.so) or "prod" (the in-tree build), optionally followed by
# "+VAR=value" environment settings:
#   LIBS="prod prod+TRT_DEFER_INTER=0 sh4" CFGS="C4 C3 ref" ROUNDS=2 FRAMES=20 tools/ab_libs.sh
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for cfg in ${CFGS:-C4 C3 ref readme}; do
    for ent in ${LIBS:-prod}; do
      lib=${ent%%+*}
      envs=()
      if [ "$ent" != "$lib" ]; then IFS='+' read -ra envs <<< "${ent#*+}"; fi
      if [ "$lib" = prod ]; then L=""; else L="variants/libtrt_$lib.so"; fi
      out=$(env "${envs[@]}" TRT_LIB=$L timeout -k 10 150 python tools/kbench.py --config "$cfg" --frames "${FRAMES:-20}" \
            --tag "$ent" ${KB_EXTRA:-} 2>/dev/null | tail -1)
      rc=$?
      [ $rc -ge 124 ] && { echo "timeout/crash rc=$rc ($ent $cfg)"; exit $rc; }
      python3 -c "
import json,sys
d=json.loads(sys.argv[1]); print(f\"round=$r cfg=$cfg lib=$ent wall_us={d['wall_us_no_events']:9.1f} kernel_med_us={d['med_us']:9.1f}\")" "$out"
    done
  done
done
