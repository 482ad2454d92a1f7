#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of tools/kbench.py for one config (CONFIG, default ref);
# the stats CSV lands in gpurun_out/prof_<config>/.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG="${CONFIG:-ref}"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$CFG" -o run -- \
    python3 "$ROOT/tools/kbench.py" --config "$CFG" --frames "${FRAMES:-30}" ${KB_ARGS:-}
cd "$ROOT"
find gpurun_out/prof_$CFG -name "*kernel_stats.csv" -exec cat {} \;
