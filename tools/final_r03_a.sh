#!/usr/bin/env bash
# Round-3 closing run, part 1: the whole GPU suite, smoke, and the bench at the driver's 20 steps
# and at its default 1000 steps (logs in gpurun_out/).
source "$(dirname "$0")/gpu_lib.sh"
pytest_gpu gpu_tests 900 tests \
 && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" \
 && step bench20 420 python bench.py --steps 20 \
 && step bench1000 420 python bench.py --no-cpu
