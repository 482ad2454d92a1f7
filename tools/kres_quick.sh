#!/usr/bin/env bash
# Register / scratch / LDS of ONE kernel instantiation, compiled alone (TRT_KRES_ONLY): a register
# study in ~1 minute instead of the full library build.  Extra -D flags after the kernel.
#   tools/kres_quick.sh 'trt::trace_kernel<3, false, 3, false>' [-DTRT_...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
K="$1"; shift
FP="-ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $FP "-DTRT_KRES_ONLY=$K" "$@" --cuda-device-only -c \
    -o /tmp/kres_quick.co "$ROOT/vkcomputeshader_tinyraytracer_amd/csrc/trt_kernel.hip" -Rpass-analysis=kernel-resource-usage 2>&1 \
    | sed 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' \
    | awk '/^Function Name:/ {show = ($0 ~ /trace_|defer_|share_/)} show && /Function Name|VGPRs|Spill|ScratchSize|Occupancy|LDS Size/ {print}'
