#!/usr/bin/env bash
# Experimental builds of libtrt.so for A/B timing (loaded with TRT_LIB=variants/libtrt_<name>.so).
# Diagnostic variants change results (they price one stage) and are never the product.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/vkcomputeshader_tinyraytracer_amd/csrc
OUT=$ROOT/variants
mkdir -p "$OUT" "$ROOT/build/diag"
FP="-ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
HOST="-O2 -std=c++17 -fPIC -ffp-contract=off -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
HDR_NEWEST=$(ls -t "$SRC"/*.h "$ROOT"/include/trt/*.h | head -n 1)
for f in trt_runtime trt_multi band_plan scene_build obj_load bvh_build image_io jpeg_entropy jpeg_api; do
    [ "$ROOT/build/diag/$f.o" -nt "$SRC/$f.cpp" ] && [ "$ROOT/build/diag/$f.o" -nt "$HDR_NEWEST" ] || /opt/rocm/bin/hipcc $HOST -x c++ -c -o "$ROOT/build/diag/$f.o" "$SRC/$f.cpp"
done
variant() { # name extra-flags...
    local name=$1
    shift
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $FP "$@" -c -o "$ROOT/build/diag/k_$name.o" "${KSRC:-$SRC/trt_kernel.hip}"
    [ "$ROOT/build/diag/jpeg_kernel.o" -nt "$SRC/jpeg_kernel.hip" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $FP -c -o "$ROOT/build/diag/jpeg_kernel.o" "$SRC/jpeg_kernel.hip"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libtrt_$name.so" "$ROOT/build/diag/k_$name.o" \
        "$ROOT/build/diag/trt_runtime.o" "$ROOT/build/diag/trt_multi.o" "$ROOT/build/diag/band_plan.o" "$ROOT/build/diag/scene_build.o" "$ROOT/build/diag/obj_load.o" \
        "$ROOT/build/diag/bvh_build.o" "$ROOT/build/diag/image_io.o" "$ROOT/build/diag/jpeg_entropy.o" \
        "$ROOT/build/diag/jpeg_api.o" "$ROOT/build/diag/jpeg_kernel.o" -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
    echo "built $OUT/libtrt_$name.so"
}
for v in "$@"; do
    case $v in
        base|cur) variant "$v" ;;
        late0) variant late0 -DTRT_LATE_MAT=0 ;;
        unroll) variant unroll -DTRT_LIGHT_UNROLL=1 ;;
        oldsize) variant oldsize -DTRT_LIGHT_UNROLL=1 -DTRT_MESH_PAIRS=1 ;;
        sh4) variant sh4 -DTRT_G3_WAVES_SHALLOW=4 ;;
        g3lds*) variant "$v" -DTRT_G3_LDS="${v#g3lds}" ;;          # g3lds8, g3lds24, ...
        g0w*) variant "$v" -DTRT_G0_WAVES="${v#g0w}" ;;             # g0w4, g0w6
        dw*) variant "$v" -DTRT_DEFER_WAVES="${v#dw}" ;;            # dw5, dw6
        pool*) variant "$v" -DTRT_DEFER_POOL_N="${v#pool}" ;;       # pool64, pool192
        swe*) variant "$v" -DTRT_SHADOW_WAVE_EXT="0.${v#swe0}" ;;   # swe005 = 0.05, swe02 = 0.2
        noswave) variant noswave -DTRT_SHADOW_WAVE=0 ;;
        nolp) variant nolp -DTRT_LEAF_PREFETCH=0 ;;
        noquant) variant noquant -DTRT_BVH_QUANT=0 ;;
        noskip) variant noskip -DTRT_SKIP_DARK=0 ;;
        noroot) variant noroot -DTRT_ROOT_SCALAR=0 ;;
        noempty) variant noempty -DTRT_BVH4_EMPTY_BOX=0 ;;
        nolds) variant nolds -DTRT_BVH_LDS=0 ;;
        bvh2) variant bvh2 -DTRT_BVH_WIDTH=2 ;;
        fastdiv) variant fastdiv -fno-hip-fp32-correctly-rounded-divide-sqrt ;;
        # diagnostic builds: they change the image (price one stage) or record timing
        dumpshadow) variant dumpshadow -DTRT_DIAG_DUMP_SHADOW ;;
        noshadow) variant noshadow -DTRT_DIAG_NO_SHADOW ;;
        nopow) variant nopow -DTRT_DIAG_NO_POW ;;
        trivial) variant trivial -DTRT_DIAG_TRIVIAL ;;
        noenvfetch) variant noenvfetch -DTRT_DIAG_NO_ENV_FETCH ;;
        notrig) variant notrig -DTRT_DIAG_NO_UV_TRIG ;;
        clock) variant clock -DTRT_DIAG_WAVE_CLOCK ;;
        work) variant work -DTRT_DIAG_PIXEL_WORK ;;
        passa) variant passa -DTRT_DIAG_PASSA_STEPS ;;
        prev) # the kernel of git revision $PREV (default HEAD), for A/B against the work tree
            git -C "$ROOT" show "${PREV:-HEAD}:vkcomputeshader_tinyraytracer_amd/csrc/trt_kernel.hip" > "$SRC/.prev_kernel.hip"
            KSRC="$SRC/.prev_kernel.hip" variant prev
            rm -f "$SRC/.prev_kernel.hip" ;;
        *) echo "unknown variant $v"; exit 2 ;;
    esac
done
