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
        base) variant base ;;
        oldsize) variant oldsize -DTRT_LIGHT_UNROLL=1 -DTRT_MESH_PAIRS=1 ;;
        sh4) variant sh4 -DTRT_G3_WAVES_SHALLOW=4 ;;
        pk0) variant pk0 -DTRT_SPHERE_PK=0 ;;
        park1) variant park1 -DTRT_G3_PARK=1 ;;
        unroll) variant unroll -DTRT_LIGHT_UNROLL=1 ;;
        lds24) variant lds24 -DTRT_G3_LDS=24 ;;
        lds32) variant lds32 -DTRT_G3_LDS=32 ;;
        cur) variant cur ;;
        late0) variant late0 -DTRT_LATE_MAT=0 ;;
        top21) variant top21 -DTRT_TOP_LDS=21 ;;
        hotd1) variant hotd1 -DTRT_HOT_DIAG=1 ;;
        sub16) variant sub16 -DTRT_SHADOW_SUBSET=16 ;;
        sub32) variant sub32 -DTRT_SHADOW_SUBSET=32 ;;
        sub8) variant sub8 -DTRT_SHADOW_SUBSET=8 ;;
        hotd2) variant hotd2 -DTRT_HOT_DIAG=2 ;;
        top5) variant top5 -DTRT_TOP_LDS=5 ;;
        sh4late) variant sh4late -DTRT_G3_WAVES_SHALLOW=4 ;;
        g3p24) variant g3p24 -DTRT_G3_SEG_PRIV=1 -DTRT_G3_LDS=24 ;;
        g3p32) variant g3p32 -DTRT_G3_SEG_PRIV=1 -DTRT_G3_LDS=32 ;;
        g3p16) variant g3p16 -DTRT_G3_SEG_PRIV=1 -DTRT_G3_LDS=16 ;;
        g3p12) variant g3p12 -DTRT_G3_LDS=12 ;;
        swe005) variant swe005 -DTRT_SHADOW_WAVE_EXT=0.05 ;;
        swe02) variant swe02 -DTRT_SHADOW_WAVE_EXT=0.2 ;;
        nolp) variant nolp -DTRT_LEAF_PREFETCH=0 ;;
        g3p20) variant g3p20 -DTRT_G3_SEG_PRIV=1 -DTRT_G3_LDS=20 ;;
        g3p28) variant g3p28 -DTRT_G3_SEG_PRIV=1 -DTRT_G3_LDS=28 ;;
        g3w4p32) variant g3w4p32 -DTRT_G3_SEG_PRIV=1 -DTRT_G3_LDS=32 -DTRT_G3_WAVES_SHALLOW=4 ;;
        unode) variant unode -DTRT_UNIFORM_NODE=1 ;;
        g0w4) variant g0w4 -DTRT_G0_WAVES=1 ;;
        g3lds8) variant g3lds8 -DTRT_G3_LDS=8 ;;
        g3lds24) variant g3lds24 -DTRT_G3_LDS=24 ;;
        g3lds12) variant g3lds12 -DTRT_G3_LDS=12 ;;
        ww1) variant ww1 -DTRT_WHILE_WHILE=1 ;;
        noswave) variant noswave -DTRT_SHADOW_WAVE=0 ;;
        unode2) variant unode2 -DTRT_UNIFORM_NODE=2 ;;
        swe002) variant swe002 -DTRT_SHADOW_WAVE_EXT=0.02 ;;
        swe01) variant swe01 -DTRT_SHADOW_WAVE_EXT=0.1 ;;
        swe05) variant swe05 -DTRT_SHADOW_WAVE_EXT=0.5 ;;
        swe007) variant swe007 -DTRT_SHADOW_WAVE_EXT=0.07 ;;
        swe015) variant swe015 -DTRT_SHADOW_WAVE_EXT=0.15 ;;
        swe025) variant swe025 -DTRT_SHADOW_WAVE_EXT=0.25 ;;
        ww2) variant ww2 -DTRT_WHILE_WHILE=2 ;;
        g0w6) variant g0w6 -DTRT_G0_WAVES=6 ;;
        noquant) variant noquant -DTRT_BVH_QUANT=0 ;;
        noskip) variant noskip -DTRT_SKIP_DARK=0 ;;
        dumpshadow) variant dumpshadow -DTRT_DIAG_DUMP_SHADOW ;;
        noshadow) variant noshadow -DTRT_DIAG_NO_SHADOW ;;
        nopow) variant nopow -DTRT_DIAG_NO_POW ;;
        fastdiv) variant fastdiv -fno-hip-fp32-correctly-rounded-divide-sqrt ;;
        xcd) variant xcd -DTRT_XCD_SWIZZLE ;;
        libmpow) variant libmpow -DTRT_LIBM_POW ;;
        trivial) variant trivial -DTRT_DIAG_TRIVIAL ;;
        noenvfetch) variant noenvfetch -DTRT_DIAG_NO_ENV_FETCH ;;
        clock) variant clock -DTRT_DIAG_WAVE_CLOCK ;;
        prio1) variant prio1 -DTRT_PRIO=1 ;;
        prio3) variant prio3 -DTRT_PRIO=3 ;;
        w5) variant w5 -DTRT_WAVES=5 ;;
        tpw2) variant tpw2 -DTRT_TPW=2 ;;
        dlds1) variant dlds1 -DTRT_DEFER_LDS=1 ;;
        dlds2) variant dlds2 -DTRT_DEFER_LDS=2 ;;
        dlds4) variant dlds4 -DTRT_DEFER_LDS=4 ;;
        dlds4b16) variant dlds4b16 -DTRT_DEFER_LDS=4 -DTRT_BVH_LDS_N=16 ;;
        persist1) variant persist1 -DTRT_PERSIST=1 -DTRT_PERSIST_WPC=20 ;;
        persist2) variant persist2 -DTRT_PERSIST=2 -DTRT_PERSIST_WPC=20 ;;
        persist4) variant persist4 -DTRT_PERSIST=4 -DTRT_PERSIST_WPC=20 ;;
        fmexec) variant fmexec -DTRT_FM_EXEC_BRANCH ;;
        nolds) variant nolds -DTRT_BVH_LDS=0 ;;
        bvh2) variant bvh2 -DTRT_BVH_WIDTH=2 ;;
        work) variant work -DTRT_DIAG_PIXEL_WORK ;;
        prev) # the kernel of git revision $PREV (default HEAD), for A/B against the work tree
            git -C "$ROOT" show "${PREV:-HEAD}:vkcomputeshader_tinyraytracer_amd/csrc/trt_kernel.hip" > "$SRC/.prev_kernel.hip"
            KSRC="$SRC/.prev_kernel.hip" variant prev
            rm -f "$SRC/.prev_kernel.hip" ;;
        tpw4) variant tpw4 -DTRT_TPW=4 ;;
        w5prio) variant w5prio -DTRT_WAVES=5 -DTRT_PRIO=3 ;;
        w4) variant w4 -DTRT_WAVES=4 ;;
        w6) variant w6 -DTRT_WAVES=6 ;;
        envpairs) variant envpairs -DTRT_ENV_PAIRS=1 ;;
        w4s16) variant w4s16 -DTRT_WAVES=4 -DTRT_BVH_LDS_N=16 ;;
        s16) variant s16 -DTRT_BVH_LDS_N=16 ;;
        noroot) variant noroot -DTRT_ROOT_SCALAR=0 ;;
        noempty) variant noempty -DTRT_BVH4_EMPTY_BOX=0 ;;
        g5) variant g5 -DTRT_G3_WAVES=5 -DTRT_G3_LDS=8 ;;
        g3lds16) variant g3lds16 -DTRT_G3_LDS=16 -DTRT_G3_WAVES_SHALLOW=4 ;;
        g4s8) variant g4s8 -DTRT_G3_LDS=8 ;;
        wpb2) variant wpb2 -DTRT_WPB=2 ;;
        wpb4) variant wpb4 -DTRT_WPB=4 ;;
        bgearly) variant bgearly -DTRT_BG_EARLY ;;
        noshare) variant noshare -DTRT_SHADOW_SHARE=0 ;;
        bgearly_wpb4) variant bgearly_wpb4 -DTRT_BG_EARLY -DTRT_WPB=4 ;;
        notrig) variant notrig -DTRT_DIAG_NO_UV_TRIG ;;
        pool64) variant pool64 -DTRT_DEFER_POOL_N=64 ;;
        norefill) variant norefill -DTRT_DEFER_REFILL=0 ;;
        t16) variant t16 -DTRT_REFILL_T=16 ;;
        t48) variant t48 -DTRT_REFILL_T=48 ;;
        t56) variant t56 -DTRT_REFILL_T=56 ;;
        srefill) variant srefill -DTRT_SHADOW_REFILL=1 ;;
        dw5) variant dw5 -DTRT_DEFER_WAVES=5 ;;
        dw6) variant dw6 -DTRT_DEFER_WAVES=6 ;;
        dw5p96) variant dw5p96 -DTRT_DEFER_WAVES=5 -DTRT_DEFER_POOL_N=96 ;;
        pool192) variant pool192 -DTRT_DEFER_POOL_N=192 ;;
        *) echo "unknown variant $v"; exit 2 ;;
    esac
done
