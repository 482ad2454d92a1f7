// trt_math.h — correctly rounded fp32 division / square root for the tracer's hot loop,
// shorter than the general sequences hipcc emits under -fhip-fp32-correctly-rounded-divide-sqrt.
//
// The arithmetic contract with the CPU oracle (oracle/trt_oracle.c) is IEEE binary32 with
// correctly rounded `/` and `sqrt`: every geometric decision (hit / miss, child rays) must be
// bit-identical.  hipcc's general lowering handles every input class (denormal scaling,
// div_scale / div_fmas / div_fixup for over/underflow): 15 VALU for sqrt, 11 for a divide.
// The operands on the tracer's paths are normal numbers of moderate size, so the functions
// below run the core of the same algorithms and fall back to the general sequence only when
// an operand leaves the range the core is exact on:
//
//   sqrt_rn(x):  v_sqrt_f32 (<= 1 ulp) then the +-1 ulp residual fix-up, for x >= 2^-96
//                (below that the general path rescales);
//   rcp_rn(b):   v_rcp_f32 then one Newton step in FMA, for 2^-125 <= |b| <= 2^125;
//   div_rn(a,b): Markstein's final correction q + (a - b q) y with y = rcp_rn(b), which is
//                the correctly rounded quotient when y is the correctly rounded reciprocal
//                and nothing over/underflows (|a|, |b| and |a/b| well inside the range).
//
// Exactness is established on the GPU by tools/dbg/fastmath_check.hip (built as
// ../fastmath_check by the Makefile, run by tests/test_gpu_fastmath.py): rcp_rn and sqrt_rn
// exhaustively over every fp32 input of their fast domain, div_rn over 2^32 random and
// structured operand pairs, all against hipcc's general correctly rounded sequences.
#pragma once

#include <hip/hip_runtime.h>

namespace trt {

// Fast-domain tests, kept as plain compares so a wave whose lanes all pass skips the
// general path with one branch.
__device__ __forceinline__ bool sqrt_fast_ok(float x) { return x >= 0x1p-96f && x <= 0x1p126f; }
__device__ __forceinline__ bool rcp_fast_ok(float b) {
    const float a = __builtin_fabsf(b);
    return a >= 0x1p-125f && a <= 0x1p125f;
}

// Core of the correctly rounded sqrt (LLVM's AMDGPU f32 fsqrt lowering without the
// denormal-range scaling): s = v_sqrt_f32(x) is within 1 ulp; the residuals of s -+ 1 ulp
// pick the correctly rounded neighbour.
__device__ __forceinline__ float sqrt_rn_core(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = rm <= 0.0f ? sm : s;
    r = rp > 0.0f ? sp : r;
    return r;
}

// Core of the correctly rounded reciprocal: v_rcp_f32 (1 ulp) + one FMA Newton step.
__device__ __forceinline__ float rcp_rn_core(float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}

// The general sequence runs only for lanes outside the fast domain, behind a wave-uniform
// branch (one compare + a scalar branch on its ballot when every lane is in range).
#ifndef TRT_FM_EXEC_BRANCH
#define TRT_FM_RARE(ok) __builtin_expect(__ballot(!(ok)) != 0ull, 0)
#endif

__device__ __forceinline__ float sqrt_rn(float x) {
#ifdef TRT_FM_EXEC_BRANCH
    if (__builtin_expect(sqrt_fast_ok(x), 1)) return sqrt_rn_core(x);
    return __builtin_sqrtf(x); // general correctly rounded sequence (compiled with -fhip-fp32-correctly-rounded-divide-sqrt)
#else
    float r = sqrt_rn_core(x);
    const bool ok = sqrt_fast_ok(x);
    if (TRT_FM_RARE(ok)) r = ok ? r : __builtin_sqrtf(x);
    return r;
#endif
}

__device__ __forceinline__ float rcp_rn(float b) {
#ifdef TRT_FM_EXEC_BRANCH
    if (__builtin_expect(rcp_fast_ok(b), 1)) return rcp_rn_core(b);
    return 1.0f / b;
#else
    float r = rcp_rn_core(b);
    const bool ok = rcp_fast_ok(b);
    if (TRT_FM_RARE(ok)) r = ok ? r : 1.0f / b;
    return r;
#endif
}

// rcp_rn for divergent per-lane loops (BVH / triangle tests): the general path behind an
// exec-masked branch instead of a ballot (measured faster there).
__device__ __forceinline__ float rcp_rn_lane(float b) {
    if (__builtin_expect(rcp_fast_ok(b), 1)) return rcp_rn_core(b);
    return 1.0f / b;
}

// a / b, correctly rounded.  Fast path: |b| in the rcp domain and |a| in [2^-100, 2^100]
// (or a == 0), which keeps a*y, b*q and the quotient far from over/underflow.
__device__ __forceinline__ bool div_fast_ok(float a, float b) {
    const float aa = __builtin_fabsf(a);
    return rcp_fast_ok(b) && ((aa >= 0x1p-100f && aa <= 0x1p100f) || a == 0.0f);
}
__device__ __forceinline__ float div_rn_core(float a, float b) {
    const float y = rcp_rn_core(b);
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ float div_rn(float a, float b) {
#ifdef TRT_FM_EXEC_BRANCH
    if (__builtin_expect(div_fast_ok(a, b), 1)) return div_rn_core(a, b);
    return a / b;
#else
    float r = div_rn_core(a, b);
    const bool ok = div_fast_ok(a, b);
    if (TRT_FM_RARE(ok)) r = ok ? r : a / b;
    return r;
#endif
}

// 1 / sqrt(x) as the two correctly rounded operations the contract prescribes
// (normalize(v) = v * (1 / sqrt(dot(v, v)))), one fast-domain test for both.
__device__ __forceinline__ float rsqrt_rn2(float x) {
#ifdef TRT_FM_EXEC_BRANCH
    if (__builtin_expect(sqrt_fast_ok(x), 1)) return rcp_rn_core(sqrt_rn_core(x));
    return 1.0f / __builtin_sqrtf(x);
#else
    float r = rcp_rn_core(sqrt_rn_core(x));
    const bool ok = sqrt_fast_ok(x);
    if (TRT_FM_RARE(ok)) r = ok ? r : 1.0f / __builtin_sqrtf(x);
    return r;
#endif
}

// sqrt(x) and 1 / sqrt(x), both correctly rounded (the contract's length(v) and normalize(v)
// of one vector), behind one fast-domain test: s = sqrt_rn(x), r = rcp_rn(s).  On the fast
// domain s lies in [2^-48, 2^63], inside rcp_rn_core's exact domain.
__device__ __forceinline__ float sqrt_rsqrt_rn(float x, float& r) {
#ifdef TRT_FM_EXEC_BRANCH
    if (__builtin_expect(sqrt_fast_ok(x), 1)) {
        const float s = sqrt_rn_core(x);
        r = rcp_rn_core(s);
        return s;
    }
    const float s = __builtin_sqrtf(x);
    r = 1.0f / s;
    return s;
#else
    float s = sqrt_rn_core(x);
    float q = rcp_rn_core(s);
    const bool ok = sqrt_fast_ok(x);
    if (TRT_FM_RARE(ok)) {
        s = ok ? s : __builtin_sqrtf(x);
        q = ok ? q : 1.0f / s;
    }
    r = q;
    return s;
#endif
}

} // namespace trt
