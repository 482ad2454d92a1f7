// trt_kernel.hip — the CDNA4 (gfx950) Whitted tracer: the hot path of the reference's
// compute shader (VulkanComputeShaderApplication/shaders/shader.comp:1-602) rebuilt for
// MI355X.
//
// Execution model
//   * One lane per pixel (per sample when spp > 1); a wave64 owns an 8x8 pixel tile and a
//     256-thread workgroup a 16x16 tile, so a wave's rays stay coherent and the batch /
//     triangle walks below are shared by all 64 lanes.
//   * The UBO (spheres, lights, camera; binding 0) rides in the kernarg segment (SGPRs).
//   * scene_intersect / shadow_intersect walk the AABB batches in index order exactly as
//     shader.comp:338-361 / 379-396 do, but wave-uniformly: a batch record is one scalar
//     load shared by the wave, `__ballot` over the lanes' slab tests skips a batch no lane
//     hits, and the hit batch's triangles are streamed as wave-uniform scalar loads
//     (v0, e1, e2 pre-subtracted on the host with the shader's own subtraction).
//   * The reference's 40-entry PathSegment stack with 32-entry volume stacks (~80 KB of
//     private memory per invocation) becomes "current segment + deferred
//     refraction children": the volume stack is provably inert and the
//     pop order (reflection before refraction, shader.comp:530/551/573) is preserved, so
//     colours accumulate in the reference order.  For max_depth <= 5 the deferred stack is
//     a register shift-stack; deeper trees use a small private array.
//   * Arithmetic contract shared with the CPU oracle: FP32, no contraction
//     (-ffp-contract=off), IEEE-correct division and square root, NaN-ignoring min/max.
#include <hip/hip_runtime.h>

#include <algorithm>


#include "../../include/trt/abi.h"
#include "trt_bands.h"
#include "trt_device.h"
#include "trt_math.h"

namespace trt {

// Orders one wave's LDS accesses (one wave per workgroup: the slab is private to the wave).
__device__ __forceinline__ void wave_lds_sync() { __syncthreads(); }
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x; }
// Rank of this lane among the set bits of `mask` below it.
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

#define TRT_EPS 0.0001f /* MIN_EPSILON, shader.comp:78 */
// Shadow queries of lights that add nothing lit or shadowed are not traced (cast_seg).
#ifndef TRT_SKIP_DARK
#define TRT_SKIP_DARK 1
#endif
// The specular term is not formed when its albedo weight is zero (cast_seg).
#ifndef TRT_SPEC_SKIP
#define TRT_SPEC_SKIP 1
#endif
#define TRT_PI 3.14159265358979323846f /* PI, shader.comp:82 */
#define TRT_GAMMA 2.2f /* GAMMA, shader.comp:81 */

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
// normalize / length with the contract's correctly rounded 1 / sqrt(.) (trt_math.h).
__device__ __forceinline__ f3 normalize3(f3 v) {
    float inv = rsqrt_rn2(dot3(v, v));
    return muls(v, inv);
}
__device__ __forceinline__ float length3(f3 v) { return sqrt_rn(dot3(v, v)); }
// normalize3(v) and length3(v) of one vector with one fast-domain test (trt_math.h)
#ifndef TRT_FUSED_NLEN
#define TRT_FUSED_NLEN 1
#endif
__device__ __forceinline__ f3 normalize_len3(f3 v, float& len) {
#if TRT_FUSED_NLEN
    float inv;
    len = sqrt_rsqrt_rn(dot3(v, v), inv);
    return muls(v, inv);
#else
    len = length3(v);
    return normalize3(v);
#endif
}
// GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N
__device__ __forceinline__ f3 reflect3(f3 I, f3 N) {
    float k = 2.0f * dot3(N, I);
    return sub(I, muls(N, k));
}
__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

// pow(x, y) for x >= 0, y > 0 (the only uses: the Phong exponent, shader.comp:502, and
// gamma, :598) as exp2(y * log2(x)) on the transcendental units (v_log_f32 / v_exp_f32):
// the form GLSL pow takes on GPUs (the Vulkan spec allows 3 + 2|x*log2 y| ulp).  x = 0 ->
// log2 = -inf -> exp2(-inf) = 0.  ocml's correctly-rounded-ish powf cost 14 us of a 61 us C2
// frame; the difference to the oracle's libm powf is a few ulp (tests/helpers.py FLOAT_TOL).
#ifdef TRT_LIBM_POW
__device__ __forceinline__ float pow_pos(float x, float y) { return powf(x, y); }
#else
__device__ __forceinline__ float pow_pos(float x, float y) {
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}
#endif
__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

// Linear -> sRGB transfer (IEC 61966-2-1) the presentation engine applies when shader.frag
// writes the sampled RGBA32F image (main.cpp:869) to the B8G8R8A8_SRGB swapchain
// (main.cpp:2341).  x in [0, 1].
__device__ __forceinline__ float srgb_encode(float x) {
    return x <= 0.0031308f ? 12.92f * x : 1.055f * pow_pos(x, 1.0f / 2.4f) - 0.055f;
}

// ---- primitives (shader.comp line refs) -------------------------------------------------

// ray_aabb_intersect, shader.comp:197-207
__device__ __forceinline__ bool aabb_hit(f3 o, f3 inv, const float* bmin, const float* bmax) {
    float t0x = (bmin[0] - o.x) * inv.x, t0y = (bmin[1] - o.y) * inv.y, t0z = (bmin[2] - o.z) * inv.z;
    float t1x = (bmax[0] - o.x) * inv.x, t1y = (bmax[1] - o.y) * inv.y, t1z = (bmax[2] - o.z) * inv.z;
    float tNear = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    float tFar = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return tNear <= tFar && tFar > TRT_EPS;
}

// ray_sphere_intersect, shader.comp:272-285
__device__ __forceinline__ bool sphere_hit(f3 o, f3 d, const SphereArg& s, float& t) {
    f3 L = sub(mk(s.c[0], s.c[1], s.c[2]), o);
    float tca = dot3(L, d);
    float d2 = dot3(L, L) - tca * tca;
    float r2 = s.r * s.r;
    if (d2 > r2) return false;
    float thc = sqrt_rn(r2 - d2);
    float t0 = tca - thc, t1 = tca + thc;
    if (t0 > TRT_EPS) t = t0;
    else if (t1 > TRT_EPS) t = t1;
    else return false;
    return true;
}

// custom_refract, shader.comp:209-221, called with eta_in = air (1.0)
__device__ __forceinline__ f3 custom_refract(f3 I, f3 N, float eta_out, float eta_in) {
    bool entering = dot3(I, N) < 0.0f;
    f3 fn = entering ? N : neg(N);
    float cosi = clamp01(dot3(neg(I), fn));
    // one quotient with selected operands (the same correctly rounded value either way)
    float eta = div_rn(entering ? eta_in : eta_out, entering ? eta_out : eta_in);
    float sint2 = eta * eta * (1.0f - cosi * cosi);
    if (sint2 > 1.0f) return mk(0.0f, 0.0f, 0.0f);
    float k = sqrt_rn(1.0f - sint2);
    f3 r = add(muls(I, eta), muls(fn, eta * cosi - k));
    return normalize3(r);
}

// ---- nearest hit (scene_intersect, shader.comp:295-362) ----------------------------------

enum : int { HIT_NONE = 0, HIT_FLOOR = 1, HIT_SPHERE = 2, HIT_TRI = 3 };

// Per-lane work counters (COUNT builds only): the units of trt_stats.
struct Cnt {
    uint32_t pri = 0, sec = 0, sh = 0, miss = 0, trin = 0, sph = 0, bt = 0, bh = 0, tt = 0, nt = 0;
    // Moller-Trumbore stages reached (the FP32 work units of the VALU roofline):
    // past the parallel test, past the u test, past the v test (t computed)
    uint32_t ta = 0, tu = 0, tv = 0;
    // shadow queries the frame skips (zero contribution) and the work inside them
    uint32_t sk = 0, ssph = 0, sbox = 0, stt = 0, sta = 0, stu = 0, stv = 0;
#ifdef TRT_DIAG_PIXEL_WORK
    uint32_t wn = 0, wt = 0, wseg = 0, wmax = 0; // diagnostic: this lane's node visits, tri tests, segments, max nodes/query
#endif
};

struct Hit {
    float t;
    int kind;
    int idx; // sphere index or triangle index
    float u, v;
    int ni;       // normal interpolation flag of the batch that produced the triangle hit
    uint32_t batch; // that batch (BVH tie-break on (t, batch, triangle))
};

// ---- batch walk: implicit 8-ary range hierarchy + the reference batch test -----------------
//
// Level 0 is the reference's batch list (Model records, shader.comp:338); level L >= 1 node k
// is the exact union box of batches [k*8^L, (k+1)*8^L).  The wave walks the tree depth-first,
// left to right, so leaves are visited in increasing batch index — the reference's loop
// order, which keeps its first-index-wins tie-break (strict `<`, shader.comp:349).  A lane
// that misses a node skips the node's whole range (`skip`); a lane reaching a leaf runs the
// reference's exact ray_aabb_intersect.  Internal nodes use node_hit(), which treats a slab
// whose product is NaN (0*inf: origin on the plane, zero direction component) as
// unconstrained; with that rule a node miss implies a miss of every batch below it
// (monotone FP32 rounding; tests/test_hierarchy_conservative.py), so the set of batches a
// lane tests triangles in is exactly the reference's.
__device__ __forceinline__ bool node_hit(f3 o, f3 inv, const float4& lo, const float4& hi) {
    const float INF = __builtin_huge_valf();
    float t0x = (lo.x - o.x) * inv.x, t1x = (hi.x - o.x) * inv.x;
    float t0y = (lo.y - o.y) * inv.y, t1y = (hi.y - o.y) * inv.y;
    float t0z = (lo.z - o.z) * inv.z, t1z = (hi.z - o.z) * inv.z;
    const bool nx = (t0x != t0x) || (t1x != t1x);
    const bool ny = (t0y != t0y) || (t1y != t1y);
    const bool nz = (t0z != t0z) || (t1z != t1z);
    const float mnx = nx ? -INF : fminf(t0x, t1x), mxx = nx ? INF : fmaxf(t0x, t1x);
    const float mny = ny ? -INF : fminf(t0y, t1y), mxy = ny ? INF : fmaxf(t0y, t1y);
    const float mnz = nz ? -INF : fminf(t0z, t1z), mxz = nz ? INF : fmaxf(t0z, t1z);
    const float tNear = fmaxf(fmaxf(mnx, mny), mnz);
    const float tFar = fminf(fminf(mxx, mxy), mxz);
    return tNear <= tFar && tFar > TRT_EPS;
}

// SHADOW = false: closest hit into h (shader.comp:338-361).  SHADOW = true: any hit with
// MIN_EPSILON < t < max_dist sets `occluded` (shader.comp:379-396).  A hit batch's triangles
// (v0, e1, e2: 48 B each) are staged through LDS 64 at a time by one coalesced load per
// lane, then read back as wave-wide broadcasts.
template <bool COUNT, bool SHADOW>
__device__ __forceinline__ void walk_batches(const KArgs& A, f3 o, f3 d, f3 inv, Hit& h, bool& occluded,
                                             float max_dist, Cnt& c, float4* slab) {
    const uint32_t nb = A.nbatch, top = A.top;
    uint32_t s = 0, L = top, skip = 0;
    while (s < nb) {
        const bool part = (!SHADOW || !occluded) && s >= skip;
        bool hit;
        BatchRec rec;
        if (L == 0) {
            rec = A.batches[s]; // wave-uniform: scalar load
            hit = part && aabb_hit(o, inv, rec.bmin, rec.bmax);
            if (COUNT && part) {
                ++c.bt;
                c.bh += hit ? 1u : 0u;
            }
        } else {
            const float4* nd = A.nodes + 2u * (A.node_off[L] + (s >> (3u * L)));
            const float4 lo = nd[0], hi = nd[1];
            hit = part && node_hit(o, inv, lo, hi);
            if (COUNT && part) ++c.nt;
        }
        const uint32_t span = 1u << (3u * L);
        if (part && !hit) skip = s + span;
        if (__ballot(hit) == 0) {
            if (SHADOW && __ballot(!occluded) == 0) return;
            s += span;
        } else if (L > 0) {
            --L; // descend into the first child; same start
            continue;
        } else {
            const int start = rec.start;
            const int count = rec.count_ni & 0x7fffffff;
            const int ni = (rec.count_ni >> 31) & 1;
            // The lanes still active here (not every lane of the tile: edge pixels and lanes
            // whose ray tree is done are masked) stage the slab together, by active-lane rank.
            const uint64_t act = __ballot(true);
            const uint32_t nact = (uint32_t)__popcll(act);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
            for (int base = 0; base < count; base += 64) {
                const int n = min(64, count - base);
                wave_lds_sync(); // orders the LDS reads of the previous slab
                for (uint32_t i = rank; i < (uint32_t)n; i += nact) {
                    const float4* g = reinterpret_cast<const float4*>(A.geo + start + base + (int)i);
                    slab[i * 3u + 0u] = g[0];
                    slab[i * 3u + 1u] = g[1];
                    slab[i * 3u + 2u] = g[2];
                }
                wave_lds_sync();
                if (hit) {
                    for (int k = 0; k < n; ++k) { // shader.comp:344-359 / 384-393
                        const float4 ga = slab[k * 3 + 0], gb = slab[k * 3 + 1], gc = slab[k * 3 + 2];
                        if (COUNT) ++c.tt;
                        const f3 v0 = mk(ga.x, ga.y, ga.z), e1 = mk(ga.w, gb.x, gb.y), e2 = mk(gb.z, gb.w, gc.x);
                        f3 hv = cross3(d, e2);
                        float a = dot3(e1, hv);
                        if (a > -TRT_EPS && a < TRT_EPS) continue;
                        if (COUNT) ++c.ta;
                        float f = rcp_rn_lane(a);
                        f3 sv = sub(o, v0);
                        float u = f * dot3(sv, hv);
                        if (u < 0.0f || u > 1.0f) continue;
                        if (COUNT) ++c.tu;
                        f3 q = cross3(sv, e1);
                        float v = f * dot3(d, q);
                        if (v < 0.0f || u + v > 1.0f) continue;
                        if (COUNT) ++c.tv;
                        float t = f * dot3(e2, q);
                        if (t <= TRT_EPS) continue;
                        if (SHADOW) {
                            if (t > TRT_EPS && t < max_dist) {
                                occluded = true;
                                break;
                            }
                        } else if (t > TRT_EPS && t < h.t) {
                            h.t = t;
                            h.kind = HIT_TRI;
                            h.idx = start + base + k;
                            h.u = u;
                            h.v = v;
                            h.ni = ni;
                        }
                    }
                }
            }
            if (SHADOW && __ballot(!occluded) == 0) return;
            s += 1;
        }
        while (L < top && (s & ((1u << (3u * (L + 1u))) - 1u)) == 0u) ++L; // climb to the aligned level
    }
}

// ---- per-lane BVH traversal (bvh_build.cpp) ----------------------------------------------
//
// Each lane walks the BVH2 on its own (ordered: nearer child first, farther child on a private
// stack), which suits incoherent refracted / shadow rays far better than the wave-wide batch
// walk.  The result is the reference's: a triangle candidate (MT hit, t > MIN_EPSILON) is
// accepted only if its batch passes ray_aabb_intersect exactly as in shader.comp:339, and it
// replaces the current best only if t is smaller or t is equal and (batch, triangle) comes
// first in the reference's loop order (its strict `t < nearest` keeps the first candidate).

// Reciprocal direction for the BVH's culling tests: components smaller than 1e-30 in
// magnitude become +-1e-30 first, so inv is finite and no slab product is 0 * inf (the NaN
// checks this saves were 60 VALU per BVH4 node visit: C3 -3 %, C4 -2 %, shipped frame -4 %).
// Over the t range of a query (< 1e10) such a ray drifts < 1e-20 along that axis, far inside
// the boxes' padding (>= 1e-6), so the culling stays conservative.  The reference's own batch
// gate keeps the exact 1/d (ray_aabb_intersect, shader.comp:197-207, 336).
__device__ __forceinline__ f3 cull_inv(f3 d) {
    auto f = [](float x) { return rcp_rn_lane(__builtin_fabsf(x) < 1e-30f ? __builtin_copysignf(1e-30f, x) : x); };
    return mk(f(d.x), f(d.y), f(d.z));
}
// The exact 1/d of the reference's batch gate, computed per triangle candidate.
__device__ __forceinline__ f3 gate_inv(f3 d) {
    return mk(rcp_rn_lane(d.x), rcp_rn_lane(d.y), rcp_rn_lane(d.z)); // shader.comp:336 / 377
}

// Padded-box entry test with distance pruning: enter if the slab interval is non-empty, ends
// beyond MIN_EPSILON, and starts no later than `best`.  NaN slabs are unconstrained.
__device__ __forceinline__ bool bvh_box(f3 o, f3 inv, const float* lo, const float* hi, float best,
                                        float& tnear) {
    // inv comes from cull_inv(): finite, so a slab product is NaN only where the origin is NaN
    // on that axis (both ends NaN), which the NaN-ignoring min/max leave unconstrained.
    const float t0x = (lo[0] - o.x) * inv.x, t1x = (hi[0] - o.x) * inv.x;
    const float t0y = (lo[1] - o.y) * inv.y, t1y = (hi[1] - o.y) * inv.y;
    const float t0z = (lo[2] - o.z) * inv.z, t1z = (hi[2] - o.z) * inv.z;
    tnear = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tfar = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return tnear <= tfar && tfar > TRT_EPS && tnear <= best;
}

// Traversal stack: the first kBvhLdsStack entries in LDS ([entry][lane], conflict-free
// ds_read/write_b32, ~50-cycle pops), deeper ones in a private (scratch) array.
#ifndef TRT_BVH_LDS
#define TRT_BVH_LDS 1
#endif
#ifndef TRT_BVH_LDS_N
#define TRT_BVH_LDS_N 24
#endif
constexpr int kBvhLdsStack = TRT_BVH_LDS ? TRT_BVH_LDS_N : 0;

// GEOM 3 is the BVH walk compiled for 4 waves per SIMD (<= 128 VGPRs), or 5 (<= 96 VGPRs)
// for plain frames of max_depth <= 4 (CAP <= 3, TRT_G3_WAVES_SHALLOW): 5 waves: C4 2.69 ->
// 2.63 ms, depth-2 C4 -5.5 %, C3 within noise (profiles/r03_ab_g5.log).  LDS per wave: the
// traversal stack's first TRT_G3_LDS entries (16: 4 KB).  Round 3 kept 8 entries beside 6 KB
// of deferred children (20 waves x 8 KB fill a CU's 160 KB); the children now live in a
// private array (TRT_G3_SEG_PRIV: a glass hit's rare push) and the stack takes the LDS:
// C4 2.626 -> 2.505 ms, C3 -5.7 %, the deferred frames unchanged; 16, 20, 24, 28 entries tie,
// 32 entries and the 4-wave build with them are slower (profiles/r04o_ab_g3_lds_stack.jsonl,
// r04p_ab_g3_lds_sweep.jsonl).  16 leaves pass A of deferred frames (5 KB segment pool + the
// stack) at 4 waves per SIMD.
#ifndef TRT_G3_WAVES
#define TRT_G3_WAVES 4
#endif
#ifndef TRT_G3_WAVES_SHALLOW
#define TRT_G3_WAVES_SHALLOW 5
#endif
#ifndef TRT_G3_LDS
#define TRT_G3_LDS 16
#endif
template <int GEOM>
constexpr int bvh_lds_entries() { return GEOM == 3 ? (TRT_BVH_LDS ? TRT_G3_LDS : 0) : kBvhLdsStack; }
// 32-bit words of a wave's BVH-stack LDS (slab_float4s below holds them)
template <int GEOM>
constexpr int slab_words() { return bvh_lds_entries<GEOM>() * 64; }
// PUSH3: the branch-free push of up to three children (push_sorted) — used by the 3-wave
// build: C3 -4 %, shipped frame -6 %; the 4-wave build (128-VGPR cap) is 3 % slower with it
// (profiles/r01_ab_push3.log).
// The private tail lives in a separate array of the caller (Mem): a stack object holding the
// dynamically indexed array AND its top index was one scratch allocation, so `sp` itself was
// kept in scratch memory and every push / pop paid a scratch load + store of it (seen in the
// ISA: scratch_load_dword ... offset:200 on every visit).  With the array apart, the stack
// object is scalarised and sp lives in a register.
// The LDS column is an address-space-3 pointer: with a generic one the compiler turned the pop's
// `sp < N ? lds[..] : priv[..]` into one load through a selected generic pointer, i.e. a
// flat_load that goes through the vector-memory pipe (TA/TD) even for LDS entries.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) float lds_f32;
template <int N, bool PUSH3 = false>
struct BvhStack {
    struct Mem {
        uint32_t priv[kBvhStack - N];
    };
    lds_u32* lds;   // this lane's column
    uint32_t* priv; // the caller's private tail (scratch)
    int sp = 0;
    __device__ __forceinline__ BvhStack(float4* slab, Mem& m)
        : lds((lds_u32*)(reinterpret_cast<uint32_t*>(slab) + lane_id())), priv(m.priv) {}
    __device__ __forceinline__ void push(uint32_t v) {
        if (sp < N) lds[sp * 64] = v;
        else priv[sp - N] = v;
        ++sp;
    }
    __device__ __forceinline__ uint32_t pop() {
        --sp;
        uint32_t v;
        if (sp < N) v = lds[sp * 64];
        else v = priv[sp - N];
        return v;
    }
    // Pushes r[nh-1], ..., r[1] (r[1] ends on top), nh in 1..4.  While three more entries fit
    // the LDS part, the three stores are unconditional: an unused one goes to slot sp + 3,
    // above the new top.
    __device__ __forceinline__ void push_sorted(const uint32_t (&r)[4], int nh) {
        if (PUSH3 && sp + 3 < N) {
#pragma unroll
            for (int k = 1; k < 4; ++k) {
                const int pos = k < nh ? sp + nh - 1 - k : sp + 3;
                lds[pos * 64] = r[k];
            }
            sp += nh - 1;
            return;
        }
        if (nh > 3) push(r[3]);
        if (nh > 2) push(r[2]);
        if (nh > 1) push(r[1]);
    }
};

template <bool COUNT, bool SHADOW, int GEOM>
__device__ __forceinline__ void trace_bvh(const KArgs& A, f3 o, f3 d, f3 inv, Hit& h, bool& occluded,
                                          float max_dist, Cnt& c, float4* slab) {
    using Stack = BvhStack<bvh_lds_entries<GEOM>(), GEOM == 2>;
    typename Stack::Mem stack_mem;
    Stack stack(slab, stack_mem);
    uint32_t node = 0;
    float best = SHADOW ? max_dist : h.t;
#ifdef TRT_DIAG_PIXEL_WORK
    uint32_t qn = 0;
#endif
    for (;;) {
        if (!(node & kBvhLeafBit)) {
#ifdef TRT_DIAG_PIXEL_WORK
            ++c.wn;
            ++qn;
            c.wmax = max(c.wmax, qn);
#endif
            const BvhNode nd = A.bvh[node];
            float ta, tb;
            const bool ha = bvh_box(o, inv, nd.lo0, nd.hi0, best, ta);
            const bool hb = bvh_box(o, inv, nd.lo1, nd.hi1, best, tb);
            if (COUNT) c.nt += 2;
            if (ha && hb) {
                const bool a_first = ta <= tb;
                stack.push(a_first ? nd.child[1] : nd.child[0]);
                node = a_first ? nd.child[0] : nd.child[1];
                continue;
            }
            if (ha || hb) {
                node = ha ? nd.child[0] : nd.child[1];
                continue;
            }
        } else {
            const uint32_t first = node & kBvhFirstMask;
            const uint32_t n = ((node >> kBvhCountShift) & 15u) + 1u;
            for (uint32_t k = first; k < first + n; ++k) {
                const TriGeo g = A.bvh_tris[k];
                if (COUNT) ++c.tt;
#ifdef TRT_DIAG_PIXEL_WORK
                ++c.wt;
#endif
                const f3 v0 = ld3(g.v0), e1 = ld3(g.e1), e2 = ld3(g.e2);
                f3 hv = cross3(d, e2);
                float a = dot3(e1, hv);
                if (a > -TRT_EPS && a < TRT_EPS) continue;
                        if (COUNT) ++c.ta;
                float f = rcp_rn_lane(a);
                f3 sv = sub(o, v0);
                float u = f * dot3(sv, hv);
                if (u < 0.0f || u > 1.0f) continue;
                        if (COUNT) ++c.tu;
                f3 q = cross3(sv, e1);
                float v = f * dot3(d, q);
                if (v < 0.0f || u + v > 1.0f) continue;
                        if (COUNT) ++c.tv;
                float t = f * dot3(e2, q);
                if (t <= TRT_EPS) continue;
                const uint32_t tri = __float_as_uint(g.pad[0]), batch = __float_as_uint(g.pad[1]);
                if (SHADOW) {
                    if (!(t < max_dist)) continue;
                } else {
                    const bool better = t < best || (t == best && h.kind == HIT_TRI &&
                                                     (batch < h.batch || (batch == h.batch && (int)tri < h.idx)));
                    if (!better) continue;
                }
                const BatchRec rec = A.batches[batch]; // the reference's gate for this triangle
                const bool pass = aabb_hit(o, gate_inv(d), rec.bmin, rec.bmax);
                if (COUNT) {
                    ++c.bt;
                    c.bh += pass ? 1u : 0u;
                }
                if (!pass) continue;
                if (SHADOW) {
                    occluded = true;
                    return;
                }
                best = t;
                h.t = t;
                h.kind = HIT_TRI;
                h.idx = (int)tri;
                h.batch = batch;
                h.u = u;
                h.v = v;
                h.ni = (int)__float_as_uint(g.pad[2]);
            }
        }
        if (stack.sp == 0) return;
        node = stack.pop();
    }
}

// Tests the leaf `node` (1-4 triangles of the BVH-ordered array).  SHADOW: returns true when
// an accepted candidate occludes.  The next triangle's record is loaded before the current
// one is tested (one exposed load latency per leaf instead of one per triangle).
template <bool COUNT, bool SHADOW>
__device__ __forceinline__ bool bvh_leaf(const KArgs& A, uint32_t node, f3 o, f3 d, f3 inv, Hit& h,
                                         float max_dist, float& best, Cnt& c) {
    const uint32_t first = node & kBvhFirstMask;
    const uint32_t n = ((node >> kBvhCountShift) & 15u) + 1u;
#ifndef TRT_LEAF_PREFETCH
#define TRT_LEAF_PREFETCH 1
#endif
    TriGeo g = A.bvh_tris[first];
    for (uint32_t k = first; k < first + n; ++k) {
        const TriGeo cur = TRT_LEAF_PREFETCH ? g : A.bvh_tris[k];
        if (TRT_LEAF_PREFETCH && k + 1 < first + n) g = A.bvh_tris[k + 1];
        if (COUNT) ++c.tt;
#ifdef TRT_DIAG_PIXEL_WORK
        ++c.wt;
#endif
        const f3 v0 = ld3(cur.v0), e1 = ld3(cur.e1), e2 = ld3(cur.e2);
        f3 hv = cross3(d, e2);
        float a = dot3(e1, hv);
        if (a > -TRT_EPS && a < TRT_EPS) continue;
                        if (COUNT) ++c.ta;
        float f = rcp_rn_lane(a);
        f3 sv = sub(o, v0);
        float u = f * dot3(sv, hv);
        if (u < 0.0f || u > 1.0f) continue;
                        if (COUNT) ++c.tu;
        f3 q = cross3(sv, e1);
        float v = f * dot3(d, q);
        if (v < 0.0f || u + v > 1.0f) continue;
                        if (COUNT) ++c.tv;
        float t = f * dot3(e2, q);
        if (t <= TRT_EPS) continue;
        const uint32_t tri = __float_as_uint(cur.pad[0]), batch = __float_as_uint(cur.pad[1]);
        if (SHADOW) {
            if (!(t < max_dist)) continue;
        } else {
            const bool better = t < best || (t == best && h.kind == HIT_TRI &&
                                             (batch < h.batch || (batch == h.batch && (int)tri < h.idx)));
            if (!better) continue;
        }
        const BatchRec rec = A.batches[batch]; // the reference's gate for this triangle
        const bool pass = aabb_hit(o, gate_inv(d), rec.bmin, rec.bmax);
        if (COUNT) {
            ++c.bt;
            c.bh += pass ? 1u : 0u;
        }
        if (!pass) continue;
        if (SHADOW) {
            h.idx = (int)k; // the occluder's BVH-ordered index (shared with the wave, trace_bvh4)
            return true;
        }
        best = t;
        h.t = t;
        h.kind = HIT_TRI;
        h.idx = (int)tri;
        h.batch = batch;
        h.u = u;
        h.v = v;
        h.ni = (int)__float_as_uint(cur.pad[2]);
    }
    return false;
}

// Shadow test of one triangle (BVH-ordered index k, wave-uniform) read through scalar loads:
// bvh_leaf's test term for term (Moller-Trumbore, t in (MIN_EPSILON, max_dist), the reference's
// batch gate), so a hit is a genuine occluder of this lane's query.
__device__ __forceinline__ bool shadow_tri_s(const KArgs& A, uint32_t k, f3 o, f3 d, float max_dist) {
    typedef __attribute__((address_space(4))) const float cfloat;
    const cfloat* T = (const cfloat*)(A.bvh_tris + k);
    const f3 v0 = mk(T[0], T[1], T[2]), e1 = mk(T[3], T[4], T[5]), e2 = mk(T[6], T[7], T[8]);
    f3 hv = cross3(d, e2);
    float a = dot3(e1, hv);
    if (a > -TRT_EPS && a < TRT_EPS) return false;
    float f = rcp_rn_lane(a);
    f3 sv = sub(o, v0);
    float u = f * dot3(sv, hv);
    if (u < 0.0f || u > 1.0f) return false;
    f3 q = cross3(sv, e1);
    float v = f * dot3(d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * dot3(e2, q);
    if (t <= TRT_EPS) return false;
    if (!(t < max_dist)) return false;
    const uint32_t batch = __builtin_amdgcn_readfirstlane(__float_as_uint(T[10]));
    const cfloat* B = (const cfloat*)(A.batches + batch);
    const float bmin[3] = {B[0], B[1], B[2]}, bmax[3] = {B[3], B[4], B[5]};
    return aabb_hit(o, gate_inv(d), bmin, bmax);
}

#ifndef TRT_BVH_WIDTH
#define TRT_BVH_WIDTH 4
#endif

#ifndef TRT_BVH4_EMPTY_BOX
#define TRT_BVH4_EMPTY_BOX 1
#endif
// One BVH4 node visit: the four child boxes tested against the ray, the entered children
// sorted nearest first; the nearest becomes `node`, the others are pushed farthest first (so
// the next pop is the next nearest).  Returns false when no child is entered.
template <bool COUNT, typename Stack>
__device__ __forceinline__ bool visit4(f3 o, f3 inv, float best, const float4& lx, const float4& ly,
                                       const float4& lz, const float4& hx, const float4& hy, const float4& hz,
                                       const uint4& ch, Stack& stack, uint32_t& node, Cnt& c) {
    float t[4];
    uint32_t r[4] = {ch.x, ch.y, ch.z, ch.w};
    const float lo[4][3] = {{lx.x, ly.x, lz.x}, {lx.y, ly.y, lz.y}, {lx.z, ly.z, lz.z}, {lx.w, ly.w, lz.w}};
    const float hi[4][3] = {{hx.x, hy.x, hz.x}, {hx.y, hy.y, hz.y}, {hx.z, hy.z, hz.z}, {hx.w, hy.w, hz.w}};
    int nh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float tn;
#if TRT_BVH4_EMPTY_BOX
        const bool ok = bvh_box(o, inv, lo[i], hi[i], best, tn); // unused slots: an all-NaN box, never entered
#else
        const bool ok = r[i] != kBvh4None && bvh_box(o, inv, lo[i], hi[i], best, tn);
#endif
        t[i] = ok ? tn : __builtin_huge_valf();
        nh += ok ? 1 : 0;
    }
    if (COUNT) c.nt += (ch.x != kBvh4None) + (ch.y != kBvh4None) + (ch.z != kBvh4None) + (ch.w != kBvh4None);
    if (nh == 0) return false;
    // sorting network on (t, ref): ascending t, misses (t = inf) last
#define TRT_CSWAP(a, b)                                   \
    do {                                                  \
        const bool sw = t[b] < t[a];                      \
        const float ta = t[a], tb = t[b];                 \
        const uint32_t ra = r[a], rb = r[b];              \
        t[a] = sw ? tb : ta;                              \
        t[b] = sw ? ta : tb;                              \
        r[a] = sw ? rb : ra;                              \
        r[b] = sw ? ra : rb;                              \
    } while (0)
    TRT_CSWAP(0, 1);
    TRT_CSWAP(2, 3);
    TRT_CSWAP(0, 2);
    TRT_CSWAP(1, 3);
    TRT_CSWAP(1, 2);
#undef TRT_CSWAP
    stack.push_sorted(r, nh);
    node = r[0];
    return true;
}

// Quantized 4-wide node (trt_device.h Bvh4QNode): per axis the plane of byte q is p + q * s,
// so its slab distance is (p - o) * inv + q * (s * inv) = A + q * B, one FMA per plane after
// three products per axis (the culling test may round freely: the boxes carry a margin of a
// grid step plus the padding, far above this rounding, so a fused multiply-add is fine here
// and only here).  The near / far plane of each axis is picked by the sign of inv once per
// node, so a child needs no per-axis min / max, and an inverted (unused) box is never entered.
#ifndef TRT_BVH_QUANT
#define TRT_BVH_QUANT 1
#endif
template <bool COUNT, typename Stack>
__device__ __forceinline__ bool visit4q(f3 o, f3 inv, float best, const float4& pe, const uint4& qa,
                                        const uint4& qb, const uint4& ch, Stack& stack, uint32_t& node, Cnt& c) {
    const uint32_t ex = __float_as_uint(pe.w);
    const float sx = __uint_as_float((ex & 0xffu) << 23);
    const float sy = __uint_as_float(((ex >> 8) & 0xffu) << 23);
    const float sz = __uint_as_float(((ex >> 16) & 0xffu) << 23);
    const float ax = (pe.x - o.x) * inv.x, bx = sx * inv.x;
    const float ay = (pe.y - o.y) * inv.y, by = sy * inv.y;
    const float az = (pe.z - o.z) * inv.z, bz = sz * inv.z;
    // qa = (qlo.x, qlo.y, qlo.z, qhi.x), qb = (qhi.y, qhi.z, -, -)
    const uint32_t nx = inv.x >= 0.0f ? qa.x : qa.w, fx = inv.x >= 0.0f ? qa.w : qa.x;
    const uint32_t ny = inv.y >= 0.0f ? qa.y : qb.x, fy = inv.y >= 0.0f ? qb.x : qa.y;
    const uint32_t nz = inv.z >= 0.0f ? qa.z : qb.y, fz = inv.z >= 0.0f ? qb.y : qa.z;
    float t[4];
    uint32_t r[4] = {ch.x, ch.y, ch.z, ch.w};
    int nh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int sh = 8 * i;
        const float tnx = __builtin_fmaf((float)((nx >> sh) & 0xffu), bx, ax);
        const float tny = __builtin_fmaf((float)((ny >> sh) & 0xffu), by, ay);
        const float tnz = __builtin_fmaf((float)((nz >> sh) & 0xffu), bz, az);
        const float tfx = __builtin_fmaf((float)((fx >> sh) & 0xffu), bx, ax);
        const float tfy = __builtin_fmaf((float)((fy >> sh) & 0xffu), by, ay);
        const float tfz = __builtin_fmaf((float)((fz >> sh) & 0xffu), bz, az);
        const float tn = fmaxf(fmaxf(tnx, tny), tnz);
        const float tf = fminf(fminf(tfx, tfy), tfz);
        const bool ok = tn <= tf && tf > TRT_EPS && tn <= best;
        t[i] = ok ? tn : __builtin_huge_valf();
        nh += ok ? 1 : 0;
    }
    if (COUNT) c.nt += (ch.x != kBvh4None) + (ch.y != kBvh4None) + (ch.z != kBvh4None) + (ch.w != kBvh4None);
    if (nh == 0) return false;
#define TRT_CSWAP(a, b)                                   \
    do {                                                  \
        const bool sw = t[b] < t[a];                      \
        const float ta = t[a], tb = t[b];                 \
        const uint32_t ra = r[a], rb = r[b];              \
        t[a] = sw ? tb : ta;                              \
        t[b] = sw ? ta : tb;                              \
        r[a] = sw ? rb : ra;                              \
        r[b] = sw ? ra : rb;                              \
    } while (0)
    TRT_CSWAP(0, 1);
    TRT_CSWAP(2, 3);
    TRT_CSWAP(0, 2);
    TRT_CSWAP(1, 3);
    TRT_CSWAP(1, 2);
#undef TRT_CSWAP
    stack.push_sorted(r, nh);
    node = r[0];
    return true;
}

// 4-wide traversal: the four child boxes of a node in one 128-B fetch, entered nearest first.
// The root is the same node for every lane: its record is read with wave-uniform (scalar)
// loads, which the scalar cache serves, instead of a dependent per-lane vector fetch at the
// start of every query.
#ifndef TRT_ROOT_SCALAR
#define TRT_ROOT_SCALAR 1
#endif
// Wave-uniform node fetch: when every lane at an internal node visits the same node, one scalar
// fetch replaces the per-lane loads (C4 -4 %, C3 -1 %, shipped frame -3 %: the walk is bound by
// the vector-memory pipe, TA/TD, not by bytes; profiles/r03_ab_c4_walk.log).
#ifndef TRT_UNIFORM_NODE
#define TRT_UNIFORM_NODE 1
#endif
// GEOM 3 kernels walk the quantized nodes only (the host picks GEOM 3 only when they exist):
// the 64-B-node and binary walks are not compiled into them, so the register allocation of
// the 96-VGPR (5-wave) build sees one walk per call site.
#ifndef TRT_G3_QONLY
#define TRT_G3_QONLY 1
#endif
template <int GEOM>
constexpr bool g3_quant_only() { return GEOM == 3 && TRT_G3_QONLY && TRT_BVH_QUANT; }
template <bool COUNT, bool SHADOW, int GEOM>
__device__ __forceinline__ void trace_bvh4(const KArgs& A, f3 o, f3 d, f3 inv, Hit& h, bool& occluded,
                                           float max_dist, Cnt& c, float4* slab) {
    using Stack = BvhStack<bvh_lds_entries<GEOM>(), GEOM == 2>;
    typename Stack::Mem stack_mem;
    Stack stack(slab, stack_mem);
    uint32_t node = 0;
    float best = SHADOW ? max_dist : h.t;
#if TRT_BVH_QUANT
    // measured: -3 % on C4 (1,600 batches, 4-wave build), +2..3 % on C3 / the shipped frame
    // (profiles/r02_ab_quant.log), so the quantized nodes serve the 4-wave build only
    if (GEOM == 3 && (g3_quant_only<GEOM>() || A.bvh4q)) {
        {
            typedef __attribute__((address_space(4))) const float cfloat;
            typedef __attribute__((address_space(4))) const uint32_t cuint;
            const cfloat* R = (const cfloat*)(A.bvh4q);
            const cuint* RC = (const cuint*)(A.bvh4q);
            const float4 pe = make_float4(R[0], R[1], R[2], R[3]);
            const uint4 qa = make_uint4(RC[4], RC[5], RC[6], RC[7]);
            const uint4 qb = make_uint4(RC[8], RC[9], RC[10], RC[11]);
            const uint4 ch = make_uint4(RC[12], RC[13], RC[14], RC[15]);
#ifdef TRT_DIAG_PIXEL_WORK
            ++c.wn;
#endif
            if (!visit4q<COUNT>(o, inv, best, pe, qa, qb, ch, stack, node, c)) return;
        }
        auto fetch = [&](uint32_t nd, float4& pe, uint4& qa, uint4& qb, uint4& ch) {
#if TRT_UNIFORM_NODE
            // every lane at an internal node visits the same node (coherent rays, top levels):
            // one scalar fetch for the wave instead of 4 per-lane dwordx4 loads through TA/TD
            const uint32_t n0 = __builtin_amdgcn_readfirstlane(nd);
            if (__ballot(nd != n0) == 0ull) {
                typedef __attribute__((address_space(4))) const float cfloat;
                typedef __attribute__((address_space(4))) const uint32_t cuint;
                const cfloat* R = (const cfloat*)(A.bvh4q + n0);
                const cuint* RC = (const cuint*)(A.bvh4q + n0);
                pe = make_float4(R[0], R[1], R[2], R[3]);
                qa = make_uint4(RC[4], RC[5], RC[6], RC[7]);
                qb = make_uint4(RC[8], RC[9], RC[10], RC[11]);
                ch = make_uint4(RC[12], RC[13], RC[14], RC[15]);
                return;
            }
#endif
            const float4* p = reinterpret_cast<const float4*>(A.bvh4q + nd);
            pe = p[0];
            qa = reinterpret_cast<const uint4*>(p)[1];
            qb = reinterpret_cast<const uint4*>(p)[2];
            ch = reinterpret_cast<const uint4*>(p)[3];
        };
        for (;;) {
            if (!(node & kBvhLeafBit)) {
                float4 pe;
                uint4 qa, qb, ch;
                fetch(node, pe, qa, qb, ch);
#ifdef TRT_DIAG_PIXEL_WORK
                ++c.wn;
#endif
                if (visit4q<COUNT>(o, inv, best, pe, qa, qb, ch, stack, node, c)) continue;
            } else if (bvh_leaf<COUNT, SHADOW>(A, node, o, d, inv, h, max_dist, best, c)) {
                occluded = true;
                return;
            }
            if (stack.sp == 0) return;
            node = stack.pop();
        }
    }
#endif
    if constexpr (g3_quant_only<GEOM>()) return;
#if TRT_ROOT_SCALAR
    {
        // constant address space: the compiler may (and, the address being uniform, does) use
        // scalar loads; the BVH is read-only for the whole launch
        typedef __attribute__((address_space(4))) const float cfloat;
        typedef __attribute__((address_space(4))) const uint32_t cuint;
        const cfloat* R = (const cfloat*)(A.bvh4);
        const cuint* RC = (const cuint*)(A.bvh4);
#ifdef TRT_DIAG_PIXEL_WORK
        ++c.wn;
#endif
        const float4 lx = make_float4(R[0], R[1], R[2], R[3]);
        const float4 ly = make_float4(R[4], R[5], R[6], R[7]);
        const float4 lz = make_float4(R[8], R[9], R[10], R[11]);
        const float4 hx = make_float4(R[12], R[13], R[14], R[15]);
        const float4 hy = make_float4(R[16], R[17], R[18], R[19]);
        const float4 hz = make_float4(R[20], R[21], R[22], R[23]);
        const uint4 ch = make_uint4(RC[24], RC[25], RC[26], RC[27]);
        if (!visit4<COUNT>(o, inv, best, lx, ly, lz, hx, hy, hz, ch, stack, node, c)) return;
    }
#endif
    for (;;) {
        if (!(node & kBvhLeafBit)) {
            float4 lx, ly, lz, hx, hy, hz;
            uint4 ch;
#if TRT_UNIFORM_NODE
            const uint32_t n0 = __builtin_amdgcn_readfirstlane(node);
            if (__ballot(node != n0) == 0ull) { // one scalar fetch for the wave (see visit4q's loop)
                typedef __attribute__((address_space(4))) const float cfloat;
                typedef __attribute__((address_space(4))) const uint32_t cuint;
                const cfloat* R = (const cfloat*)(A.bvh4 + n0);
                const cuint* RC = (const cuint*)(A.bvh4 + n0);
                lx = make_float4(R[0], R[1], R[2], R[3]);
                ly = make_float4(R[4], R[5], R[6], R[7]);
                lz = make_float4(R[8], R[9], R[10], R[11]);
                hx = make_float4(R[12], R[13], R[14], R[15]);
                hy = make_float4(R[16], R[17], R[18], R[19]);
                hz = make_float4(R[20], R[21], R[22], R[23]);
                ch = make_uint4(RC[24], RC[25], RC[26], RC[27]);
            } else
#endif
            {
                const float4* p = reinterpret_cast<const float4*>(A.bvh4 + node);
                lx = p[0], ly = p[1], lz = p[2], hx = p[3], hy = p[4], hz = p[5];
                ch = reinterpret_cast<const uint4*>(p)[6];
            }
#ifdef TRT_DIAG_PIXEL_WORK
            ++c.wn;
#endif
            if (visit4<COUNT>(o, inv, best, lx, ly, lz, hx, hy, hz, ch, stack, node, c)) continue;
        } else if (bvh_leaf<COUNT, SHADOW>(A, node, o, d, inv, h, max_dist, best, c)) {
            occluded = true;
            return;
        }
        if (stack.sp == 0) return;
        node = stack.pop();
    }
}

// A ray whose origin or direction is NaN on every axis (e.g. the children and shadow rays of
// a hit whose smooth normal normalised a zero vector: 0 * inf) makes every slab of
// ray_aabb_intersect NaN, so the reference's batch test (shader.comp:197-207) fails for every
// batch and no triangle can be hit.  The conservative hierarchies treat NaN slabs as
// unconstrained and would visit every node to find that out (a full BVH traversal, ~1 ms):
// skip the mesh instead — the same (empty) result.
__device__ __forceinline__ bool ray_misses_all_batches(f3 o, f3 d) {
    return (o.x != o.x || d.x != d.x) && (o.y != o.y || d.y != d.y) && (o.z != o.z || d.z != d.z);
}

// Wave-coherent any-hit walk of the quantized BVH4 for shadow rays.  The shading loop queries
// one light at a time (shade loop below), so the rays a wave asks about at once share their end
// point and, from a tile's neighbouring shading points, nearly share their origin: they visit
// nearly the same nodes.  Here the wave walks ONE node sequence: a child is entered when any
// lane still walking enters it, nodes and leaf triangles are read with scalar loads (one fetch
// per wave, no per-lane vector-memory instruction at all: the per-lane walk is bound by the
// vector-memory pipe, TA/TD), every lane tests the boxes and triangles against its own ray,
// and a lane leaves as soon as it is occluded.  The answer is the per-lane walk's: any hit is
// order-free, an accepted triangle is accepted on its own test (Moller-Trumbore, t < max_dist
// and the reference's batch gate, exactly as bvh_leaf), and the union of the lanes' walks
// contains every lane's own walk (the boxes are conservative), so no occluder is missed.
// The walk order follows the first walking lane's entry distances.  Taken only when the
// walking lanes' origins are within TRT_SHADOW_WAVE_EXT of the first one's: always on, the union
// walks cost C4 +11 %, C3 +19 %, the shipped frame +50 %; gated at 0.1 scene units, C4 -3.6 %,
// the others within noise (0.02 / 0.07 / 0.15 / 0.25 / 0.5 measured, profiles/r03_ab_shadow_wave_*).
// Shadow rays are 59 % of C4's frame (profiles/r03_ab_noshadow_c4.log).  The stack is wave-uniform
// and lives in the wave's BVH-stack LDS (no traversal of this wave is live during a shadow
// query): one lane writes an entry, every lane reads it back as a broadcast.
#ifndef TRT_SHADOW_WAVE
#define TRT_SHADOW_WAVE 1
#endif
#ifndef TRT_SHADOW_WAVE_EXT
#define TRT_SHADOW_WAVE_EXT 0.1
#endif
constexpr int kShadowWaveStack = 128; // >= kBvhStack
__device__ __forceinline__ bool shadow_wave_q(const KArgs& A, f3 o, f3 d, f3 inv, float max_dist, float4* slab) {
    typedef __attribute__((address_space(4))) const float cfloat;
    typedef __attribute__((address_space(4))) const uint32_t cuint;
    lds_u32* ws = (lds_u32*)reinterpret_cast<uint32_t*>(slab);
    uint32_t sp = 0u, node = 0u;
    for (;;) {
        if (!(node & kBvhLeafBit)) {
            const cfloat* R = (const cfloat*)(A.bvh4q + node);
            const cuint* RC = (const cuint*)(A.bvh4q + node);
            const uint32_t ex = RC[3];
            const float sx = __uint_as_float((ex & 0xffu) << 23);
            const float sy = __uint_as_float(((ex >> 8) & 0xffu) << 23);
            const float sz = __uint_as_float(((ex >> 16) & 0xffu) << 23);
            const float ax = (R[0] - o.x) * inv.x, bx = sx * inv.x;
            const float ay = (R[1] - o.y) * inv.y, by = sy * inv.y;
            const float az = (R[2] - o.z) * inv.z, bz = sz * inv.z;
            const uint32_t qlx = RC[4], qly = RC[5], qlz = RC[6], qhx = RC[7], qhy = RC[8], qhz = RC[9];
            const uint32_t nx = inv.x >= 0.0f ? qlx : qhx, fx = inv.x >= 0.0f ? qhx : qlx;
            const uint32_t ny = inv.y >= 0.0f ? qly : qhy, fy = inv.y >= 0.0f ? qhy : qly;
            const uint32_t nz = inv.z >= 0.0f ? qlz : qhz, fz = inv.z >= 0.0f ? qhz : qlz;
            float key[4];
            uint32_t r[4] = {RC[12], RC[13], RC[14], RC[15]};
            uint32_t nh = 0u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int sh = 8 * i;
                const float tnx = __builtin_fmaf((float)((nx >> sh) & 0xffu), bx, ax);
                const float tny = __builtin_fmaf((float)((ny >> sh) & 0xffu), by, ay);
                const float tnz = __builtin_fmaf((float)((nz >> sh) & 0xffu), bz, az);
                const float tfx = __builtin_fmaf((float)((fx >> sh) & 0xffu), bx, ax);
                const float tfy = __builtin_fmaf((float)((fy >> sh) & 0xffu), by, ay);
                const float tfz = __builtin_fmaf((float)((fz >> sh) & 0xffu), bz, az);
                const float tn = fmaxf(fmaxf(tnx, tny), tnz);
                const float tf = fminf(fminf(tfx, tfy), tfz);
                const bool ok = tn <= tf && tf > TRT_EPS && tn <= max_dist;
                const bool any = __ballot(ok) != 0ull;
                // an entered child's key is finite (a NaN or infinite entry distance of that lane
                // becomes 3e38), so entered children sort strictly before the missed ones (+inf)
                const float k0 = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(tn)));
                key[i] = any ? (k0 < 3.0e38f ? k0 : 3.0e38f) : __builtin_huge_valf();
                nh += any ? 1u : 0u;
            }
            if (nh != 0u) {
                // entered children nearest first (by the first walking lane's entry distance)
#define TRT_CSWAP(a, b)                                   \
    do {                                                  \
        const bool sw = key[b] < key[a];                  \
        const float ta = key[a], tb = key[b];             \
        const uint32_t ra = r[a], rb = r[b];              \
        key[a] = sw ? tb : ta;                            \
        key[b] = sw ? ta : tb;                            \
        r[a] = sw ? rb : ra;                              \
        r[b] = sw ? ra : rb;                              \
    } while (0)
                TRT_CSWAP(0, 1);
                TRT_CSWAP(2, 3);
                TRT_CSWAP(0, 2);
                TRT_CSWAP(1, 3);
                TRT_CSWAP(1, 2);
#undef TRT_CSWAP
#pragma unroll
                for (int k = 3; k >= 1; --k)
                    if ((uint32_t)k < nh) {
                        const uint32_t v = __builtin_amdgcn_readfirstlane(r[k]);
                        if (lane_id() == __builtin_amdgcn_readfirstlane(lane_id())) ws[sp] = v;
                        ++sp;
                    }
                node = __builtin_amdgcn_readfirstlane(r[0]);
                continue;
            }
        } else {
            const uint32_t first = node & kBvhFirstMask;
            const uint32_t n = ((node >> kBvhCountShift) & 15u) + 1u;
            for (uint32_t k = first; k < first + n; ++k)
                if (shadow_tri_s(A, k, o, d, max_dist)) return true; // bvh_leaf's test, term for term
        }
        if (sp == 0u) return false;
        --sp;
        node = __builtin_amdgcn_readfirstlane(ws[sp]);
    }
}

template <bool COUNT, int GEOM>
__device__ __forceinline__ void scene_intersect(const KArgs& A, f3 o, f3 d, Hit& h, Cnt& c, float4* slab) {
    h.t = 1e10f;
    h.kind = HIT_NONE;
    h.idx = 0;
    h.u = 0.0f;
    h.v = 0.0f;
    h.ni = 0;
    h.batch = 0;
    if (A.flags & TRT_FLAG_FLOOR) { // shader.comp:302-320
        if (fabsf(d.y) > TRT_EPS) {
            float t = div_rn(-(o.y + 4.0f), d.y);
            if (t > TRT_EPS && t < h.t) {
                f3 p = add(o, muls(d, t));
                if (fabsf(p.x) < 10.0f && p.z < -5.0f && p.z > -30.0f) {
                    h.t = t;
                    h.kind = HIT_FLOOR;
                }
            }
        }
    }
    if (A.flags & TRT_FLAG_SPHERES) { // shader.comp:322-335
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float t = 1e10f;
            if (COUNT) ++c.sph;
            const bool hit = sphere_hit(o, d, A.sph[i], t);
            if (hit && t < h.t) {
                h.t = t;
                h.kind = HIT_SPHERE;
                h.idx = i;
            }
        }
    }
    if (GEOM == 0 || A.nbatch == 0) return;
    if (GEOM >= 2 && ray_misses_all_batches(o, d)) return;
    f3 inv = GEOM >= 2 ? cull_inv(d) : mk(rcp_rn_lane(d.x), rcp_rn_lane(d.y), rcp_rn_lane(d.z)); // shader.comp:336
    bool unused = false;
    if (GEOM >= 2) {
        if (g3_quant_only<GEOM>() || (TRT_BVH_WIDTH == 4 && A.bvh4)) trace_bvh4<COUNT, false, GEOM>(A, o, d, inv, h, unused, 0.0f, c, slab);
        else trace_bvh<COUNT, false, GEOM>(A, o, d, inv, h, unused, 0.0f, c, slab);
    }
    else walk_batches<COUNT, false>(A, o, d, inv, h, unused, 0.0f, c, slab);
}

// shadow_intersect, shader.comp:364-399: any hit on spheres / triangles; floor excluded.
template <bool COUNT, int GEOM>
__device__ __forceinline__ bool shadow_intersect(const KArgs& A, f3 o, f3 d, float max_dist, Cnt& c,
                                                 float4* slab) {
#ifdef TRT_DIAG_NO_SHADOW
    return false; // diagnostic build only: prices the shadow rays
#endif
#ifdef TRT_DIAG_DUMP_SHADOW
    if (A.diag) { // diagnostic build only: appends the query to A.diag (counters[31]) untraced
        const uint64_t act = __ballot(true);
        const int leader = __ffsll((unsigned long long)act) - 1;
        unsigned long long base = 0;
        if ((int)lane_id() == leader) base = atomicAdd(&A.counters[31], (unsigned long long)__popcll(act));
        base = __shfl(base, leader, 64);
        float4* r = A.diag + 2 * (base + lane_rank(act));
        r[0] = make_float4(o.x, o.y, o.z, max_dist);
        r[1] = make_float4(d.x, d.y, d.z, 0.0f);
        return false;
    }
#endif
    if (A.flags & TRT_FLAG_SPHERES) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float t = 1e10f;
            if (COUNT) ++c.sph;
            if (sphere_hit(o, d, A.sph[i], t) && t < max_dist) return true;
        }
    }
    if (GEOM == 0 || A.nbatch == 0) return false;
    if (GEOM >= 2 && ray_misses_all_batches(o, d)) return false;
    f3 inv = GEOM >= 2 ? cull_inv(d) : mk(rcp_rn_lane(d.x), rcp_rn_lane(d.y), rcp_rn_lane(d.z)); // shader.comp:377
    bool occluded = false;
    Hit unused;
    if (GEOM >= 2) {
#if TRT_SHADOW_WAVE && TRT_BVH_QUANT
        if constexpr (!COUNT && GEOM == 3 && TRT_BVH_WIDTH == 4 && slab_words<GEOM>() >= kShadowWaveStack)
            if (A.bvh4q) {
                // only when the walking lanes' origins lie within TRT_SHADOW_WAVE_EXT of the
                // first one's (L-inf): scattered origins make the union of the walks far longer
                // than any one of them
                const float fx = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(o.x)));
                const float fy = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(o.y)));
                const float fz = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(o.z)));
                const float e = fmaxf(fmaxf(fabsf(o.x - fx), fabsf(o.y - fy)), fabsf(o.z - fz));
                const bool near = e <= (float)TRT_SHADOW_WAVE_EXT;
                const uint64_t nm = __ballot(near);
                if (nm == __ballot(true)) return shadow_wave_q(A, o, d, inv, max_dist, slab);
            }
#endif
        if (g3_quant_only<GEOM>() || (TRT_BVH_WIDTH == 4 && A.bvh4)) trace_bvh4<COUNT, true, GEOM>(A, o, d, inv, unused, occluded, max_dist, c, slab);
        else trace_bvh<COUNT, true, GEOM>(A, o, d, inv, unused, occluded, max_dist, c, slab);
    }
    else walk_batches<COUNT, true>(A, o, d, inv, unused, occluded, max_dist, c, slab);
    return occluded;
}

// ---- background (direction_to_uv + texture(), shader.comp:410-416, 455-458) --------------

// UNORM8 -> float, c / 255 correctly rounded (the oracle's `(float)c / 255.0f`), as
// q = c * RN(1/255) plus one FMA remainder correction: bit-identical to the IEEE quotient for
// every c in [0, 255] (exhaustive exact-rational check: tests/test_envmap_math.py), 3 VALU ops
// instead of the 11-instruction correctly-rounded division sequence (12 per envmap sample).
__device__ __forceinline__ float unorm8(uint32_t c) {
    const float x = (float)c, r = 1.0f / 255.0f;
    const float q = x * r;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, x), r, q);
}

#ifndef TRT_ENV_PAIRROWS
#define TRT_ENV_PAIRROWS 1
#endif
#ifndef TRT_ENV_PAIRS
#define TRT_ENV_PAIRS 1
#endif
// The four texels of a bilinear footprint and its weights: the gather is issued here and
// consumed by env_blend, so a caller can place independent work between the two.
struct EnvFetch {
    uint32_t c00, c10, c01, c11;
    float a, b;
};

__device__ __forceinline__ EnvFetch env_fetch(const KArgs& A, f3 d) {
#ifdef TRT_DIAG_NO_ENV_FETCH
    {   // diagnostic: uv math without the texel gathers
        float u = (atan2f(d.z, d.x) + TRT_PI) / (2.0f * TRT_PI), v = acosf(fminf(fmaxf(d.y, -1.0f), 1.0f)) / TRT_PI;
        return EnvFetch{0u, 0xffu, 0xff00u, 0xff0000u, u, v};
    }
#endif
#ifdef TRT_DIAG_NO_UV_TRIG
    // diagnostic: prices atan2 / acos (wrong texels): C2 13.85 -> 13.23 us per frame; SLEEF-style
    // minimax polynomials in their place measured 13.95 (profiles/r04c_ab_c2_stages.jsonl), so
    // ocml's stay
    float theta = d.z * 3.0f, phi = (d.y + 1.0f) * 1.5f;
#else
    float theta = atan2f(d.z, d.x);
    float phi = acosf(fminf(fmaxf(d.y, -1.0f), 1.0f));
#endif
    // direction_to_uv, shader.comp:410-416.  atan/acos are already ocml's (within a few ulp
    // of the oracle's libm, tests/helpers.py FLOAT_TOL), so the two divisions by constants
    // are products with the rounded reciprocals (<= 1 ulp apart from the quotients).
    float u = (theta + TRT_PI) * (1.0f / (2.0f * TRT_PI));
    float v = phi * (1.0f / TRT_PI);
    // Sampler: LINEAR, CLAMP_TO_EDGE, level 0 (main.cpp:1091-1106), R8G8B8A8_UNORM.
    const int W = (int)A.env_w, H = (int)A.env_h;
    float x = u * (float)W - 0.5f, y = v * (float)H - 0.5f;
    if (!(x == x)) x = 0.0f;
    if (!(y == y)) y = 0.0f;
    float xf = floorf(x), yf = floorf(y);
    float a = x - xf, b = y - yf;
    // clamp in float first so the int conversion is always in range
    int ix0 = (int)fminf(fmaxf(xf, -1.0f), (float)W);
    int iy0 = (int)fminf(fmaxf(yf, -1.0f), (float)H);
    int ix1 = min(max(ix0 + 1, 0), W - 1);
    int iy1 = min(max(iy0 + 1, 0), H - 1);
    ix0 = min(max(ix0, 0), W - 1);
    iy0 = min(max(iy0, 0), H - 1);
    EnvFetch e;
#if TRT_ENV_PAIRROWS
    if (A.envp) {
        // ix0 - ix1 and iy0 - iy1 as below: column xf + 1 and row yf + 1 of the pair rows
        const int c = (int)fminf(fmaxf(xf, -1.0f), (float)W) + 1;
        const int r = (int)fminf(fmaxf(yf, -1.0f), (float)H) + 1;
        uint4 q;
        __builtin_memcpy(&q, A.envp + ((uint32_t)r * (uint32_t)(W + 3) + (uint32_t)c), sizeof(q));
        e.c00 = q.x;
        e.c01 = q.y;
        e.c10 = q.z;
        e.c11 = q.w;
        e.a = a;
        e.b = b;
        return e;
    }
#endif
#if TRT_ENV_PAIRS
    if (W >= 2) {
        // Each row's two texels in one 8-byte load at base = min(ix0, W - 2): the footprint is
        // (base, base + 1) except at the clamped edges, where ix0 / ix1 pick within the pair.
        const int base = min(ix0, W - 2);
        const uint2 p0 = *reinterpret_cast<const uint2*>(A.env + ((uint32_t)iy0 * (uint32_t)W + (uint32_t)base));
        const uint2 p1 = *reinterpret_cast<const uint2*>(A.env + ((uint32_t)iy1 * (uint32_t)W + (uint32_t)base));
        e.c00 = ix0 == base ? p0.x : p0.y;
        e.c10 = ix1 == base ? p0.x : p0.y;
        e.c01 = ix0 == base ? p1.x : p1.y;
        e.c11 = ix1 == base ? p1.x : p1.y;
    } else
#endif
    {
        const uint32_t* row0 = A.env + (size_t)iy0 * (size_t)W;
        const uint32_t* row1 = A.env + (size_t)iy1 * (size_t)W;
        e.c00 = row0[ix0];
        e.c10 = row0[ix1];
        e.c01 = row1[ix0];
        e.c11 = row1[ix1];
    }
    e.a = a;
    e.b = b;
    return e;
}

// Bilinear blend of a fetched footprint (the second half of `background`).
__device__ __forceinline__ f3 env_blend(const EnvFetch& e) {
    const float a = e.a, b = e.b;
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b);
    float w01 = (1.0f - a) * b, w11 = a * b;
    float r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int sh = 8 * k;
        float t00 = unorm8((e.c00 >> sh) & 255u), t10 = unorm8((e.c10 >> sh) & 255u);
        float t01 = unorm8((e.c01 >> sh) & 255u), t11 = unorm8((e.c11 >> sh) & 255u);
        r[k] = ((w00 * t00 + w10 * t10) + w01 * t01) + w11 * t11;
    }
    return mk(r[0], r[1], r[2]);
}

__device__ __forceinline__ f3 background(const KArgs& A, f3 d) {
    if (!(A.flags & TRT_FLAG_ENVMAP)) return mk(0.2f, 0.7f, 0.8f); // BACKGROUND_COLOR :77
    return env_blend(env_fetch(A, d));
}

// ---- cast_ray (shader.comp:423-583) --------------------------------------------------------

struct Seg {
    f3 o, d;
    float thr; // throughput is (s,s,s): vec3(1) times scalar albedo weights
    int depth;
};

// LIFO of deferred refraction children.  A workgroup is one wave, so for CAP <= 4 the
// stack lives in LDS laid out [entry][field][lane]: every push/pop is 8 lane-contiguous
// ds_write_b32/ds_read_b32 (conflict-free), and no VGPRs hold waiting segments.  Deeper
// trees (max_depth > 5) use a private array (LDS is kept for 16 resident waves per CU).
// Split launches (trace in depth windows) use a hybrid: the window's entries in LDS and a
// private tail that only a child traced in place after a full task queue can reach.
constexpr int LDS_STACK_MAX = 4;
// TRT_G3_SEG_PRIV: the per-pixel loop of GEOM 3 kernels (not split) keeps its deferred children
// in a private array, and the LDS goes to the BVH traversal stack (TRT_G3_LDS entries): a
// child is pushed once per glass hit, a traversal entry several times per ray.
#ifndef TRT_G3_SEG_PRIV
#define TRT_G3_SEG_PRIV 1
#endif
template <int CAP, int GEOM = 0, bool HYB = false>
constexpr bool seg_lds() { return CAP >= 1 && CAP <= LDS_STACK_MAX && (HYB || !(GEOM == 3 && TRT_G3_SEG_PRIV)); }
template <int CAP, int GEOM = 0, bool HYB = false>
constexpr int lds_stack_floats_() { return seg_lds<CAP, GEOM, HYB>() ? CAP * 8 * 64 : 1; }
template <int CAP, int GEOM = 0, bool HYB = false>
constexpr int lds_stack_floats() { return lds_stack_floats_<CAP, GEOM, HYB>(); }

template <int CAP, bool LDS = (CAP <= LDS_STACK_MAX)>
struct DeferStack;

__device__ __forceinline__ void lds_put(lds_f32* p, const Seg& x) {
    p[0] = x.o.x;
    p[64] = x.o.y;
    p[128] = x.o.z;
    p[192] = x.d.x;
    p[256] = x.d.y;
    p[320] = x.d.z;
    p[384] = x.thr;
    p[448] = __int_as_float(x.depth);
}
__device__ __forceinline__ Seg lds_get(const lds_f32* p) {
    return Seg{mk(p[0], p[64], p[128]), mk(p[192], p[256], p[320]), p[384], __float_as_int(p[448])};
}

// As BvhStack: the private entries live in the caller's Mem, so `n` stays in a register.
template <int CAP>
struct DeferStack<CAP, true> {
    struct Mem {};
    lds_f32* base; // this lane's column: base[(e * 8 + f) * 64]
    int n = 0;
    __device__ __forceinline__ DeferStack(float* lds, Mem&) : base((lds_f32*)(lds + lane_id())) {}
    __device__ __forceinline__ void push(const Seg& x) {
        lds_put(base + n * 8 * 64, x);
        ++n;
    }
    __device__ __forceinline__ Seg pop() {
        --n;
        return lds_get(base + n * 8 * 64);
    }
};

template <int CAP>
struct DeferStack<CAP, false> {
    struct Mem {
        Seg s[CAP];
    };
    Seg* s;
    int n = 0;
    __device__ __forceinline__ DeferStack(float*, Mem& m) : s(m.s) {}
    __device__ __forceinline__ void push(const Seg& x) { s[n++] = x; }
    __device__ __forceinline__ Seg pop() { return s[--n]; }
};

// CL entries in LDS, then CP private ones.
template <int CL, int CP>
struct HybridStack {
    struct Mem {
        Seg s[CP];
    };
    lds_f32* base;
    Seg* s;
    int n = 0;
    __device__ __forceinline__ HybridStack(float* lds, Mem& m) : base((lds_f32*)(lds + lane_id())), s(m.s) {}
    __device__ __forceinline__ void push(const Seg& x) {
        if (n < CL) lds_put(base + n * 8 * 64, x);
        else s[n - CL] = x;
        ++n;
    }
    __device__ __forceinline__ Seg pop() {
        --n;
        if (n < CL) return lds_get(base + n * 8 * 64);
        return s[n - CL];
    }
};

template <int CAP, bool SPLIT, int GEOM = 0>
struct StackOf {
    using type = DeferStack<CAP, seg_lds<CAP, GEOM>()>;
};
template <int CAP, int GEOM>
struct StackOf<CAP, true, GEOM> {
    using type = HybridStack<CAP, (int)TRT_MAX_DEPTH_LIMIT - 1 - CAP>;
};

// ---- subtree split: task queues ------------------------------------------------------------


// Wave-aggregated append of up to two tasks per lane (one atomic per wave).  A task that does
// not fit the queue is not written and its flag is cleared: the caller traces it in place.
// DEFER: each task also carries its parent link (la / lb: parent event slot << 1 | refraction).
template <bool DEFER = false>
__device__ __forceinline__ void enqueue2(const KArgs& A, bool& sa, const Seg& a, bool& sb, const Seg& b,
                                         uint32_t pixel, uint32_t la = 0, uint32_t lb = 0) {
    const uint64_t ba = __ballot(sa), bb = __ballot(sb);
    if ((ba | bb) == 0ull) return;
    const uint32_t na = (uint32_t)__popcll(ba), nb = (uint32_t)__popcll(bb);
    const uint64_t act = __ballot(true);
    const int leader = __ffsll((unsigned long long)act) - 1;
    uint32_t base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(A.q_out_n, na + nb);
    base = __shfl(base, leader, 64);
    const uint32_t ia = base + lane_rank(ba), ib = base + na + lane_rank(bb);
    auto put = [&](bool& f, uint32_t i, const Seg& x, uint32_t link) {
        if (!f) return;
        if (i >= A.q_cap) {
            f = false;
            atomicAdd(&A.ctr->overflow, 1u);
            return;
        }
        float4* q = reinterpret_cast<float4*>(A.q_out + i);
        q[0] = make_float4(x.o.x, x.o.y, x.o.z, x.d.x);
        q[1] = make_float4(x.d.y, x.d.z, x.thr, __uint_as_float((pixel << kTaskDepthBits) | (uint32_t)x.depth));
        if (DEFER) A.q_link_out[i] = link;
    };
    put(sa, ia, a, la);
    put(sb, ib, b, lb);
}

// Colours of split pixels are summed in 32.32 fixed point (integer adds: the same result in
// any order); finalize_spilled converts back.
__device__ __forceinline__ unsigned long long to_fixed(float v) {
    return (unsigned long long)(long long)((double)v * 4294967296.0);
}
__device__ __forceinline__ float from_fixed(unsigned long long v) {
    return (float)((double)(long long)v * (1.0 / 4294967296.0));
}

// ---- deferred shadows: the per-lane event pool (trt_device.h kEvRows) --------------------
// One frame's deferred scratch (a deferred launch traces A.dframes frames, each with its own
// event pool, query queue, per-pixel roots, fallback list and counters: frame f's are the bases
// in KArgs plus f times the per-frame strides).  Wave-uniform.
struct DScratch {
    float4* ev;
    float4* shq;
    uint2* px_ev;
    uint32_t* fb;
    DeferCtr* dctr;
};
__device__ __forceinline__ DScratch dscratch(const KArgs& A, uint32_t f) {
    return DScratch{A.ev + f * A.ev_fstride, A.shq + f * A.shq_fstride, A.px_ev + (size_t)f * A.px_fstride,
                    A.fb + (size_t)f * A.px_fstride, A.dctr + f};
}
struct EvLog {
    DScratch S;          // the frame's scratch
    uint32_t stripe = 0; // the stripe of the event pool and query queue (wave-uniform)
    uint32_t k = 0;      // events this lane has logged
    uint32_t chunk = 0;  // the chunk holding event k - 1
    bool ovf = false;    // event pool or query queue full: the lane's pixels go to defer_fallback
};

// Slot of this lane's next event; pass A calls it on every lane once per step of the wave.
// Lanes that start a chunk together share one (each lane owns its column of a chunk; one
// wave-aggregated atomic).  A slot only names where the event lives: the tree links (plane 3)
// give the order, so chunks are not chained.
__device__ __forceinline__ uint32_t ev_alloc(const KArgs& A, EvLog& L) {
    const uint32_t row = L.k % kEvRows;
    const bool need = row == 0u && !L.ovf;
    const uint64_t m = __ballot(need);
    if (m) {
        const int leader = __ffsll((unsigned long long)m) - 1;
        uint32_t base = 0;
        if ((int)lane_id() == leader) base = atomicAdd(&L.S.dctr->chunks[L.stripe * kCtrStride], 1u);
        base = __shfl(base, leader, 64);
        if (need) {
            if (base >= A.ev_cap) L.ovf = true;
            else L.chunk = base + L.stripe * A.ev_cap;
        }
    }
    ++L.k;
    return (L.chunk * kEvRows + row) * 64u + lane_id();
}
// Plane p (0..3) of event slot s = (chunk * kEvRows + row) * 64 + lane.
__device__ __forceinline__ float4* ev_plane(float4* ev, uint32_t s, uint32_t p) {
    return ev + ((size_t)(s >> 6) * 4u + p) * 64u + (s & 63u);
}

// The closest hit's shading inputs (shader.comp:302-360): point, normal, material.
struct Surf {
    f3 p, n;
    float alb[4], kd[3], sexp, ior;
};

template <bool COUNT>
__device__ __forceinline__ Surf resolve_hit(const KArgs& A, const Seg& cur, const Hit& h, Cnt& cnt) {
    Surf s;
    s.p = add(cur.o, muls(cur.d, h.t));
    if (h.kind == HIT_FLOOR) {
        s.n = mk(0.0f, 1.0f, 0.0f);
        float c0 = 0.3f, c1 = 0.3f, c2 = 0.3f;
        if (A.flags & TRT_FLAG_CHECKER) { // shader.comp:312
            float m = floorf(s.p.x * 0.5f + 1024.0f) + floorf(s.p.z * 0.5f);
            float mod2 = m - 2.0f * floorf(m / 2.0f);
            if (!(mod2 == 0.0f)) {
                c1 = 0.2f;
                c2 = 0.1f;
            }
        }
        s.alb[0] = 2.0f; s.alb[1] = 0.0f; s.alb[2] = 0.0f; s.alb[3] = 0.0f;
        s.kd[0] = c0; s.kd[1] = c1; s.kd[2] = c2;
        s.sexp = 1.0f;
        s.ior = 1.0f;
    } else if (h.kind == HIT_SPHERE) {
        const SphereArg& sp = A.sph[h.idx];
        s.n = normalize3(sub(s.p, mk(sp.c[0], sp.c[1], sp.c[2])));
#pragma unroll
        for (int k = 0; k < 4; ++k) s.alb[k] = sp.m.albedo[k];
        s.kd[0] = sp.m.kd[0]; s.kd[1] = sp.m.kd[1]; s.kd[2] = sp.m.kd[2];
        s.sexp = sp.m.spec_exp;
        s.ior = sp.m.ior;
    } else {
        if (COUNT) ++cnt.trin;
        const TriShade& ts = A.shade[h.idx];
        if (h.ni == 0) {
            const TriGeo& g = A.geo[h.idx];
            s.n = normalize3(cross3(ld3(g.e1), ld3(g.e2)));
        } else {
            float w = 1.0f - h.u - h.v;
            f3 nn = add(add(muls(ld3(ts.n0), w), muls(ld3(ts.n1), h.u)), muls(ld3(ts.n2), h.v));
            s.n = normalize3(nn);
        }
        const Mat& m = A.mats[ts.material];
#pragma unroll
        for (int k = 0; k < 4; ++k) s.alb[k] = m.albedo[k];
        s.kd[0] = m.kd[0]; s.kd[1] = m.kd[1]; s.kd[2] = m.kd[2];
        s.sexp = m.spec_exp;
        s.ior = m.ior;
    }
    return s;
}

// One light of the Phong loop (shader.comp:491-505): direction, distance, shadow origin and the
// diffuse / specular terms; `matters`: a light whose two terms both vanish from the colour (a
// zero term, or a zero albedo weight: diffuse * 0 = 0 for any finite diffuse) adds exactly
// nothing lit or shadowed, so its shadow query cannot change the pixel and a frame does not
// trace it.  The counting pass keeps the reference's behaviour (traces it and adds the terms
// when lit: its counters and image are the reference's, and tests/test_gpu_parity.py checks
// that its image equals the frame's bit for bit) and reports the skipped queries and their work.
struct LightTerm {
    f3 ld, so;
    float dist, diff, spec;
    bool matters;
};

__device__ __forceinline__ LightTerm light_term(const KArgs& A, const Surf& s, f3 v, int i) {
    LightTerm t;
    f3 L = mk(A.light[i][0], A.light[i][1], A.light[i][2]);
    t.ld = normalize_len3(sub(L, s.p), t.dist);
    t.so = dot3(t.ld, s.n) < 0.0f ? sub(s.p, muls(s.n, TRT_EPS)) : add(s.p, muls(s.n, TRT_EPS));
    t.diff = 1.0f * fmaxf(0.0f, dot3(s.n, t.ld));
    t.spec = 0.0f; // not formed under a zero specular weight (cast_seg)
    if (!TRT_SPEC_SKIP || s.alb[1] != 0.0f) {
        const f3 rdir = reflect3(neg(t.ld), s.n);
#ifdef TRT_DIAG_NO_POW
        t.spec = 1.0f * fmaxf(0.0f, dot3(rdir, v)) * s.sexp; // diagnostic: prices powf
#else
        t.spec = 1.0f * pow_pos(fmaxf(0.0f, dot3(rdir, v)), s.sexp);
#endif
    }
    t.matters = TRT_SKIP_DARK == 0 || (s.alb[0] != 0.0f && t.diff != 0.0f) || (s.alb[1] != 0.0f && t.spec != 0.0f);
    return t;
}

// Children (shader.comp:509-575).  Children that the reference would push and then drop unseen
// at the depth / throughput test (shader.comp:449) are not made (mk_* false).
__device__ __forceinline__ void make_children(const Seg& cur, const Surf& s, int D, Seg& refr, bool& mk_refr,
                                              Seg& refl, bool& mk_refl) {
    const int cd = cur.depth + 1;
    mk_refr = mk_refl = false;
    bool skip_reflect = false;
    if (s.alb[3] > 0.0f) {
        f3 rd = custom_refract(cur.d, s.n, s.ior, 1.0f);
        float rl;
        const f3 rn = normalize_len3(rd, rl);
        if (rl > 0.0001f) {
            rd = rn;
        } else { // total internal reflection: one reflected child, shader.comp:533-555
            rd = normalize3(reflect3(cur.d, s.n));
            skip_reflect = true;
        }
        f3 off = dot3(rd, s.n) < 0.0f ? muls(neg(s.n), TRT_EPS) : muls(s.n, TRT_EPS);
        refr = Seg{add(s.p, off), rd, cur.thr * s.alb[3], cd};
        float tt = (refr.thr * refr.thr + refr.thr * refr.thr) + refr.thr * refr.thr;
        mk_refr = cd < D && !(tt < 0.001f);
    }
    if (s.alb[2] > 0.0f && !skip_reflect) {
        f3 rd = normalize3(reflect3(cur.d, s.n));
        f3 off = dot3(rd, s.n) < 0.0f ? muls(neg(s.n), TRT_EPS) : muls(s.n, TRT_EPS);
        refl = Seg{add(s.p, off), rd, cur.thr * s.alb[2], cd};
        float tt = (refl.thr * refl.thr + refl.thr * refl.thr) + refl.thr * refl.thr;
        mk_refl = cd < D && !(tt < 0.001f);
    }
}

// TRT_LATE_MAT (mesh kernels, GEOM >= 2, per-pixel loop): the light loop runs in three phases
// -- the three lights' diffuse / specular terms, then the shadow walks, then the lit terms summed
// in light order -- and the material (albedo weights, kd, index of refraction) is fetched again
// after the walks instead of being held across them.  Across a walk the lane keeps the hit
// point, normal, direction, colour, throughput, depth, the hit's kind and index and the six
// terms, not the eleven material floats the 96-VGPR build spilled to scratch.  Same operations
// in the same order: bit-identical.
#ifndef TRT_LATE_MAT
#define TRT_LATE_MAT 1
#endif
struct MatVals {
    float alb[4], kd[3], sexp, ior;
};
__device__ __forceinline__ MatVals load_mat(const KArgs& A, int kind, int idx, f3 p) {
    MatVals m;
    if (kind == HIT_FLOOR) {
        float c0 = 0.3f, c1 = 0.3f, c2 = 0.3f;
        if (A.flags & TRT_FLAG_CHECKER) { // shader.comp:312
            float q = floorf(p.x * 0.5f + 1024.0f) + floorf(p.z * 0.5f);
            float mod2 = q - 2.0f * floorf(q / 2.0f);
            if (!(mod2 == 0.0f)) {
                c1 = 0.2f;
                c2 = 0.1f;
            }
        }
        m.alb[0] = 2.0f; m.alb[1] = 0.0f; m.alb[2] = 0.0f; m.alb[3] = 0.0f;
        m.kd[0] = c0; m.kd[1] = c1; m.kd[2] = c2;
        m.sexp = 1.0f;
        m.ior = 1.0f;
    } else if (kind == HIT_SPHERE) {
        const Mat& mm = A.sph[idx].m;
#pragma unroll
        for (int k = 0; k < 4; ++k) m.alb[k] = mm.albedo[k];
        m.kd[0] = mm.kd[0]; m.kd[1] = mm.kd[1]; m.kd[2] = mm.kd[2];
        m.sexp = mm.spec_exp;
        m.ior = mm.ior;
    } else {
        const Mat& mm = A.mats[A.shade[idx].material];
#pragma unroll
        for (int k = 0; k < 4; ++k) m.alb[k] = mm.albedo[k];
        m.kd[0] = mm.kd[0]; m.kd[1] = mm.kd[1]; m.kd[2] = mm.kd[2];
        m.sexp = mm.spec_exp;
        m.ior = mm.ior;
    }
    return m;
}

// The DFS of one segment tree (root = a primary ray, or a task of a split launch).  Returns
// the unclamped colour sum in the reference's pop order.  SPLIT: children at depth
// >= A.split_d1 are handed to the task queue (`spilled` is set) instead of being traced.
// HYB: the deferred refraction children live in CAP LDS entries plus a private tail.  (The
// shading here is written out rather than through resolve_hit / light_term / make_children:
// the factored form compiles the C2 and C4 kernels with more live registers — C2 spilled.)
template <int CAP, bool COUNT, int GEOM, bool SPLIT, bool HYB = SPLIT>
__device__ __forceinline__ f3 cast_seg(const KArgs& A, Seg cur, Cnt& cnt, float* lds, float4* slab,
                                       uint32_t pixel, bool& spilled) {
    const int D = (int)A.max_depth;
    f3 color = mk(0.0f, 0.0f, 0.0f);
    using Stk = typename StackOf<CAP, HYB, GEOM>::type;
    typename Stk::Mem stk_mem;
    Stk stk(lds, stk_mem);
    for (;;) {
        if (COUNT && cur.depth > 0) ++cnt.sec;
#ifdef TRT_DIAG_PIXEL_WORK
        ++cnt.wseg;
#endif
        Hit h;
        scene_intersect<COUNT, GEOM>(A, cur.o, cur.d, h, cnt, slab);
        bool have_next = false;
        Seg next;
        if (h.kind == HIT_NONE) {
            if (COUNT) ++cnt.miss;
            f3 bg = background(A, cur.d);
            color = add(color, muls(bg, cur.thr));
        } else {
            // Resolve the closest hit: point, normal, material (shader.comp:302-360).
            f3 p = add(cur.o, muls(cur.d, h.t));
            f3 n;
            float alb[4], kd[3], sexp, ior;
            if (h.kind == HIT_FLOOR) {
                n = mk(0.0f, 1.0f, 0.0f);
                float c0 = 0.3f, c1 = 0.3f, c2 = 0.3f;
                if (A.flags & TRT_FLAG_CHECKER) { // shader.comp:312
                    float m = floorf(p.x * 0.5f + 1024.0f) + floorf(p.z * 0.5f);
                    float mod2 = m - 2.0f * floorf(m / 2.0f);
                    if (!(mod2 == 0.0f)) {
                        c1 = 0.2f;
                        c2 = 0.1f;
                    }
                }
                alb[0] = 2.0f; alb[1] = 0.0f; alb[2] = 0.0f; alb[3] = 0.0f;
                kd[0] = c0; kd[1] = c1; kd[2] = c2;
                sexp = 1.0f;
                ior = 1.0f;
            } else if (h.kind == HIT_SPHERE) {
                const SphereArg& s = A.sph[h.idx];
                n = normalize3(sub(p, mk(s.c[0], s.c[1], s.c[2])));
#pragma unroll
                for (int k = 0; k < 4; ++k) alb[k] = s.m.albedo[k];
                kd[0] = s.m.kd[0]; kd[1] = s.m.kd[1]; kd[2] = s.m.kd[2];
                sexp = s.m.spec_exp;
                ior = s.m.ior;
            } else {
                if (COUNT) ++cnt.trin;
                const TriShade& ts = A.shade[h.idx];
                if (h.ni == 0) {
                    const TriGeo& g = A.geo[h.idx];
                    n = normalize3(cross3(ld3(g.e1), ld3(g.e2)));
                } else {
                    float w = 1.0f - h.u - h.v;
                    f3 nn = add(add(muls(ld3(ts.n0), w), muls(ld3(ts.n1), h.u)), muls(ld3(ts.n2), h.v));
                    n = normalize3(nn);
                }
                const Mat& m = A.mats[ts.material];
#pragma unroll
                for (int k = 0; k < 4; ++k) alb[k] = m.albedo[k];
                kd[0] = m.kd[0]; kd[1] = m.kd[1]; kd[2] = m.kd[2];
                sexp = m.spec_exp;
                ior = m.ior;
            }
            // Phong with three shadow rays, shader.comp:483-507.
            f3 v = neg(cur.d);
            f3 diffuse = mk(0.0f, 0.0f, 0.0f), specular = mk(0.0f, 0.0f, 0.0f);
            constexpr bool LATE = GEOM >= 2 && TRT_LATE_MAT && !HYB;
            if constexpr (LATE) {
                // Phase 1: the three lights' terms (light_term's arithmetic), before any walk.
                float dif[3], spc[3];
                uint32_t need = 0u;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    f3 L = mk(A.light[i][0], A.light[i][1], A.light[i][2]);
                    float dist;
                    f3 ld = normalize_len3(sub(L, p), dist);
                    dif[i] = 1.0f * fmaxf(0.0f, dot3(n, ld));
                    spc[i] = 0.0f;
                    if (!TRT_SPEC_SKIP || alb[1] != 0.0f) {
                        const f3 rdir = reflect3(neg(ld), n);
#ifdef TRT_DIAG_NO_POW
                        spc[i] = 1.0f * fmaxf(0.0f, dot3(rdir, v)) * sexp;
#else
                        spc[i] = 1.0f * pow_pos(fmaxf(0.0f, dot3(rdir, v)), sexp);
#endif
                    }
                    const bool matters = TRT_SKIP_DARK == 0 || (alb[0] != 0.0f && dif[i] != 0.0f) ||
                                         (alb[1] != 0.0f && spc[i] != 0.0f);
                    need |= (matters ? 1u : 0u) << i;
                }
                // Phase 2: the shadow walks (the loop stays rolled: one inlined walk).
                uint32_t lit = 0u;
                for (int i = 0; i < 3; ++i) {
                    if (COUNT) ++cnt.sh;
                    const bool matters = (need >> i) & 1u;
                    if (!COUNT && !matters) continue;
                    f3 L = mk(A.light[i][0], A.light[i][1], A.light[i][2]);
                    float dist;
                    f3 ld = normalize_len3(sub(L, p), dist);
                    f3 so = dot3(ld, n) < 0.0f ? sub(p, muls(n, TRT_EPS)) : add(p, muls(n, TRT_EPS));
                    const Cnt before = cnt;
                    const bool occl = shadow_intersect<COUNT, GEOM>(A, so, ld, dist, cnt, slab);
                    if (COUNT && !matters) {
                        ++cnt.sk;
                        cnt.ssph += cnt.sph - before.sph;
                        cnt.sbox += (cnt.nt + cnt.bt) - (before.nt + before.bt);
                        cnt.stt += cnt.tt - before.tt;
                        cnt.sta += cnt.ta - before.ta;
                        cnt.stu += cnt.tu - before.tu;
                        cnt.stv += cnt.tv - before.tv;
                    }
                    if (!occl) lit |= 1u << i;
                }
                // Phase 3: the material again (an opaque index: not the pre-walk registers).
                int hk = h.kind, hi = h.idx;
                asm volatile("" : "+v"(hk), "+v"(hi));
                const MatVals mv = load_mat(A, hk, hi, p);
                const f3 kdv2 = mk(mv.kd[0], mv.kd[1], mv.kd[2]);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (!((lit >> i) & 1u)) continue;
                    diffuse = add(diffuse, muls(kdv2, dif[i]));
                    specular = add(specular, muls(kdv2, spc[i]));
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) alb[k] = mv.alb[k];
                ior = mv.ior;
            }
            if constexpr (!LATE) {
            f3 kdv = mk(kd[0], kd[1], kd[2]);
            // Mesh kernels (GEOM >= 2) keep the light loop rolled: unrolled, each of the three
            // lights inlines its own copy of the shadow walks (the wave-coherent one and the
            // per-lane BVH walk), which multiplied the kernel's code past the instruction cache
            // (TRT_LIGHT_UNROLL=1 restores it).
#ifndef TRT_LIGHT_UNROLL
#define TRT_LIGHT_UNROLL 0
#endif
            constexpr int kLightUnroll = GEOM >= 2 && !TRT_LIGHT_UNROLL ? 1 : 3;
#pragma unroll kLightUnroll
            for (int i = 0; i < 3; ++i) {
                f3 L = mk(A.light[i][0], A.light[i][1], A.light[i][2]);
                float dist;
                f3 ld = normalize_len3(sub(L, p), dist);
                f3 so = dot3(ld, n) < 0.0f ? sub(p, muls(n, TRT_EPS)) : add(p, muls(n, TRT_EPS));
                const float diff = 1.0f * fmaxf(0.0f, dot3(n, ld));
                // With a zero specular weight (the floor, the diffuse meshes) the specular sum only
                // ever enters the colour as specular * 0 = 0 (it is finite), so it is not formed.
                float spec = 0.0f;
                if (!TRT_SPEC_SKIP || alb[1] != 0.0f) {
                    const f3 rdir = reflect3(neg(ld), n);
#ifdef TRT_DIAG_NO_POW
                    spec = 1.0f * fmaxf(0.0f, dot3(rdir, v)) * sexp; // diagnostic: prices powf
#else
                    spec = 1.0f * pow_pos(fmaxf(0.0f, dot3(rdir, v)), sexp);
#endif
                }
                // A light whose diffuse term and specular term both vanish from the colour (a
                // zero term, or a zero albedo weight: diffuse * 0 = 0 for any finite diffuse)
                // adds exactly nothing whether it is lit or shadowed, so its shadow query cannot
                // change the pixel and the frame does not trace it.  The counting pass keeps the
                // reference's behaviour (traces it and adds the terms when lit: its counters and
                // image are the reference's, and tests/test_gpu_parity.py checks that its image
                // equals the frame's bit for bit) and reports the skipped queries and their work.
                const bool matters = TRT_SKIP_DARK == 0 || (alb[0] != 0.0f && diff != 0.0f) ||
                                     (alb[1] != 0.0f && spec != 0.0f);
                if (COUNT) ++cnt.sh;
                if (!COUNT && !matters) continue;
                const Cnt before = cnt;
                const bool occl = shadow_intersect<COUNT, GEOM>(A, so, ld, dist, cnt, slab);
                if (COUNT && !matters) {
                    ++cnt.sk;
                    cnt.ssph += cnt.sph - before.sph;
                    cnt.sbox += (cnt.nt + cnt.bt) - (before.nt + before.bt);
                    cnt.stt += cnt.tt - before.tt;
                    cnt.sta += cnt.ta - before.ta;
                    cnt.stu += cnt.tu - before.tu;
                    cnt.stv += cnt.tv - before.tv;
                }
                if (occl) continue;
                diffuse = add(diffuse, muls(kdv, diff));
                specular = add(specular, muls(kdv, spec));
            }
            } // !LATE
            color = add(color, muls(add(muls(diffuse, alb[0]), muls(specular, alb[1])), cur.thr));
            // Children (shader.comp:509-575).  Children that the reference would push and
            // then drop unseen at the depth / throughput test (shader.comp:449) are not made.
            const int cd = cur.depth + 1;
            bool mk_refr = false, mk_refl = false;
            Seg refr, refl;
            bool skip_reflect = false;
            if (alb[3] > 0.0f) {
                f3 rd = custom_refract(cur.d, n, ior, 1.0f);
                float rl;
                const f3 rn = normalize_len3(rd, rl);
                if (rl > 0.0001f) {
                    rd = rn;
                } else { // total internal reflection: one reflected child, shader.comp:533-555
                    rd = normalize3(reflect3(cur.d, n));
                    skip_reflect = true;
                }
                f3 off = dot3(rd, n) < 0.0f ? muls(neg(n), TRT_EPS) : muls(n, TRT_EPS);
                refr = Seg{add(p, off), rd, cur.thr * alb[3], cd};
                float tt = (refr.thr * refr.thr + refr.thr * refr.thr) + refr.thr * refr.thr;
                mk_refr = cd < D && !(tt < 0.001f);
            }
            if (alb[2] > 0.0f && !skip_reflect) {
                f3 rd = normalize3(reflect3(cur.d, n));
                f3 off = dot3(rd, n) < 0.0f ? muls(neg(n), TRT_EPS) : muls(n, TRT_EPS);
                refl = Seg{add(p, off), rd, cur.thr * alb[2], cd};
                float tt = (refl.thr * refl.thr + refl.thr * refl.thr) + refl.thr * refl.thr;
                mk_refl = cd < D && !(tt < 0.001f);
            }
            if (SPLIT && cd >= (int)A.split_d1) { // window edge: both children become tasks
                bool sa = mk_refl, sb = mk_refr;
                enqueue2(A, sa, refl, sb, refr, pixel);
                if (sa) mk_refl = false;
                if (sb) mk_refr = false;
                spilled = spilled || sa || sb;
            }
            // Reference pushes refraction then reflection and pops reflection first.
            if (mk_refl) {
                if (mk_refr) stk.push(refr);
                next = refl;
                have_next = true;
            } else if (mk_refr) {
                next = refr;
                have_next = true;
            }
        }
        if (have_next) {
            cur = next;
        } else if (stk.n > 0) {
            cur = stk.pop();
        } else {
            break;
        }
    }
    return color;
}

// ---- deferred shadows, pass A: the wave's shared segment pool ------------------------------
//
// Pass A traces a tile's segment trees without their shadow rays.  Its segments need no order
// (each event links into its pixel's tree, trt_device.h), so the wave's lanes share their
// pending segments: a lane that has finished its own work takes one from a LIFO pool of pending
// refraction children in LDS (wave-aggregated, one rank per idle lane), and a lane that makes
// two children continues with the reflection child and puts the other into the pool.  A deep
// glass pixel's tree is spread over every lane of its wave instead of keeping one lane busy
// while the others idle (round 3: 19.6 of 64 lanes active in pass A of the shipped frame).
// When the pool is full a child goes to the lane's private overflow stack (<= MAX_DEPTH - 1
// entries: their depths increase from bottom to top).
#ifndef TRT_DEFER_POOL_N
#define TRT_DEFER_POOL_N 128
#endif
constexpr uint32_t kPool = TRT_DEFER_POOL_N;
constexpr int kPoolFields = 10; // o.xyz, d.xyz, thr, depth, parent link, pixel
constexpr int defer_pool_floats() { return (int)kPool * kPoolFields; }

struct PSeg {
    Seg s;
    uint32_t link; // parent event slot << 1 | (1: refraction child), or kEvRoot
    uint32_t pix;  // output pixel
};

// SoA [field][entry]: the lanes of one take / push touch consecutive entries (conflict-free).
__device__ __forceinline__ void pool_put(lds_f32* P, uint32_t e, const PSeg& x) {
    P[0 * kPool + e] = x.s.o.x;
    P[1 * kPool + e] = x.s.o.y;
    P[2 * kPool + e] = x.s.o.z;
    P[3 * kPool + e] = x.s.d.x;
    P[4 * kPool + e] = x.s.d.y;
    P[5 * kPool + e] = x.s.d.z;
    P[6 * kPool + e] = x.s.thr;
    P[7 * kPool + e] = __int_as_float(x.s.depth);
    P[8 * kPool + e] = __uint_as_float(x.link);
    P[9 * kPool + e] = __uint_as_float(x.pix);
}
__device__ __forceinline__ PSeg pool_get(const lds_f32* P, uint32_t e) {
    PSeg x;
    x.s = Seg{mk(P[0 * kPool + e], P[1 * kPool + e], P[2 * kPool + e]),
              mk(P[3 * kPool + e], P[4 * kPool + e], P[5 * kPool + e]), P[6 * kPool + e],
              __float_as_int(P[7 * kPool + e])};
    x.link = __float_as_uint(P[8 * kPool + e]);
    x.pix = __float_as_uint(P[9 * kPool + e]);
    return x;
}

// A pixel whose log does not fit (event pool, query queue or task queue full) is re-traced in
// place by defer_fallback: its tree root becomes kEvNone and it is listed once.
__device__ __forceinline__ void defer_mark_fallback(const DScratch& S, uint32_t pix) {
    if (atomicExch(&S.px_ev[pix].x, kEvNone) != kEvNone) S.fb[atomicAdd(&S.dctr->nfb, 1u)] = pix;
}

// One traced segment of pass A: its event (slot `slot`, linked to `link` of pixel `pix`), its
// shadow queries and its children.  `h` is the segment's closest hit (unused when the event
// pool overflowed).  On return `have` says whether the lane continues with a child (then in
// `cur` / `link`), and `have_other` whether it offers a second child to the wave.
template <bool SPLIT>
__device__ __forceinline__ void defer_shade(const KArgs& A, EvLog& L, uint32_t slot, const Hit& h, Seg& cur,
                                            uint32_t& link, uint32_t pix, bool& have, PSeg& other, bool& have_other) {
    const int D = (int)A.max_depth;
    Cnt cnt;
    have = false;
    const DScratch& S = L.S;
    if (L.ovf && link == kEvRoot) { // no event this frame yet: list the pixel
        atomicExch(&S.px_ev[pix].x, kEvNone);
        S.fb[atomicAdd(&S.dctr->nfb, 1u)] = pix;
        return;
    }
    if (L.ovf) {
        defer_mark_fallback(S, pix);
        return;
    }
    // where this segment's event lives: the pixel's root, or its parent's child link
    if (link == kEvRoot) atomicExch(&S.px_ev[pix].x, slot);
    else reinterpret_cast<uint32_t*>(ev_plane(S.ev, link >> 1, 3))[2u + (link & 1u)] = slot;
    if (h.kind == HIT_NONE) {
        const f3 c = muls(background(A, cur.d), cur.thr);
        *ev_plane(S.ev, slot, 0) = make_float4(c.x, c.y, c.z, __uint_as_float(kEvTagConst));
        return;
    }
    const Surf s = resolve_hit<false>(A, cur, h, cnt);
    const f3 v = neg(cur.d);
    float dterm[3] = {0.0f, 0.0f, 0.0f}, sterm[3] = {0.0f, 0.0f, 0.0f};
    uint32_t qmask = 0; // lights whose shadow query went to A.shq
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const LightTerm t = light_term(A, s, v, i);
        if (!t.matters) continue;
        // append the query (lanes of one light together: neighbouring queries of the dense
        // pass-B queue share a light and nearby origins)
        const uint64_t m = __ballot(true);
        const int leader = __ffsll((unsigned long long)m) - 1;
        uint32_t base = 0;
        if ((int)lane_id() == leader) base = atomicAdd(&S.dctr->nq[L.stripe * kCtrStride], (uint32_t)__popcll(m));
        base = __shfl(base, leader, 64);
        const uint32_t qi = base + lane_rank(m);
        if (qi < A.shq_cap) {
            float4* q = S.shq + 2 * ((size_t)L.stripe * A.shq_cap + qi);
            q[0] = make_float4(t.so.x, t.so.y, t.so.z, t.dist);
            q[1] = make_float4(t.ld.x, t.ld.y, t.ld.z, __uint_as_float((slot << 2) | (uint32_t)i));
            qmask |= 1u << i;
            dterm[i] = t.diff;
            sterm[i] = t.spec;
        } else {
            L.ovf = true;
        }
    }
    bool mk_refr, mk_refl;
    Seg refr, refl;
    make_children(cur, s, D, refr, mk_refr, refl, mk_refl);
    const uint32_t lrefl = slot << 1, lrefr = (slot << 1) | 1u;
    const uint32_t kids = (mk_refl ? kEvTagRefl : 0u) | (mk_refr ? kEvTagRefr : 0u);
    if (SPLIT && cur.depth + 1 >= (int)A.split_d1 && !L.ovf) {
        // window edge: both children become tasks of the next round
        bool sa = mk_refl, sb = mk_refr;
        enqueue2<true>(A, sa, refl, sb, refr, pix, lrefl, lrefr);
        if (sa != mk_refl || sb != mk_refr) L.ovf = true; // task queue full
        mk_refl = mk_refr = false;
    }
    if (L.ovf) {
        defer_mark_fallback(S, pix);
        return;
    }
    if (qmask == 0u) { // no light can add anything: the colour term is known now
        f3 diffuse = mk(0.0f, 0.0f, 0.0f), specular = mk(0.0f, 0.0f, 0.0f);
        const f3 c = muls(add(muls(diffuse, s.alb[0]), muls(specular, s.alb[1])), cur.thr);
        *ev_plane(S.ev, slot, 0) = make_float4(c.x, c.y, c.z, __uint_as_float(kEvTagConst | kids));
    } else { // pass B ORs the occluded lights into plane 3's second word
        *ev_plane(S.ev, slot, 0) = make_float4(s.kd[0], s.kd[1], s.kd[2], __uint_as_float(qmask | kids));
        *ev_plane(S.ev, slot, 1) = make_float4(dterm[0], dterm[1], dterm[2], s.alb[0]);
        *ev_plane(S.ev, slot, 2) = make_float4(sterm[0], sterm[1], sterm[2], s.alb[1]);
        *reinterpret_cast<float2*>(ev_plane(S.ev, slot, 3)) = make_float2(cur.thr, 0.0f);
    }
    // continue with the reflection child (the reference pops it first; here it keeps the lane
    // on nearby rays), offer the refraction child to the wave
    if (mk_refl) {
        if (mk_refr) {
            other = PSeg{refr, lrefr, pix};
            have_other = true;
        }
        cur = refl;
        link = lrefl;
        have = true;
    } else if (mk_refr) {
        cur = refr;
        link = lrefr;
        have = true;
    }
}

// The wave's pending-segment pool (defer_walk): a lane without work takes its
// private overflow first, then the pool's top entries (wave-aggregated, one per idle lane by
// rank); `want` lanes get work.  pool_n is wave-uniform.
__device__ __forceinline__ void pool_refill(const lds_f32* P, uint32_t& pool_n, PSeg* priv, int& pn, bool want,
                                            bool& got, Seg& cur, uint32_t& link, uint32_t& pix) {
    got = false;
    if (want && pn > 0) {
        --pn;
        cur = priv[pn].s;
        link = priv[pn].link;
        pix = priv[pn].pix;
        got = true;
    }
    const uint64_t idle = __ballot(want && !got);
    if (idle != 0ull && pool_n != 0u) {
        const uint32_t take = min((uint32_t)__popcll(idle), pool_n);
        if (want && !got) {
            const uint32_t r = lane_rank(idle);
            if (r < take) {
                const PSeg x = pool_get(P, pool_n - 1u - r);
                cur = x.s;
                link = x.link;
                pix = x.pix;
                got = true;
            }
        }
        pool_n -= take;
    }
}
// Lanes with a second child put it into the pool (or their private overflow when it is full).
__device__ __forceinline__ void pool_offer(lds_f32* P, uint32_t& pool_n, PSeg* priv, int& pn, bool have_other,
                                           const PSeg& other) {
    const uint64_t pm = __ballot(have_other);
    if (pm == 0ull) return;
    const uint32_t room = kPool - pool_n;
    wave_lds_sync(); // this step's takes have read the entries the pushes may reuse
    if (have_other) {
        const uint32_t r = lane_rank(pm);
        if (r < room) pool_put(P, pool_n + r, other);
        else priv[pn++] = other;
    }
    pool_n += min((uint32_t)__popcll(pm), room);
    wave_lds_sync(); // the pushes land before the next step's takes
}

// Pass A over the segments the wave's lanes start with (`have`: the lane holds `cur`, whose
// event links to `link` of pixel `pix`) and everything they spawn.  Every lane of the wave
// must call it (ballots, the shared pool); it returns when no lane holds work.
template <int GEOM, bool SPLIT>
__device__ __forceinline__ void defer_walk(const KArgs& A, float* lds, float4* slab, EvLog& L, bool have, Seg cur,
                                           uint32_t link, uint32_t pix) {
    lds_f32* P = (lds_f32*)lds;
    Cnt cnt;
    PSeg priv[kMaxTreeDepth];
    int pn = 0;
    uint32_t pool_n = 0; // wave-uniform
#ifdef TRT_DIAG_PASSA_STEPS
    // diagnostic: per wave, steps and lanes with a segment per step, weighted by the step's
    // duration (100-MHz clock): counters[24..28] = sum dt, sum active * dt, steps, sum active, waves
    unsigned long long d_dt = 0, d_adt = 0, d_steps = 0, d_act = 0;
    uint64_t d_t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t d_a = 0;
#endif
    for (;;) {
        bool got;
        pool_refill(P, pool_n, priv, pn, !have, got, cur, link, pix);
        have = have || got;
#ifdef TRT_DIAG_PASSA_STEPS
        {
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            if (d_steps) {
                d_dt += t - d_t0;
                d_adt += (t - d_t0) * d_a;
            }
            d_t0 = t;
            d_a = (uint32_t)__popcll(__ballot(have));
            if (d_a) {
                ++d_steps;
                d_act += d_a;
            }
        }
#endif
        if (__ballot(have) == 0ull) {
#ifdef TRT_DIAG_PASSA_STEPS
            if (lane_id() == 0u) {
                atomicAdd(&A.counters[24], d_dt);
                atomicAdd(&A.counters[25], d_adt);
                atomicAdd(&A.counters[26], d_steps);
                atomicAdd(&A.counters[27], d_act);
                atomicAdd(&A.counters[28], 1ull);
            }
#endif
            break;
        }
        // every lane takes this step's slot, working or not: the lanes stay on one row of one
        // chunk (one chunk per kEvRows steps of the wave, coalesced event stores); idle lanes'
        // slots stay unused
        const uint32_t slot = ev_alloc(A, L);
        bool have_other = false;
        PSeg other;
        if (have) {
            Hit h;
            h.kind = HIT_NONE;
            if (!L.ovf) scene_intersect<false, GEOM>(A, cur.o, cur.d, h, cnt, slab);
            defer_shade<SPLIT>(A, L, slot, h, cur, link, pix, have, other, have_other);
        }
        pool_offer(P, pool_n, priv, pn, have_other, other);
    }
}

template <int CAP, bool COUNT, int GEOM>
__device__ __forceinline__ f3 cast_ray(const KArgs& A, f3 orig, f3 dir, Cnt& cnt, float* lds,
                                       float4* slab) {
    bool unused = false;
    const f3 c = cast_seg<CAP, COUNT, GEOM, false>(A, Seg{orig, dir, 1.0f, 0}, cnt, lds, slab, 0u, unused);
    return mk(clamp01(c.x), clamp01(c.y), clamp01(c.z)); // shader.comp:582
}

// ---- primary rays (main.cpp:1496-1506 on the host; shader.comp:592-595) -----------------

__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

__device__ __forceinline__ f3 primary_dir(const KArgs& A, uint32_t x, uint32_t y, uint32_t sample) {
    const uint32_t W = A.width, H = A.height;
    const uint32_t pix = y * W + x; // W, H <= 65536: fits
    f3 d;
    if (A.rays_in) {
        const float* r = A.rays_in + 8 * (size_t)pix; // Ray.dir (binding 1)
        d = mk(r[0], r[1], r[2]);
    } else {
        // main.cpp:1501-1502 divides pix + 1 by W; with x + 1 <= W that is y + (x + 1 == W):
        // the last column takes the next row's dy (App. B-1).  No 64-bit division per pixel.
        const uint32_t row = ((A.flags & TRT_FLAG_ROW_QUIRK) && x + 1u == W) ? y + 1u : y;
        float dx, dy;
        if (A.spp <= 1) { // exact in float: half-integers (main.cpp:1501-1502)
            dx = ((float)x + 0.5f) - (float)W * 0.5f;
            dy = -((float)row + 0.5f) + (float)H * 0.5f;
        } else {
            uint32_t k = pcg_hash(A.seed ^ 0x9E3779B9u);
            uint32_t a = pcg_hash(k + (uint32_t)pix);
            uint32_t b = pcg_hash(a + sample);
            uint32_t c = pcg_hash(b);
            float jx = (float)(b >> 8) * (1.0f / 16777216.0f);
            float jy = (float)(c >> 8) * (1.0f / 16777216.0f);
            dx = ((float)x + jx) - (float)W * 0.5f;
            dy = (float)H * 0.5f - ((float)row + jy);
        }
        d = normalize3(mk(dx, dy, A.dz)); // glm::normalize, main.cpp:1504
    }
    return normalize3(d); // shader.comp:593
}

// ---- the kernel ------------------------------------------------------------------------

__device__ __forceinline__ uint32_t band_row(const KArgs& A, uint32_t k) {
    if (A.band_rows == 0 || A.band_count <= 1) return k;
    return band_frame_row(k, A.band_rows, A.band_count, A.band_index); // trt_bands.h
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// Gamma (shader.comp:598) and the dual store (rayOut binding 2, storage image binding 3) of
// output pixel o; `c` is the clamped colour.
__device__ __forceinline__ void store_pixel(const KArgs& A, const FrameRec& F, size_t o, f3 c) {
    if (F.in_place) { // compact row k -> its frame row (band_row)
        const uint32_t k = (uint32_t)(o / A.width), x = (uint32_t)(o % A.width);
        o = (size_t)band_row(A, k) * A.width + x;
    }
    const float gx = pow_pos(c.x, TRT_GAMMA), gy = pow_pos(c.y, TRT_GAMMA), gz = pow_pos(c.z, TRT_GAMMA);
#ifdef TRT_DIAG_WAVE_CLOCK
    if (false) // out32 carries the workgroup clock records
#else
    if (A.out32) // rayOut[idx].resultColor, shader.comp:601
#endif
    {
        reinterpret_cast<float4*>(A.out32)[o] = make_float4(gx, gy, gz, 1.0f);
    }
    if (F.out8) { // rgba8 storage image, shader.comp:61, 600
        float ex = gx, ey = gy, ez = gz;
        if (A.flags & TRT_FLAG_SRGB_OUT) { // as displayed through the sRGB swapchain
            ex = srgb_encode(gx);
            ey = srgb_encode(gy);
            ez = srgb_encode(gz);
        }
        uint32_t r = (uint32_t)floorf(ex * 255.0f + 0.5f);
        uint32_t g = (uint32_t)floorf(ey * 255.0f + 0.5f);
        uint32_t b = (uint32_t)floorf(ez * 255.0f + 0.5f);
        F.out8[o] = r | (g << 8) | (b << 16) | (255u << 24);
    }
}

// One 8x8 pixel tile of compact output rows: the wave's 64 lanes, one pixel each.  SPLIT
// (spp == 1 only): a pixel whose tree handed subtrees to the task queue parks its partial
// colour in A.acc and is finished by finalize_spilled.
// DEFER: pass A with A.defer_sub > 1 gives each tile defer_sub waves (sub = 0 .. defer_sub - 1):
// wave `sub` starts with 64 / defer_sub of the tile's pixels (rows sub * 8 / defer_sub ...) and
// its other lanes take work from the wave's segment pool as the trees grow, so a glass tile's
// segments are spread over more waves (a shorter frame latency) at the price of idle lanes in
// cheap tiles.
template <int CAP, bool COUNT, int GEOM, bool SPLIT, bool DEFER = false, bool HYB = SPLIT>
__device__ __forceinline__ void trace_tile(const KArgs& A, const FrameRec& F, uint32_t tile, Cnt& cnt, float* lds,
                                           float4* slab, uint32_t sub = 0, uint32_t frame = 0) {
    const uint32_t lane = lane_id();
    if (tile >= A.ntiles) return;
    const uint32_t x = (tile % A.ntx) * 8u + (lane & 7u);
    uint32_t k = (tile / A.ntx) * 8u + (lane >> 3);
    const f3 orig = mk(F.cam[0], F.cam[1], F.cam[2]);
    if constexpr (DEFER) { // pass A of a deferred-shadow frame (spp == 1): every lane walks
        // (split launches keep one wave per tile: their grid is the tile count)
        const uint32_t S = (!SPLIT && A.defer_sub > 1u) ? A.defer_sub : 1u, rows = 8u / S;
        k = (tile / A.ntx) * 8u + sub * rows + (lane >> 3);
        const bool valid = x < A.width && k < A.rows && (lane >> 3) < rows;
        EvLog L;
        L.S = dscratch(A, frame); // this frame's scratch (frame `frame` of the launch)
        // multiplicative hash of the tile: a frame's costly region (a glass object) spans few
        // tile columns, so tile % stripes would pile its queries into a few stripes
        L.stripe = ((tile * S + sub) * 0x9E3779B1u) >> (32 - 7);
        static_assert(kDeferStripes == 128u, "stripe hash yields 7 bits");
        const size_t o = valid ? (size_t)k * A.width + x : 0u;
        const Seg root = valid ? Seg{orig, primary_dir(A, x, band_row(A, k), 0), 1.0f, 0} : Seg{orig, orig, 0.0f, 0};
        defer_walk<GEOM, SPLIT>(A, lds, slab, L, valid, root, kEvRoot, (uint32_t)o);
        return;
    }
    if (x >= A.width || k >= A.rows) return;
#ifdef TRT_DIAG_TRIVIAL
    if (F.out8) F.out8[(size_t)k * A.width + x] = 0xff000000u | x; // diagnostic: launch + store only
    return;
#endif
    const uint32_t y = band_row(A, k);
    const size_t o = (size_t)k * A.width + x;
    if (SPLIT) {
        bool spilled = false;
        const f3 c = cast_seg<CAP, COUNT, GEOM, true>(A, Seg{orig, primary_dir(A, x, y, 0), 1.0f, 0}, cnt, lds,
                                                      slab, (uint32_t)o, spilled);
        cnt.pri += 1;
        const uint64_t sp = __ballot(spilled);
        if (spilled) {
            unsigned long long* a = A.acc + 4 * o;
            a[0] = to_fixed(c.x);
            a[1] = to_fixed(c.y);
            a[2] = to_fixed(c.z);
        }
        if (sp) {
            const int leader = __ffsll((unsigned long long)sp) - 1;
            uint32_t base = 0;
            if ((int)lane == leader) base = atomicAdd(&A.ctr->spilled, (uint32_t)__popcll(sp));
            base = __shfl(base, leader, 64);
            if (spilled) A.spilled[base + lane_rank(sp)] = (uint32_t)o;
        }
        if (!spilled) store_pixel(A, F, o, mk(clamp01(c.x), clamp01(c.y), clamp01(c.z)));
        return;
    }
    const uint32_t spp = A.spp ? A.spp : 1u;
    f3 acc = mk(0.0f, 0.0f, 0.0f);
    for (uint32_t s = 0; s < spp; ++s) {
        f3 d = primary_dir(A, x, y, s);
        f3 c = cast_ray<CAP, COUNT, GEOM>(A, orig, d, cnt, lds, slab);
        acc = (spp == 1u) ? c : add(acc, c);
    }
    cnt.pri += spp;
    if (spp > 1u) acc = mk(div_rn(acc.x, (float)spp), div_rn(acc.y, (float)spp), div_rn(acc.z, (float)spp));
#ifdef TRT_DIAG_PIXEL_WORK
    // diagnostic: out32 = (node visits, triangle tests, segments, max node visits of one query)
    if (A.out32) reinterpret_cast<float4*>(A.out32)[o] = make_float4((float)cnt.wn, (float)cnt.wt, (float)cnt.wseg, (float)cnt.wmax);
    return;
#endif
    store_pixel(A, F, o, acc);
}

// spp > 1 with one lane per SAMPLE (A.spp_lanes; spp a power of two in [2, 64]).  Wave `sub` of
// 8x8 tile `tile` traces the 64 / spp pixels of sub-block `sub` (2x2 pixels at 16 spp), spp lanes
// per pixel: the 16 jittered samples of a pixel are nearly one ray, so a wave's walks are far
// more coherent than 64 neighbouring pixels' (the wave-uniform node fetch fires more often) and
// the wave-coherent shadow walk applies to all of them.  The pixel's colour is then the
// per-pixel loop's running sum, ((0 + c0) + c1) + ..., gathered from its lanes in sample order
// with the same additions, and divided by spp — bit-identical to trace_tile's loop.
template <int CAP, bool COUNT, int GEOM>
__device__ __forceinline__ void trace_samples(const KArgs& A, const FrameRec& F, uint32_t tile, uint32_t sub, Cnt& cnt,
                                              float* lds, float4* slab) {
    const uint32_t lane = lane_id();
    if (tile >= A.ntiles) return;
    const uint32_t spp = A.spp, lg = 31u - __builtin_clz(64u / spp); // log2 of the pixels per wave
    const uint32_t bw = 1u << ((lg + 1u) / 2u), bh = (64u / spp) / bw;  // sub-block of bw x bh pixels
    const uint32_t cols = 8u / bw;
    const uint32_t pi = lane / spp, smp = lane % spp;
    const uint32_t x = (tile % A.ntx) * 8u + (sub % cols) * bw + pi % bw;
    const uint32_t k = (tile / A.ntx) * 8u + (sub / cols) * bh + pi / bw;
    const bool valid = x < A.width && k < A.rows;
    f3 c = mk(0.0f, 0.0f, 0.0f);
    if (valid) {
        const f3 orig = mk(F.cam[0], F.cam[1], F.cam[2]);
        c = cast_ray<CAP, COUNT, GEOM>(A, orig, primary_dir(A, x, band_row(A, k), smp), cnt, lds, slab);
        cnt.pri += 1;
    }
    // the sample-order sum, gathered by every lane from its pixel's lanes (lane base + t holds
    // sample t); lanes of invalid pixels gather their (zero) colours and store nothing
    const int base = (int)(lane - smp);
    f3 acc = mk(0.0f, 0.0f, 0.0f);
    for (uint32_t t = 0; t < spp; ++t) {
        const int src = base + (int)t;
        acc = add(acc, mk(__shfl(c.x, src, 64), __shfl(c.y, src, 64), __shfl(c.z, src, 64)));
    }
    if (!valid || smp != 0u) return;
    acc = mk(div_rn(acc.x, (float)spp), div_rn(acc.y, (float)spp), div_rn(acc.z, (float)spp));
    store_pixel(A, F, (size_t)k * A.width + x, acc);
}

// Blocks b and b+8 share an XCD (round-robin dispatch, MI355X_MICROARCH.md): give each XCD
// 2x2-tile chunks (16x16 px) so neighbouring pixels' envmap texels and batch records hit
// the same XCD L2.  Chunk c of XCD x is global chunk c*8+x; chunks are row-major over the
// image in 2x2 tile units.  Bijective on [0, ntiles) (tail tiles map to themselves).
//
// Frame f of a multi-frame launch can deal the chunk classes rotated (xcd_rot: class
// (x + f / 2^(xcd_rot - 1)) mod 8 to XCD x) and skewed per chunk row (xcd_skew: row cy's chunk
// columns shifted by xcd_skew * cy, diagonal classes).  Both are bijections of the chunks, so
// every tile is traced once; they only move work between XCDs.  Why: the hardware deals blocks
// to the XCDs round-robin, statically, so an XCD whose chunk class is costlier (the glass
// spheres' stripes) finishes its share of a launch later than the others.
// perm (xcd_inter 2): chunk k of the evenly dealt ones is chunk (k * xcd_mult) mod nfull, a
// bijection (xcd_mult is coprime to nfull) that makes each XCD's chunks a 2-D lattice spread over
// the whole image instead of every 8th chunk column.
__device__ __forceinline__ uint32_t xcd_deal(const KArgs& A, uint32_t b, uint32_t roff, bool perm = false) {
    const uint32_t tyn = A.ntiles / A.ntx;
    const uint32_t cw = A.ntx / 2u, ch = tyn / 2u;                 // whole 2x2 chunks
    const uint32_t nchunk = cw * ch, nfull = (nchunk / 8u) * 8u;   // dealt evenly to the XCDs
    auto chunk_tile = [&](uint32_t chunk, uint32_t sub) {
        uint32_t cx = chunk % cw;
        const uint32_t cy = chunk / cw;
        if (A.xcd_skew) cx = (cx + A.xcd_skew * cy) % cw;
        return (cy * 2u + sub / 2u) * A.ntx + cx * 2u + (sub % 2u);
    };
    if (b < nfull * 4u) {
        const uint32_t j = b / 8u; // j-th block of XCD x
        uint32_t x = b % 8u;
        x = (x + roff) & 7u;
        uint32_t k = (j / 4u) * 8u + x;
        if (perm) k = (k * A.xcd_mult) % nfull; // fits 32 bits: the host keeps xcd_mult 1 for >= 65536 chunks
        return chunk_tile(k, j % 4u);
    }
    // leftovers: the last nchunk % 8 chunks, then the odd right column, then the odd bottom row
    uint32_t r = b - nfull * 4u;
    const uint32_t nc = (nchunk - nfull) * 4u;
    if (r < nc) return chunk_tile(nfull + r / 4u, r % 4u);
    r -= nc;
    const uint32_t na = (A.ntx & 1u) ? ch * 2u : 0u;
    if (r < na) return r * A.ntx + (A.ntx - 1u);
    r -= na;
    return (ch * 2u) * A.ntx + r; // tile rows odd: the last tile row
}

// Block b's tile with the chunk classes rotated for frame f of this launch (xcd_rot: by
// f / 2^(xcd_rot - 1)).  Successive single-frame launches keep one dealing: rotating them too
// (a per-launch offset) cost the shipped frame's 8 in-flight deferred frames +5 % (consecutive
// frames' tiles on one XCD share its L2) for README -2 %, profiles/r03_ab_launch_off.log.
__device__ __forceinline__ uint32_t xcd_tile(const KArgs& A, uint32_t b, uint32_t f = 0) {
    return xcd_deal(A, b, A.xcd_rot ? (f >> (A.xcd_rot - 1u)) : 0u);
}
// the unrotated dealing
__device__ __forceinline__ uint32_t xcd_tile_base(const KArgs& A, uint32_t b) { return xcd_deal(A, b, 0u); }

// Frame-interleaved dealing of a multi-frame launch (xcd_inter): the launch walks the chunk
// groups once, and each XCD traces chunk group g of every frame before group g + 1 (frame f's
// chunk of group g rotated by f, so every XCD sees every chunk class).  All frames advance
// together, so the launch ends on the last chunk groups of all frames instead of on the last
// frame's whole tile order (whose costliest tiles then start near the end).  Sets f; tiles
// outside whole chunk groups (leftovers) are dealt frame by frame after them.
// F: the launch's frames (or frame pairs, frame_pair).
// xcd_inter 2: no rotation — chunk group g's chunk on XCD x is the same in every frame of the
// launch, so that XCD traces that chunk in all frames back to back and the texels its primary
// rays miss into (the same directions in every frame: the camera only translates) stay in its L2;
// the permuted classes (xcd_deal perm) keep the XCDs balanced without the rotation.
__device__ __forceinline__ uint32_t inter_tile(const KArgs& A, uint32_t vb, uint32_t& f, uint32_t F) {
    const uint32_t tyn = A.ntiles / A.ntx;
    const uint32_t nchunk = (A.ntx / 2u) * (tyn / 2u), nfull = (nchunk / 8u) * 8u;
    const uint32_t per = nfull * 4u; // blocks per frame in whole chunk groups
    if (vb < F * per) {
        const uint32_t x = vb % 8u, i = vb / 8u, q = i / 4u;
        f = q % F;
        const uint32_t g = q / F; // chunk group: chunks g * 8 .. g * 8 + 7
        // block (g * 8 + ((x + f) & 7)) * 4 + i % 4 of frame f, in xcd_tile's unrotated dealing
        const bool fixed = A.xcd_inter == 2u;
        const uint32_t c = fixed ? x : (x + f) & 7u;
        return xcd_deal(A, (g * 4u + i % 4u) * 8u + c, 0u, fixed);
    }
    const uint32_t r = vb - F * per, nl = A.ntiles - per;
    f = r / nl;
    return xcd_tile_base(A, per + r % nl);
}

// One 64-lane workgroup per 8x8 tile.  The hardware dispatcher hands each freed wave slot
// the next tile, which balances the very uneven per-tile cost (sky vs. glass sphere) with
// no atomics.  (Measured on C2: a persistent grid pulling tiles from per-XCD atomic queue
// heads was 1.5-4.5x slower — 12,288 dequeues per ~60 us frame saturate the heads — and a
// static grid-stride over the resident waves 1.2-2x slower from imbalance.)
// GEOM: 0 = no triangles (spheres/floor only, e.g. C1/C2: the triangle code is compiled
// out, 4 waves per SIMD); 1 = the reference-order batch walk; 2 = per-lane BVH.
#ifndef TRT_WAVES
#define TRT_WAVES 1
#endif
// Frame pairs (TRT_FRAME_GROUP=2) for mesh frames: compiled only on request (measured slower
// for meshes: C4 +2.5 %, C3 +10 %, profiles/r03_ab_frame_pair.log)
#ifndef TRT_MESH_PAIRS
#define TRT_MESH_PAIRS 0
#endif

__device__ __forceinline__ void flush_counts(const KArgs& A, const Cnt& cnt) {
    const uint32_t v[20] = {cnt.pri, cnt.sec, cnt.sh, cnt.miss, cnt.trin, cnt.sph, cnt.bt, cnt.bh, cnt.tt, cnt.nt,
                            cnt.ta, cnt.tu, cnt.tv, cnt.sk, cnt.ssph, cnt.sbox, cnt.stt, cnt.sta, cnt.stu, cnt.stv};
#pragma unroll
    for (int i = 0; i < 20; ++i) {
        unsigned long long w = wave_sum((unsigned long long)v[i]);
        if (lane_id() == 0) atomicAdd(&A.counters[i], w);
    }
}

template <int GEOM>
constexpr int slab_float4s() {
    return GEOM == 1 ? 64 * 3 : GEOM >= 2 ? (bvh_lds_entries<GEOM>() > 0 ? bvh_lds_entries<GEOM>() * 16 : 1) : 1;
}
// Triangle-free frames (GEOM 0: C1 / C2) are latency-bound on the dependent chain intersection
// -> shading -> envmap gather; 5 waves per SIMD (<= 96 VGPRs) hide more of it than the 4 the
// unconstrained build reaches (109 VGPRs): C2 15.5 -> 14.2 us per frame (round 3,
// profiles/r03_ab_waves_c2.log; round 1 measured a 6-wave cap 20 % slower).
#ifndef TRT_G0_WAVES
#define TRT_G0_WAVES 5
#endif
template <int GEOM, int CAP = 99>
constexpr int waves_per_simd() {
    return GEOM == 3 ? (CAP <= 3 ? TRT_G3_WAVES_SHALLOW : TRT_G3_WAVES) : GEOM == 0 ? TRT_G0_WAVES : TRT_WAVES;
}

// Waves per SIMD of pass A of a deferred frame (the quantized walk without shadow rays): 4 like
// the other deep walks, or TRT_DEFER_WAVES.
#ifndef TRT_DEFER_WAVES
#define TRT_DEFER_WAVES 4
#endif
template <int GEOM, int CAP, bool SPLIT, bool DEFER>
constexpr int trace_waves() {
    return (DEFER && GEOM == 3) ? TRT_DEFER_WAVES : waves_per_simd<GEOM, ((SPLIT || DEFER) ? 99 : CAP)>();
}

template <int CAP, bool COUNT, int GEOM, bool SPLIT, bool DEFER = false, bool HYB = SPLIT>
__global__ __launch_bounds__(64, (trace_waves<GEOM, CAP, SPLIT, DEFER>())) void trace_kernel(KArgs A) {
    __shared__ float lds[DEFER ? defer_pool_floats() : lds_stack_floats<CAP, GEOM, HYB>()];
    // GEOM 1: one batch slab, 64 x (v0, e1, e2); GEOM 2: the BVH traversal stacks
    __shared__ float4 slab[slab_float4s<GEOM>()];
    const uint32_t vb = blockIdx.x;
    Cnt cnt;
#ifdef TRT_DIAG_WAVE_CLOCK
    // diagnostic: per-workgroup (tile | xcc << 28, start lo, duration, start hi) of the
    // 100 MHz constant clock, written to out32 (tools/waveclock.py)
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    // frame f = vb / ntiles of a multi-frame launch (plain frames only: split / deferred frames
    // and counting passes launch one frame)
    uint32_t f = 0, t = vb, tile;
    if (!SPLIT && !DEFER && A.spp_lanes) { // one lane per sample: ntiles * spp waves per frame
        const uint32_t per = A.ntiles * A.spp;
        f = vb / per;
        const uint32_t r = vb - f * per;
        trace_samples<CAP, COUNT, GEOM>(A, A.fr[f], xcd_tile(A, r / A.spp), r % A.spp, cnt, lds, slab);
        if (COUNT) flush_counts(A, cnt);
        return;
    }
    if (!SPLIT && !DEFER && A.nframes > 1u) {
        // frame pairs serve triangle-free frames only (the host sets frame_group 2 for them by
        // default): mesh kernels do not compile the two extra trace_tile copies (code size)
        if (A.xcd_inter && A.frame_group > 1u && (GEOM == 0 || TRT_MESH_PAIRS)) {
            // frame pairs: the block traces its tile in frames 2p and 2p + 1 (consecutive frames'
            // tiles cost nearly the same, so the pairs keep the waves balanced) — half the
            // workgroups, so half the per-workgroup launch and slot-refill overhead.  Two calls,
            // not a loop over a group size: the loop form compiled to a slower kernel (C2 13.8 ->
            // 14.9 us per frame, profiles/r03_ab_frame_group_loop.log)
            uint32_t pr;
            tile = inter_tile(A, vb, pr, (A.nframes + 1u) / 2u);
            f = 2u * pr;
            trace_tile<CAP, COUNT, GEOM, SPLIT, DEFER, HYB>(A, A.fr[f], tile, cnt, lds, slab);
            if (f + 1u < A.nframes) trace_tile<CAP, COUNT, GEOM, SPLIT, DEFER, HYB>(A, A.fr[f + 1u], tile, cnt, lds, slab);
            if (COUNT) flush_counts(A, cnt);
            return;
        } else if (A.xcd_inter) {
            tile = inter_tile(A, vb, f, A.nframes);
        } else {
            f = vb / A.ntiles;
            t = vb - f * A.ntiles;
            tile = xcd_tile(A, t, f);
        }
    } else if (DEFER && !SPLIT) { // defer_sub waves per tile of each of dframes frames (trace_tile)
        const uint32_t Sd = A.defer_sub > 1u ? A.defer_sub : 1u, per = A.ntiles * Sd;
        if (A.defer_inter && A.dframes > 1u) {
            // the group's frames block by block, so they advance together; within each XCD
            // (block vb runs on XCD vb % 8), so every XCD traces every frame, with frame f's
            // chunk classes (xcd_tile: class t % 8) rotated by f as inter_tile does, so every
            // XCD also sees every class (a costly class on one XCD would end the group late);
            // blocks past the last whole round of 8 are dealt frame by frame
            const uint32_t F = A.dframes, per8 = per & ~7u;
            if (vb < F * per8) {
                const uint32_t x = vb & 7u, j = vb >> 3;
                f = j % F;
                t = (j / F) * 8u + ((x + f) & 7u);
            } else {
                const uint32_t r = vb - F * per8, nl = per - per8;
                f = r / nl;
                t = per8 + r % nl;
            }
        } else {
            f = vb / per;
            t = vb - f * per;
        }
        tile = xcd_tile(A, t / Sd);
        trace_tile<CAP, COUNT, GEOM, SPLIT, DEFER, HYB>(A, A.fr[f], tile, cnt, lds, slab, t % Sd, f);
#ifdef TRT_DIAG_WAVE_CLOCK
        // diagnostic: pass A's record per block of a single deferred frame in out32 (waveclock.py
        // --records ntiles * defer_sub)
        if (threadIdx.x == 0 && A.out32 && A.dframes <= 1u) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            uint32_t* rec = reinterpret_cast<uint32_t*>(A.out32) + 4 * (size_t)blockIdx.x;
            uint32_t xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            rec[0] = tile | ((xcc & 15u) << 28);
            rec[1] = (uint32_t)t_start;
            rec[2] = (uint32_t)(t_end - t_start);
            rec[3] = (uint32_t)(t_start >> 32);
        }
#endif
        return;
    } else {
        tile = xcd_tile(A, t);
    }
    trace_tile<CAP, COUNT, GEOM, SPLIT, DEFER, HYB>(A, A.fr[f], tile, cnt, lds, slab);
#ifdef TRT_DIAG_WAVE_CLOCK
    __syncthreads();
    // single-frame launches write the records to out32; multi-frame launches to the diagnostic
    // buffer (trt_diag_set_buffer), with the frame in bits 20-27
    float* clk = A.out32 ? A.out32 : reinterpret_cast<float*>(A.diag);
    if (threadIdx.x == 0 && clk) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t* rec = reinterpret_cast<uint32_t*>(clk) + 4 * (size_t)blockIdx.x;
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        rec[0] = (A.out32 ? xcd_tile(A, blockIdx.x) : (tile | (f << 20))) | ((xcc & 15u) << 28);
        rec[1] = (uint32_t)t_start;
        rec[2] = (uint32_t)(t_end - t_start);
        rec[3] = (uint32_t)(t_start >> 32);
    }
#endif
    if (COUNT) flush_counts(A, cnt);
}

// One round of a split frame: persistent waves take 64 tasks at a time (static schedule) from
// the previous launch's queue, trace each task's subtree within the depth window (its
// window-edge children go to the next queue) and add the subtree's colour to its pixel's
// fixed-point sum.  Every wave leaves once the queue is drained.
//
// DEFER: a task is a segment of some pixel's tree whose event links into its parent's (the
// link its parent queued with it); the wave's 64 tasks and their subtrees share the wave's
// segment pool (defer_walk).
template <int CAP, bool COUNT, int GEOM, bool DEFER = false>
__global__ __launch_bounds__(64, waves_per_simd<GEOM>()) void trace_tasks(KArgs A) {
    __shared__ float lds[DEFER ? defer_pool_floats() : lds_stack_floats<CAP, GEOM, true>()];
    __shared__ float4 slab[slab_float4s<GEOM>()];
    Cnt cnt;
    const uint32_t n = min(*A.q_in_n, A.q_cap);
    // static schedule: wave b takes the 64-task blocks b, b + G, ... (a dequeue atomic per block
    // on one device-scope counter cost ~4x the tasks' own work: profiles/r02_ab_tasks_static.log)
    for (uint32_t base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u) {
        const uint32_t t = base + threadIdx.x;
        if constexpr (DEFER) {
            const bool valid = t < n;
            Seg root{mk(0.0f, 0.0f, 0.0f), mk(0.0f, 0.0f, 0.0f), 0.0f, 0};
            uint32_t pixel = 0, link = kEvRoot;
            if (valid) {
                const float4* q = reinterpret_cast<const float4*>(A.q_in + t);
                const float4 a = q[0], b = q[1];
                const uint32_t pd = __float_as_uint(b.w);
                pixel = pd >> kTaskDepthBits;
                root = Seg{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), b.z, (int)(pd & ((1u << kTaskDepthBits) - 1u))};
                link = A.q_link_in[t];
            }
            EvLog L;
            L.S = dscratch(A, 0u); // split launches trace one frame
            // wave-uniform (ev_alloc and the query appends reserve from one stripe per wave)
            L.stripe = ((base / 64u + 0x5bd1e995u * A.split_d1) * 0x9E3779B1u) >> (32 - 7);
            defer_walk<GEOM, true>(A, lds, slab, L, valid, root, link, pixel);
            continue;
        }
        if (t < n) {
            const float4* q = reinterpret_cast<const float4*>(A.q_in + t);
            const float4 a = q[0], b = q[1];
            const uint32_t pd = __float_as_uint(b.w);
            const uint32_t pixel = pd >> kTaskDepthBits;
            const Seg root{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), b.z, (int)(pd & ((1u << kTaskDepthBits) - 1u))};
            bool spilled = false;
            const f3 c = cast_seg<CAP, COUNT, GEOM, true>(A, root, cnt, lds, slab, pixel, spilled);
            unsigned long long* acc = A.acc + 4 * (size_t)pixel;
            atomicAdd(acc + 0, to_fixed(c.x));
            atomicAdd(acc + 1, to_fixed(c.y));
            atomicAdd(acc + 2, to_fixed(c.z));
        }
    }
    if (COUNT) flush_counts(A, cnt);
}

// Finishes the pixels whose trees were split: fixed-point sum -> clamp -> gamma -> store.
__global__ __launch_bounds__(256) void finalize_spilled(KArgs A) {
    const uint32_t n = A.ctr->spilled;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t o = A.spilled[i];
        const unsigned long long* acc = A.acc + 4 * (size_t)o;
        const f3 c = mk(from_fixed(acc[0]), from_fixed(acc[1]), from_fixed(acc[2]));
        store_pixel(A, A.fr[0], o, mk(clamp01(c.x), clamp01(c.y), clamp01(c.z)));
    }
}

template <int CAP, bool COUNT, int GEOM>
static void launch_split(const KArgs& A0, hipStream_t stream, dim3 grid, dim3 block) {
    KArgs A = A0;
    const uint32_t D = A.max_depth, W = A.split_w;
    A.split_d1 = W;
    A.q_out = A.q_buf[0];
    A.q_out_n = &A.ctr->produced[0];
    hipLaunchKernelGGL((trace_kernel<CAP, COUNT, GEOM, true>), grid, block, 0, stream, A);
    uint32_t r = 1;
    for (uint32_t d0 = W; d0 < D && r <= kMaxSplitRounds; d0 += W, ++r) {
        A.split_d1 = d0 + W;
        A.q_in = A.q_buf[(r - 1) & 1];
        A.q_in_n = &A.ctr->produced[r - 1];
        A.q_in_head = &A.ctr->head[r - 1];
        A.q_out = A.q_buf[r & 1];
        A.q_out_n = &A.ctr->produced[r];
        // persistent: 3 one-wave workgroups per SIMD (the mesh kernels' occupancy; 4 for GEOM 3)
        hipLaunchKernelGGL((trace_tasks<CAP, COUNT, GEOM>), dim3(A.num_cus * (GEOM == 3 ? 4 * TRT_G3_WAVES : 12)), dim3(64), 0,
                           stream, A);
    }
    hipLaunchKernelGGL(finalize_spilled, dim3(A.num_cus), dim3(256), 0, stream, A);
}

// ---- deferred-shadow frame: passes B, C and the fallback ----------------------------------
//
// Pass B: the frame's shadow queries (shadow_intersect, shader.comp:364-399; any hit, so their
// order is free), 64 consecutive queries of one stripe per wave step — every lane of a wave
// runs a query, where in the per-pixel loop a wave runs the shadow rays of whichever of its
// lanes sit at a hit.  Static schedule: wave w takes stripe w % kDeferStripes and every
// (blocks per frame / kDeferStripes)-th 64-query block of it.  An occluded query ORs its
// light's bit into its event.  A launch of dframes frames gives each frame gridDim / dframes
// blocks (a multiple of kDeferStripes).
template <int GEOM>
__global__ __launch_bounds__(64, waves_per_simd<GEOM>()) void defer_shadows(KArgs A) {
    __shared__ float4 slab[slab_float4s<GEOM>()];
    Cnt cnt;
    const uint32_t F = max(A.dframes, 1u), per = gridDim.x / F;
    const bool inter = A.defer_inter > 1u && F > 1u; // frames block by block (pass A's dealing)
    const uint32_t f = inter ? blockIdx.x % F : blockIdx.x / per, b = inter ? blockIdx.x / F : blockIdx.x - f * per;
    const DScratch S = dscratch(A, f);
    const uint32_t s = b % kDeferStripes, K = per / kDeferStripes;
    const uint32_t n = min(S.dctr->nq[s * kCtrStride], A.shq_cap);
    const float4* Q = S.shq + 2 * (size_t)s * A.shq_cap;
    for (uint32_t base = (b / kDeferStripes) * 64u; base < n; base += K * 64u) {
        const uint32_t i = base + threadIdx.x;
        if (i < n) {
            const float4 a = Q[2 * (size_t)i], q = Q[2 * (size_t)i + 1];
            if (shadow_intersect<false, GEOM>(A, mk(a.x, a.y, a.z), mk(q.x, q.y, q.z), a.w, cnt, slab)) {
                const uint32_t t = __float_as_uint(q.w);
                atomicOr(reinterpret_cast<uint32_t*>(ev_plane(S.ev, t >> 2, 3)) + 1, 1u << (t & 3u));
            }
        }
    }
}

// Pass C: each pixel's event tree summed in the reference's pop order (shader.comp:530-575:
// a segment, then its reflection subtree, then its refraction subtree) with exactly cast_seg's
// arithmetic (a lit light's kd * diffuse / kd * specular terms added in light order, then
// colour += thr * (diffuse * albedo.x + specular * albedo.y)); then clamp, gamma and the dual
// store.  Lane = the pixel's lane in its pass-A tile; block f * ntiles + tile: frame f.
__global__ __launch_bounds__(64) void defer_resolve(KArgs A) {
    const uint32_t F = max(A.dframes, 1u), lane = threadIdx.x;
    uint32_t f, tile;
    if (A.defer_inter > 1u && F > 1u) {
        // pass A's dealing (trace_kernel): tile t of frame f on the XCD whose pass-A block traced
        // it (one pass-A wave per tile when a group runs), so its events are in that XCD's L2
        const uint32_t vb = blockIdx.x, per8 = A.ntiles & ~7u;
        uint32_t t;
        if (vb < F * per8) {
            const uint32_t j = vb >> 3;
            f = j % F;
            t = (j / F) * 8u + (((vb & 7u) + f) & 7u);
        } else {
            const uint32_t r = vb - F * per8, nl = A.ntiles - per8;
            f = r / nl;
            t = per8 + r % nl;
        }
        tile = xcd_tile(A, t);
    } else {
        f = blockIdx.x / A.ntiles;
        tile = blockIdx.x - f * A.ntiles;
    }
    const uint32_t x = (tile % A.ntx) * 8u + (lane & 7u);
    const uint32_t k = (tile / A.ntx) * 8u + (lane >> 3);
    if (x >= A.width || k >= A.rows) return;
    const DScratch S = dscratch(A, f);
    const size_t o = (size_t)k * A.width + x;
    const uint32_t root = S.px_ev[o].x;
    if (root == kEvNone) return; // defer_fallback's pixel
    f3 color = mk(0.0f, 0.0f, 0.0f);
    uint32_t stk[kMaxTreeDepth]; // pending refraction subtrees, one per depth of the path
    uint32_t s = root, sp = 0, steps = 0;
    for (;;) {
        // a tree has at most 2^MAX_DEPTH - 1 events: a corrupt log must not hang the GPU
        if (++steps > (1u << kMaxTreeDepth) || s >= A.ev_cap * kDeferStripes * kEvRows * 64u) {
            if (atomicCAS(&S.dctr->pad[0], 0u, 1u) == 0u) {
                uint32_t* d = S.dctr->pad;
                d[1] = (uint32_t)o; d[2] = root; d[3] = s; d[4] = sp; d[5] = steps;
            }
            color = mk(1.0f, 0.0f, 1.0f);
            break;
        }
        const float4 p0 = *ev_plane(S.ev, s, 0);
        const uint32_t tag = __float_as_uint(p0.w);
        const float4 p3 = *ev_plane(S.ev, s, 3);
        if (tag & kEvTagConst) {
            color = add(color, mk(p0.x, p0.y, p0.z));
        } else {
            const float4 p1 = *ev_plane(S.ev, s, 1), p2 = *ev_plane(S.ev, s, 2);
            const uint32_t lit = tag & 7u & ~__float_as_uint(p3.y);
            const f3 kdv = mk(p0.x, p0.y, p0.z);
            const float dterm[3] = {p1.x, p1.y, p1.z}, sterm[3] = {p2.x, p2.y, p2.z};
            f3 diffuse = mk(0.0f, 0.0f, 0.0f), specular = mk(0.0f, 0.0f, 0.0f);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                if (!((lit >> i) & 1u)) continue;
                diffuse = add(diffuse, muls(kdv, dterm[i]));
                specular = add(specular, muls(kdv, sterm[i]));
            }
            color = add(color, muls(add(muls(diffuse, p1.w), muls(specular, p2.w)), p3.x));
        }
        const uint32_t refl = __float_as_uint(p3.z), refr = __float_as_uint(p3.w);
        if (tag & kEvTagRefl) {
            if ((tag & kEvTagRefr) && sp < kMaxTreeDepth) stk[sp++] = refr;
            s = refl;
        } else if (tag & kEvTagRefr) {
            s = refr;
        } else if (sp > 0u) {
            s = stk[--sp];
        } else {
            break;
        }
    }
    store_pixel(A, A.fr[f], o, mk(clamp01(color.x), clamp01(color.y), clamp01(color.z)));
}

// Pixels whose log did not fit (event pool or query queue full) are traced again from scratch
// by the per-pixel loop with in-place shadow rays (persistent waves over the list).
template <int CAP, int GEOM>
__global__ __launch_bounds__(64, waves_per_simd<GEOM>()) void defer_fallback(KArgs A) {
    __shared__ float lds[lds_stack_floats<CAP, GEOM, false>()];
    __shared__ float4 slab[slab_float4s<GEOM>()];
    Cnt cnt;
    for (uint32_t f = 0; f < max(A.dframes, 1u); ++f) { // each frame of the launch, its list
        const DScratch S = dscratch(A, f);
        const uint32_t n = S.dctr->nfb;
        const f3 orig = mk(A.fr[f].cam[0], A.fr[f].cam[1], A.fr[f].cam[2]);
        for (uint32_t base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u) {
            const uint32_t i = base + threadIdx.x;
            if (i < n) {
                const uint32_t o = S.fb[i];
                const uint32_t k = o / A.width, x = o % A.width;
                const f3 c = cast_ray<CAP, false, GEOM>(A, orig, primary_dir(A, x, band_row(A, k), 0), cnt, lds, slab);
                store_pixel(A, A.fr[f], o, c);
            }
        }
    }
}

static uint32_t defer_stages() { // debug: TRT_DEFER_STAGES bitmask of passes to launch
    const char* e = getenv("TRT_DEFER_STAGES");
    return e ? (uint32_t)strtoul(e, nullptr, 0) : 0xFFu;
}


#ifndef TRT_DEFER_LDS
#define TRT_DEFER_LDS 3 /* deferred refraction children of a deep deferred frame kept in LDS */
#endif
template <int CAP, int GEOM, bool HYB>
static void launch_defer(const KArgs& A0, hipStream_t stream, dim3 grid, dim3 block) {
    KArgs A = A0;
    const uint32_t stages = defer_stages();
    const uint32_t D = A.max_depth, W = A.split_w, F = std::max(A.dframes, 1u);
    if (HYB && W >= 1 && W < D && A.ctr && A.q_link_buf[0]) {
        // subtree split: the tile kernel traces depths < W, each round the next window
        A.split_d1 = W;
        A.q_out = A.q_buf[0];
        A.q_link_out = A.q_link_buf[0];
        A.q_out_n = &A.ctr->produced[0];
        if (stages & 1) hipLaunchKernelGGL((trace_kernel<0, false, GEOM, true, true, false>), grid, block, 0, stream, A);
        uint32_t r = 1;
        for (uint32_t d0 = W; d0 < D && r <= kMaxSplitRounds && (stages & 2); d0 += W, ++r) {
            A.split_d1 = d0 + W;
            A.q_in = A.q_buf[(r - 1) & 1];
            A.q_link_in = A.q_link_buf[(r - 1) & 1];
            A.q_in_n = &A.ctr->produced[r - 1];
            A.q_in_head = &A.ctr->head[r - 1];
            A.q_out = A.q_buf[r & 1];
            A.q_link_out = A.q_link_buf[r & 1];
            A.q_out_n = &A.ctr->produced[r];
            hipLaunchKernelGGL((trace_tasks<0, false, GEOM, true>), dim3(A.num_cus * (GEOM == 3 ? 4 * TRT_G3_WAVES : 12)),
                               dim3(64), 0, stream, A);
        }
    } else {
        // dframes frames in one launch: ntiles * defer_sub blocks per frame
        const uint32_t S = A.defer_sub > 1u ? A.defer_sub : 1u;
        hipLaunchKernelGGL((trace_kernel<0, false, GEOM, false, true, false>), dim3(grid.x * S * F), block, 0, stream, A);
    }
    // persistent: up to 8 waves per SIMD (the shadow-only kernel is light on VGPRs and LDS;
    // waves that find the queue drained exit at once); a frame group shares the grid (each frame
    // a multiple of kDeferStripes blocks)
    if (stages & 4) {
        const uint32_t total = ((A.num_cus * 32 + kDeferStripes - 1) / kDeferStripes) * kDeferStripes;
        const uint32_t per = std::max(kDeferStripes, (total / F / kDeferStripes) * kDeferStripes);
        hipLaunchKernelGGL(defer_shadows<GEOM>, dim3(per * F), dim3(64), 0, stream, A);
    }
    if (stages & 8) hipLaunchKernelGGL(defer_resolve, dim3(A.ntiles * F), dim3(64), 0, stream, A);
    if (!(stages & 16)) return;
    // the fallback runs the per-pixel loop (deep frames: its full-depth private stack)
    if constexpr (HYB)
        hipLaunchKernelGGL((defer_fallback<(int)TRT_MAX_DEPTH_LIMIT - 1, GEOM>), dim3(A.num_cus), dim3(64), 0, stream, A);
    else
        hipLaunchKernelGGL((defer_fallback<CAP, GEOM>), dim3(A.num_cus), dim3(64), 0, stream, A);
}

// Batch of independent shadow queries (any hit, shader.comp:364-399): one lane per query of
// `rays` (2 float4 each: origin + max distance, direction), 64 consecutive queries per wave;
// occ[i] = 1 if query i is occluded.  The building block of a deferred-shadow frame and the
// diagnostic that prices coherent shadow tracing (tools/shadow_exp.py).
template <int GEOM>
__global__ __launch_bounds__(64, waves_per_simd<GEOM>()) void shadow_batch_kernel(KArgs A, const float4* __restrict__ rays,
                                                                                uint32_t n, uint32_t* __restrict__ occ) {
    __shared__ float4 slab[slab_float4s<GEOM>()];
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    const float4 a = rays[2 * (size_t)i], b = rays[2 * (size_t)i + 1];
    Cnt cnt;
    occ[i] = shadow_intersect<false, GEOM>(A, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), a.w, cnt, slab) ? 1u : 0u;
}

hipError_t launch_shadow_batch(const KArgs& A0, const float4* rays, uint32_t n, uint32_t* occ, hipStream_t stream) {
    KArgs A = A0;
    A.diag = nullptr;
    const int geom = A.nbatch == 0 ? 0 : (A.bvh && !(A.flags & TRT_FLAG_BATCH_WALK)) ? (A.bvh_waves4 ? 3 : 2) : 1;
    const dim3 grid((n + 63u) / 64u), block(64);
    if (!n) return hipSuccess;
    if (geom == 0) hipLaunchKernelGGL(shadow_batch_kernel<0>, grid, block, 0, stream, A, rays, n, occ);
    else if (geom == 1) hipLaunchKernelGGL(shadow_batch_kernel<1>, grid, block, 0, stream, A, rays, n, occ);
    else if (geom == 2) hipLaunchKernelGGL(shadow_batch_kernel<2>, grid, block, 0, stream, A, rays, n, occ);
    else hipLaunchKernelGGL(shadow_batch_kernel<3>, grid, block, 0, stream, A, rays, n, occ);
    return hipGetLastError();
}

// Launch helper: picks the deferred-stack capacity from max_depth (children are made only
// for depth+1 < max_depth, so at most max_depth-1 refraction children wait at once; inside a
// split window of w depths at most w - 1 do, so split launches keep w - 1 in LDS).  With a
// split window (A.split_w in [2, 5], spp == 1, max_depth > window) the frame is traced in
// depth windows: the tile kernel, one trace_tasks round per further window, finalize_spilled.
#ifdef TRT_KRES_ONLY
// tools/kres_quick.sh: compile only the kernels named by TRT_KRES_ONLY (register studies in a
// fraction of the full build's time; the library is not linkable from this object)
hipError_t launch_trace(const KArgs& A, hipStream_t stream, bool) {
    hipLaunchKernelGGL((TRT_KRES_ONLY), dim3(1), dim3(64), 0, stream, A);
    return hipGetLastError();
}
#else
hipError_t launch_trace(const KArgs& A, hipStream_t stream, bool count) {
    const uint32_t D = A.max_depth;
    const dim3 grid(A.ntiles), block(64);
    const int geom = A.nbatch == 0 ? 0 : (A.bvh && !(A.flags & TRT_FLAG_BATCH_WALK)) ? (A.bvh_waves4 ? 3 : 2) : 1;
    if (A.defer && !count && A.spp <= 1 && A.dctr && A.ev && A.shq && A.px_ev && A.fb) {
        hipError_t e = hipMemsetAsync(A.dctr, 0, sizeof(DeferCtr) * std::max(A.dframes, 1u), stream);
        if (e == hipSuccess && A.split_w >= 1 && A.ctr) e = hipMemsetAsync(A.ctr, 0, sizeof(SplitCtr), stream);
        if (e != hipSuccess) return e;
#define TRT_DEFER_G(CAP, HYB)                                                \
    do {                                                                     \
        if (geom == 0) launch_defer<CAP, 0, HYB>(A, stream, grid, block);    \
        else if (geom == 1) launch_defer<CAP, 1, HYB>(A, stream, grid, block); \
        else if (geom == 2) launch_defer<CAP, 2, HYB>(A, stream, grid, block); \
        else launch_defer<CAP, 3, HYB>(A, stream, grid, block);              \
    } while (0)
        // deep trees: TRT_DEFER_LDS deferred children in LDS + a private tail
        if (D <= 1) TRT_DEFER_G(0, false);
        else if (D <= 2) TRT_DEFER_G(1, false);
        else if (D <= 3) TRT_DEFER_G(2, false);
        else if (D <= 4) TRT_DEFER_G(3, false);
        else TRT_DEFER_G(TRT_DEFER_LDS, true);
#undef TRT_DEFER_G
        return hipGetLastError();
    }
    if (A.split_w >= 2 && A.split_w <= 5 && A.split_w < D && A.spp <= 1 && A.acc && A.ctr) {
        hipError_t e = hipMemsetAsync(A.ctr, 0, sizeof(SplitCtr), stream);
        if (e != hipSuccess) return e;
#define TRT_SPLIT_G(CAP, G)                                                 \
    do {                                                                    \
        if (count) launch_split<CAP, true, G>(A, stream, grid, block);            \
        else launch_split<CAP, false, G>(A, stream, grid, block);                 \
    } while (0)
#define TRT_SPLIT(CAP)                            \
    do {                                          \
        if (geom == 0) TRT_SPLIT_G(CAP, 0);       \
        else if (geom == 1) TRT_SPLIT_G(CAP, 1);  \
        else if (geom == 2) TRT_SPLIT_G(CAP, 2);  \
        else TRT_SPLIT_G(CAP, 3);                 \
    } while (0)
        switch (A.split_w) {
        case 2: TRT_SPLIT(1); break;
        case 3: TRT_SPLIT(2); break;
        case 4: TRT_SPLIT(3); break;
        default: TRT_SPLIT(4); break;
        }
#undef TRT_SPLIT
#undef TRT_SPLIT_G
        return hipGetLastError();
    }
    // a plain launch traces A.nframes frames: ntiles blocks per frame (frame-major)
    const uint32_t fblocks = A.spp_lanes ? std::max(A.nframes, 1u) * A.spp
                             : A.nframes > 1u && A.xcd_inter && A.frame_group > 1u && (geom == 0 || TRT_MESH_PAIRS)
                                 ? (A.nframes + 1u) / 2u
                                 : std::max(A.nframes, 1u);
    const dim3 fgrid(A.ntiles * fblocks);
#define TRT_LAUNCH_G(CAP, G)                                                                             \
    do {                                                                                                 \
        if (count) hipLaunchKernelGGL((trace_kernel<CAP, true, G, false>), fgrid, block, 0, stream, A);  \
        else hipLaunchKernelGGL((trace_kernel<CAP, false, G, false>), fgrid, block, 0, stream, A);       \
    } while (0)
#define TRT_LAUNCH(CAP)                          \
    do {                                         \
        if (geom == 0) TRT_LAUNCH_G(CAP, 0);     \
        else if (geom == 1) TRT_LAUNCH_G(CAP, 1); \
        else if (geom == 2) TRT_LAUNCH_G(CAP, 2); \
        else TRT_LAUNCH_G(CAP, 3);               \
    } while (0)
    if (D <= 1) TRT_LAUNCH(0);
    else if (D <= 2) TRT_LAUNCH(1);
    else if (D <= 3) TRT_LAUNCH(2);
    else if (D <= 4) TRT_LAUNCH(3);
    else if (D <= 5) TRT_LAUNCH(4);
    else if (D <= 8) TRT_LAUNCH(7);
    else TRT_LAUNCH(19);
#undef TRT_LAUNCH
#undef TRT_LAUNCH_G
    return hipGetLastError();
}
#endif

} // namespace trt

// ---- envmap pair rows (KArgs::envp) --------------------------------------------------------
namespace trt {

__global__ __launch_bounds__(256) void envp_kernel(const uint32_t* __restrict__ env, uint2* __restrict__ out,
                                                   uint32_t W, uint32_t H) {
    const uint32_t r = blockIdx.y, pw = W + 3u;
    const uint32_t y0 = r == 0u ? 0u : min(r - 1u, H - 1u), y1 = min(r, H - 1u);
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < pw; c += gridDim.x * blockDim.x) {
        const uint32_t x = c == 0u ? 0u : min(c - 1u, W - 1u);
        out[(size_t)r * pw + c] = make_uint2(env[(size_t)y0 * W + x], env[(size_t)y1 * W + x]);
    }
}

hipError_t launch_envp(const uint32_t* env, uint2* out, uint32_t W, uint32_t H, hipStream_t stream) {
    if (!W || !H) return hipSuccess;
    hipLaunchKernelGGL(envp_kernel, dim3((W + 3u + 255u) / 256u, H + 2u), dim3(256), 0, stream, env, out, W, H);
    return hipGetLastError();
}

} // namespace trt

// ---- multi-GPU frame assembly (trt_multi.cpp) ----------------------------------------------
//
// Re-interleaves the compact band-group buffers an exchange delivered to a root (the layout of
// band_plan.cpp / abi.h trt_band_plan): output row y of the root's frame f (0..J-1) belongs to
// band b = y / B, band group g = b % NG, compact row k = (b / NG) * B + y % B (trt_bands.h, the
// inverse of band_row above); group g = q * G + v of sender q sits at gather + (((q * J + f) *
// G + v) * max_rows + k) * W.  One 256-thread workgroup per output row; rows are copied as
// 16-byte vectors when aligned.
namespace trt {

__global__ __launch_bounds__(256) void interleave_kernel(const uint32_t* __restrict__ gather, uint32_t* __restrict__ out,
                                                         uint32_t W, uint32_t H, uint32_t B, uint32_t NG, uint32_t G,
                                                         uint32_t J, uint32_t max_rows, size_t stride_px, int vec4,
                                                         uint32_t skip_lo, uint32_t skip_hi) {
    const uint32_t f = blockIdx.x / H, y = blockIdx.x % H;
    uint32_t g, k;
    band_of_row(y, B, NG, g, k); // trt_bands.h
    if (g >= skip_lo && g < skip_hi) return; // the root's own groups, rendered in place
    const uint32_t q = g / G, v = g % G;
    const uint32_t* src = gather + ((size_t)((q * J + f) * G + v) * max_rows + k) * W;
    uint32_t* dst = out + (size_t)f * stride_px + (size_t)y * W;
    if (vec4) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (uint32_t i = threadIdx.x; i < W / 4u; i += blockDim.x) d4[i] = s4[i];
    } else {
        for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) dst[i] = src[i];
    }
}

hipError_t launch_interleave(const uint32_t* gather, uint32_t* out, uint32_t width, uint32_t height,
                             uint32_t band_rows, uint32_t groups, uint32_t groups_per_rank, uint32_t max_rows,
                             uint32_t nframes, size_t frame_stride_px, hipStream_t stream, uint32_t skip_lo,
                             uint32_t skip_hi) {
    if (skip_lo == 0 && skip_hi >= groups) return hipSuccess; // every group was rendered in place
    if (!width || !height || !nframes || !groups_per_rank) return hipSuccess;
    const int vec4 = (width % 4u == 0u) && ((reinterpret_cast<uintptr_t>(out) & 15u) == 0u) &&
                     (frame_stride_px % 4u == 0u) && ((reinterpret_cast<uintptr_t>(gather) & 15u) == 0u);
    hipLaunchKernelGGL(interleave_kernel, dim3(height * nframes), dim3(256), 0, stream, gather, out, width, height,
                       band_rows, groups, groups_per_rank, nframes, max_rows, frame_stride_px, vec4, skip_lo, skip_hi);
    return hipGetLastError();
}

} // namespace trt
