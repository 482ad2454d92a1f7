// trt_runtime.cpp — the C-ABI (include/trt/abi.h) over the HIP runtime.
//
// Replaces the reference's Vulkan compute plumbing: createShaderStorageBuffers() /
// createUniformBuffers() / the background texture upload (main.cpp:928-1111, 1494-1664)
// become trt_upload_scene(); updateUniformBuffer() (main.cpp:2165-2179) becomes
// trt_update_ubo(); recordComputeCommandBuffer() + vkQueueSubmit (main.cpp:2108-2131,
// 2181-2205) become trt_render().  No exception crosses the ABI; failures set the context's
// last error and return a negative TRT_ERR_* code (the reference throws std::runtime_error
// and exits, main.cpp:2565-2573).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "../../include/trt/abi.h"
#include "jpeg.h"
#include "trt_bands.h"
#include "trt_ctx.h"
#include "trt_device.h"

namespace trt {
// HIP creates a stream's hardware queue at its first submission, which costs ~0.1 ms: every
// stream the library creates gets a 4-byte fill of scratch memory (then a sync) right away, so
// that cost never lands in a frame loop.
hipError_t touch_stream(hipStream_t s, void* scratch) {
    hipError_t e = hipMemsetAsync(scratch, 0, 4, s);
    return e == hipSuccess ? hipStreamSynchronize(s) : e;
}
hipError_t launch_trace(const KArgs& A, hipStream_t stream, bool count);
hipError_t launch_envp(const uint32_t* env, uint2* out, uint32_t W, uint32_t H, hipStream_t stream);
hipError_t launch_shadow_batch(const KArgs& A, const float4* rays, uint32_t n, uint32_t* occ, hipStream_t stream);
uint32_t collapse_bvh4(const std::vector<BvhNode>& b2, std::vector<Bvh4Node>& b4);
uint32_t bvh_depth(const std::vector<BvhNode>& b2);
bool quantize_bvh4(const std::vector<Bvh4Node>& b4, std::vector<Bvh4QNode>& out);
bool build_bvh(const trt_triangle* tris, uint32_t ntri, const trt_model* models, uint32_t nmodel,
               std::vector<BvhNode>& nodes, std::vector<TriGeo>& leaf_tris);
}

using trt::BatchRec;
using trt::KArgs;
using trt::Mat;
using trt::TriGeo;
using trt::TriShade;


namespace {

int fail(trt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(trt_ctx* c, hipError_t e, const char* what) {
    // an allocation failure is reported through the return code; its sticky last-error state
    // must not surface in the caller's next HIP call (a torch launch check)
    if (e == hipErrorOutOfMemory) (void)hipGetLastError();
    return fail(c, e == hipErrorOutOfMemory ? TRT_ERR_OOM : TRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Failure injection (tests only, with TRT_ENABLE_TEST_HOOKS=1): TRT_TEST_FAIL_DEFER_SLOT=k makes
// the deferred-frame scratch allocation of in-flight slot k report out-of-memory.
int test_fail_defer_slot() {
    const char* on = std::getenv("TRT_ENABLE_TEST_HOOKS");
    const char* e = std::getenv("TRT_TEST_FAIL_DEFER_SLOT");
    return (on && std::atoi(on) == 1 && e) ? std::atoi(e) : -1;
}

#define HIP_TRY(ctx, expr)                                       \
    do {                                                         \
        hipError_t e_ = (expr);                                  \
        if (e_ != hipSuccess) return hip_fail((ctx), e_, #expr); \
    } while (0)

void free_scene(trt_ctx* c) {
    (void)hipFree(c->d_batches);
    (void)hipFree(c->d_nodes);
    (void)hipFree(c->d_bvh);
    (void)hipFree(c->d_bvh4);
    (void)hipFree(c->d_bvh4q);
    (void)hipFree(c->d_bvh_tris);
    (void)hipFree(c->d_geo);
    (void)hipFree(c->d_shade);
    (void)hipFree(c->d_mats);
    (void)hipFree(c->d_env);
    c->d_batches = nullptr;
    c->d_nodes = nullptr;
    c->d_bvh = nullptr;
    c->d_bvh4 = nullptr;
    c->d_bvh4q = nullptr;
    c->d_bvh_tris = nullptr;
    c->top = 0;
    c->d_geo = nullptr;
    c->d_shade = nullptr;
    c->d_mats = nullptr;
    c->d_env = nullptr;
    c->envp_ok = false;
    c->nbatch = c->ntri = c->nmat = c->env_w = c->env_h = 0;
    std::memset(c->scene_bytes, 0, sizeof(c->scene_bytes));
    c->have_scene = false;
}

// Grow-only device scratch buffer.
int ensure(trt_ctx* c, void** p, size_t* cap, size_t bytes, const char* what) {
    if (bytes <= *cap && *p) return TRT_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return hip_fail(c, e, what);
    *cap = bytes;
    return TRT_OK;
}

Mat to_mat(const trt_material& m) {
    Mat r{};
    r.albedo[0] = m.albedo.x;
    r.albedo[1] = m.albedo.y;
    r.albedo[2] = m.albedo.z;
    r.albedo[3] = m.albedo.w;
    r.kd[0] = m.diffuse_specular.x;
    r.kd[1] = m.diffuse_specular.y;
    r.kd[2] = m.diffuse_specular.z;
    r.spec_exp = m.diffuse_specular.w;
    r.ior = m.refractive.x;
    return r;
}

void fill_ubo_args(KArgs& A, const trt_ubo& u) {
    const trt_sphere* s[4] = {&u.sphere0, &u.sphere1, &u.sphere2, &u.sphere3};
    for (int i = 0; i < 4; ++i) {
        A.sph[i].c[0] = s[i]->center_radius.x;
        A.sph[i].c[1] = s[i]->center_radius.y;
        A.sph[i].c[2] = s[i]->center_radius.z;
        A.sph[i].r = s[i]->center_radius.w;
        A.sph[i].m = to_mat(s[i]->material);
    }
    const trt_vec4* l[3] = {&u.light0, &u.light1, &u.light2};
    for (int i = 0; i < 3; ++i) {
        A.light[i][0] = l[i]->x;
        A.light[i][1] = l[i]->y;
        A.light[i][2] = l[i]->z;
    }
}

void fill_frame(trt::FrameRec& f, const trt_ubo& u, uint8_t* out8, bool in_place) {
    f.cam[0] = u.camPos.x;
    f.cam[1] = u.camPos.y;
    f.cam[2] = u.camPos.z;
    f.in_place = in_place ? 1u : 0u;
    f.out8 = reinterpret_cast<uint32_t*>(out8);
}

// Frames that may share a launch: every UBO field but camPos equal (byte-wise).
bool same_but_camera(const trt_ubo& a, const trt_ubo& b) {
    constexpr size_t cam = offsetof(trt_ubo, camPos);
    return std::memcmp(&a, &b, cam) == 0 &&
           std::memcmp(reinterpret_cast<const char*>(&a) + cam + sizeof(trt_vec4),
                       reinterpret_cast<const char*>(&b) + cam + sizeof(trt_vec4),
                       sizeof(trt_ubo) - cam - sizeof(trt_vec4)) == 0;
}

} // namespace

extern "C" {

const char* trt_version(void) { return "trt-mi355x 0.2 (gfx950, abi 2)"; }

void trt_params_default(trt_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->width = 1024;  // main.cpp:35
    p->height = 768;  // main.cpp:36
    p->max_depth = 20; // shader.comp:75
    p->spp = 1;
    p->fov = 1.05f; // main.cpp:1498
    p->flags = TRT_FLAGS_REFERENCE;
}

uint32_t trt_output_rows(const trt_params* p) {
    if (!p) return 0;
    if (p->band_rows == 0 || p->band_count <= 1) return p->height;
    if (p->band_index >= p->band_count) return 0;
    return trt::band_group_rows(p->height, p->band_rows, p->band_count, p->band_index);
}

int trt_create(trt_ctx** out, int hip_device) {
    if (!out) return TRT_ERR_INVALID;
    *out = nullptr;
    trt_ctx* c = new (std::nothrow) trt_ctx();
    if (!c) return TRT_ERR_OOM;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0 || hip_device < 0 || hip_device >= n) {
        delete c;
        return TRT_ERR_HIP;
    }
    c->device = hip_device;
    if (hipSetDevice(hip_device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc((void**)&c->d_counters, 32 * sizeof(unsigned long long)) != hipSuccess) {
        trt_destroy(c);
        return TRT_ERR_HIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) == hipSuccess && prop.multiProcessorCount > 0)
        c->num_cus = (uint32_t)prop.multiProcessorCount;
    c->stream = c->own_stream;
    if (trt::touch_stream(c->own_stream, c->d_counters) != hipSuccess) {
        trt_destroy(c);
        return TRT_ERR_HIP;
    }
    if (const char* e = std::getenv("TRT_BVH_WAVES4")) c->bvh_waves4 = std::atoi(e) != 0 ? 1 : 0;
    if (const char* e = std::getenv("TRT_SPP_LANES")) c->spp_lanes = std::atoi(e) != 0;
    if (const char* e = std::getenv("TRT_DEFER_PPW")) { // pass-A pixels per wave: 64, 32, 16 or 8
        const int ppw = std::atoi(e);
        c->defer_sub = ppw == 8 ? 8u : ppw == 16 ? 4u : ppw == 32 ? 2u : ppw == 64 ? 1u : 0u;
    }
    if (const char* e = std::getenv("GPU_MAX_HW_QUEUES")) c->hw_queues = (uint32_t)std::max(1, std::atoi(e));
    if (const char* e = std::getenv("TRT_DEFER_INTER")) c->defer_inter = (uint32_t)std::min(2, std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("TRT_DEFER_GROUP"))
        c->defer_group = (uint32_t)std::min((int)trt::kMaxLaunchFrames, std::max(1, std::atoi(e)));
    if (const char* e = std::getenv("TRT_DEFER_IN_FLIGHT")) {
        c->defer_in_flight = (uint32_t)std::min((int)TRT_BUILD_MAX_IN_FLIGHT, std::max(1, std::atoi(e)));
        c->defer_in_flight_set = true;
    }
    if (const char* e = std::getenv("TRT_XCD_ROT")) c->xcd_rot = (uint32_t)std::min(8, std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("TRT_XCD_SKEW")) c->xcd_skew = (uint32_t)std::min(7, std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("TRT_XCD_INTER")) c->xcd_inter = (uint32_t)std::min(2, std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("TRT_FRAME_GROUP")) c->frame_group = std::min(2, std::max(1, std::atoi(e)));
    *out = c;
    return TRT_OK;
}

int trt_destroy(trt_ctx* c) {
    if (!c) return TRT_ERR_INVALID;
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    if (c->stream && c->stream != c->own_stream) (void)hipStreamSynchronize(c->stream);
    // frames of earlier trt_render calls may still run on other streams (render_slot): every
    // buffer below may be in use until the device drains
    (void)hipDeviceSynchronize();
    free_scene(c);
    (void)hipFree(c->d_envp);
    (void)hipFree(c->d_out8);
    (void)hipFree(c->d_out32);
    (void)hipFree(c->d_rays);
    (void)hipFree(c->d_counters);
    for (hipEvent_t e : c->fev) (void)hipEventDestroy(e);
    for (auto& b : c->split) {
        (void)hipFree(b.q[0]);
        (void)hipFree(b.q[1]);
        (void)hipFree(b.qlink[0]);
        (void)hipFree(b.qlink[1]);
        (void)hipFree(b.acc);
        (void)hipFree(b.spilled);
        (void)hipFree(b.ctr);
        (void)hipFree(b.ev);
        (void)hipFree(b.shq);
        (void)hipFree(b.px_ev);
        (void)hipFree(b.fb);
        (void)hipFree(b.dctr);
        if (b.done) (void)hipEventDestroy(b.done);
    }
    for (hipStream_t s : c->aux) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
    for (hipEvent_t e : c->aux_ev) (void)hipEventDestroy(e);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return TRT_OK;
}

const char* trt_last_error(const trt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int trt_set_stream(trt_ctx* c, void* s) {
    if (!c) return TRT_ERR_INVALID;
    c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own_stream;
    return TRT_OK;
}

int trt_set_frames_in_flight(trt_ctx* c, uint32_t n) {
    if (!c) return TRT_ERR_INVALID;
    if (n > TRT_BUILD_MAX_IN_FLIGHT)
        return fail(c, TRT_ERR_INVALID, "trt_set_frames_in_flight: n must be 0 (auto) or in [1, TRT_MAX_FRAMES_IN_FLIGHT]");
    c->frames_in_flight = n;
    return TRT_OK;
}

int trt_set_subtree_split(trt_ctx* c, int window) {
    if (!c) return TRT_ERR_INVALID;
    if (window != TRT_SPLIT_AUTO && window != TRT_SPLIT_OFF && (window < 2 || window > 5))
        return fail(c, TRT_ERR_INVALID, "trt_set_subtree_split: window must be 0 (auto), 1 (off) or 2..5");
    c->subtree_split = window;
    return TRT_OK;
}

int trt_set_deferred_shadows(trt_ctx* c, int mode) {
    if (!c) return TRT_ERR_INVALID;
    if (mode != TRT_DEFER_AUTO && mode != TRT_DEFER_OFF && mode != TRT_DEFER_ON)
        return fail(c, TRT_ERR_INVALID, "trt_set_deferred_shadows: mode must be TRT_DEFER_AUTO, _OFF or _ON");
    c->deferred_shadows = mode;
    return TRT_OK;
}

int trt_defer_stats(trt_ctx* c, uint32_t slot, uint64_t out[5]) {
    if (!c || !out) return TRT_ERR_INVALID;
    if (slot >= TRT_BUILD_MAX_IN_FLIGHT) return fail(c, TRT_ERR_INVALID, "trt_defer_stats: slot out of range");
    const auto& b = c->split[slot];
    for (int i = 0; i < 5; ++i) out[i] = 0;
    if (!b.dctr) return TRT_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (b.last && b.done) HIP_TRY(c, hipEventSynchronize(b.done));
    trt::DeferCtr d{};
    HIP_TRY(c, hipMemcpy(&d, b.dctr, sizeof(d), hipMemcpyDeviceToHost));
    // taken = min(requested, the stripe capacity the slot's last frame ran with: its own size or
    // a test hook's, not the slot's allocation, which may be larger)
    const size_t ev_s = b.used_ev_cap, q_s = b.used_shq_cap;
    for (uint32_t s = 0; s < trt::kDeferStripes; ++s) {
        out[0] += std::min<size_t>(d.chunks[s * trt::kCtrStride], ev_s);
        out[1] += std::min<size_t>(d.nq[s * trt::kCtrStride], q_s);
    }
    out[2] = d.nfb;
    out[3] = b.ev_chunks;
    out[4] = b.shq_cap;
    return TRT_OK;
}

int trt_synchronize(trt_ctx* c) {
    if (!c) return TRT_ERR_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return TRT_OK;
}

int trt_update_ubo(trt_ctx* c, const trt_ubo* ubo) {
    if (!c || !ubo) return fail(c, TRT_ERR_INVALID, "trt_update_ubo: null argument");
    c->ubo = *ubo;
    return TRT_OK;
}

int trt_upload_scene(trt_ctx* c, const trt_ubo* ubo, const trt_triangle* tris, uint32_t ntri,
                     const trt_model* models, uint32_t nmodel, const uint8_t* env,
                     uint32_t env_w, uint32_t env_h) {
    if (!c) return TRT_ERR_INVALID;
    if (!ubo) return fail(c, TRT_ERR_INVALID, "trt_upload_scene: null ubo");
    if (ntri && !tris) return fail(c, TRT_ERR_INVALID, "trt_upload_scene: null triangles");
    if (nmodel && !models) return fail(c, TRT_ERR_INVALID, "trt_upload_scene: null models");
    if (env && (env_w == 0 || env_h == 0))
        return fail(c, TRT_ERR_INVALID, "trt_upload_scene: zero-size envmap");
    for (uint32_t i = 0; i < nmodel; ++i) {
        const int64_t s = models[i].params0.x, n = models[i].params0.y;
        if (s < 0 || n < 0 || s + n > (int64_t)ntri)
            return fail(c, TRT_ERR_INVALID,
                        "trt_upload_scene: model " + std::to_string(i) +
                            " triangle range outside the triangle buffer");
    }
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    free_scene(c);

    // Repack binding 6 (Model) and binding 5 (Triangle) for the wave-uniform walks.
    std::vector<BatchRec> batches(nmodel);
    for (uint32_t i = 0; i < nmodel; ++i) {
        const trt_model& m = models[i];
        BatchRec& b = batches[i];
        b.bmin[0] = m.bboxMin.x;
        b.bmin[1] = m.bboxMin.y;
        b.bmin[2] = m.bboxMin.z;
        b.bmax[0] = m.bboxMax.x;
        b.bmax[1] = m.bboxMax.y;
        b.bmax[2] = m.bboxMax.z;
        b.start = m.params0.x;
        b.count_ni = (m.params0.y & 0x7fffffff) | (m.params0.z != 0 ? (int32_t)0x80000000 : 0);
    }
    // Implicit 8-ary range hierarchy: node k of level L is the exact union of the boxes of
    // batches [k*8^L, (k+1)*8^L).  A NaN coordinate anywhere below makes the node infinite
    // (always entered), so culling stays conservative for degenerate input.
    std::vector<float4> nodes;
    uint32_t node_off[11] = {0};
    uint32_t top = 0;
    while (top < 10 && (1ull << (3 * top)) < (unsigned long long)nmodel) ++top;
    {
        std::vector<float4> prev_lo(nmodel), prev_hi(nmodel);
        for (uint32_t i = 0; i < nmodel; ++i) {
            const BatchRec& b = batches[i];
            prev_lo[i] = make_float4(b.bmin[0], b.bmin[1], b.bmin[2], 0.0f);
            prev_hi[i] = make_float4(b.bmax[0], b.bmax[1], b.bmax[2], 0.0f);
        }
        const float inf = std::numeric_limits<float>::infinity();
        for (uint32_t L = 1; L <= top; ++L) {
            const size_t n = (prev_lo.size() + 7) / 8;
            node_off[L] = (uint32_t)(nodes.size() / 2);
            std::vector<float4> lo(n), hi(n);
            for (size_t k = 0; k < n; ++k) {
                float4 a = make_float4(inf, inf, inf, 0.0f), z = make_float4(-inf, -inf, -inf, 0.0f);
                bool bad = false;
                for (size_t j = 8 * k; j < std::min(prev_lo.size(), 8 * k + 8); ++j) {
                    const float4 &l = prev_lo[j], &h = prev_hi[j];
                    bad |= std::isnan(l.x) || std::isnan(l.y) || std::isnan(l.z) || std::isnan(h.x) ||
                           std::isnan(h.y) || std::isnan(h.z);
                    a.x = std::min(a.x, l.x); a.y = std::min(a.y, l.y); a.z = std::min(a.z, l.z);
                    z.x = std::max(z.x, h.x); z.y = std::max(z.y, h.y); z.z = std::max(z.z, h.z);
                }
                if (bad) {
                    a = make_float4(-inf, -inf, -inf, 0.0f);
                    z = make_float4(inf, inf, inf, 0.0f);
                }
                lo[k] = a;
                hi[k] = z;
                nodes.push_back(a);
                nodes.push_back(z);
            }
            prev_lo.swap(lo);
            prev_hi.swap(hi);
        }
    }
    std::vector<TriGeo> geo(ntri);
    std::vector<TriShade> shade(ntri);
    std::vector<Mat> mats;
    std::map<std::string, uint32_t> mat_index;
    for (uint32_t j = 0; j < ntri; ++j) {
        const trt_triangle& t = tris[j];
        TriGeo& g = geo[j];
        g.v0[0] = t.v0.x;
        g.v0[1] = t.v0.y;
        g.v0[2] = t.v0.z;
        // edge1 = v1 - v0, edge2 = v2 - v0 (shader.comp:230-231): same float subtraction
        g.e1[0] = t.v1.x - t.v0.x;
        g.e1[1] = t.v1.y - t.v0.y;
        g.e1[2] = t.v1.z - t.v0.z;
        g.e2[0] = t.v2.x - t.v0.x;
        g.e2[1] = t.v2.y - t.v0.y;
        g.e2[2] = t.v2.z - t.v0.z;
        g.pad[0] = g.pad[1] = g.pad[2] = 0.0f;
        TriShade& s = shade[j];
        s.n0[0] = t.v0_norm.x;
        s.n0[1] = t.v0_norm.y;
        s.n0[2] = t.v0_norm.z;
        s.n1[0] = t.v1_norm.x;
        s.n1[1] = t.v1_norm.y;
        s.n1[2] = t.v1_norm.z;
        s.n2[0] = t.v2_norm.x;
        s.n2[1] = t.v2_norm.y;
        s.n2[2] = t.v2_norm.z;
        std::string key(reinterpret_cast<const char*>(&t.material), sizeof(trt_material));
        auto it = mat_index.find(key);
        if (it == mat_index.end()) {
            it = mat_index.emplace(key, (uint32_t)mats.size()).first;
            mats.push_back(to_mat(t.material));
        }
        s.material = it->second;
        s.pad[0] = s.pad[1] = 0;
    }
    if (mats.empty()) mats.push_back(Mat{});

    auto upload = [&](void** dst, const void* src, size_t bytes, const char* what) -> int {
        if (bytes == 0) bytes = 16; // never bind a null buffer
        hipError_t e = hipMalloc(dst, bytes);
        if (e != hipSuccess) return hip_fail(c, e, what);
        if (src) {
            e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
            if (e != hipSuccess) return hip_fail(c, e, what);
        }
        return TRT_OK;
    };
    int rc;
    if ((rc = upload((void**)&c->d_batches, nmodel ? batches.data() : nullptr,
                     sizeof(BatchRec) * nmodel, "upload batches")) != TRT_OK ||
        (rc = upload((void**)&c->d_geo, ntri ? geo.data() : nullptr, sizeof(TriGeo) * ntri,
                     "upload triangle geometry")) != TRT_OK ||
        (rc = upload((void**)&c->d_shade, ntri ? shade.data() : nullptr, sizeof(TriShade) * ntri,
                     "upload triangle shading")) != TRT_OK ||
        (rc = upload((void**)&c->d_mats, mats.data(), sizeof(Mat) * mats.size(),
                     "upload materials")) != TRT_OK ||
        (rc = upload((void**)&c->d_nodes, nodes.empty() ? nullptr : nodes.data(), sizeof(float4) * nodes.size(),
                     "upload batch hierarchy")) != TRT_OK) {
        free_scene(c);
        return rc;
    }
    std::vector<trt::BvhNode> bvh;
    std::vector<TriGeo> bvh_tris;
    size_t bvh4_n = 0;
    if (nmodel && trt::build_bvh(tris, ntri, models, nmodel, bvh, bvh_tris)) {
        std::vector<trt::Bvh4Node> bvh4;
        // the 4-wide walk only when its worst-case stack fits (else the BVH2 walk: <= depth)
        if (trt::collapse_bvh4(bvh, bvh4) > (uint32_t)trt::kBvhStack) bvh4.clear();
        bvh4_n = bvh4.size();
        std::vector<trt::Bvh4QNode> bvh4q;
        const bool quant = !bvh4.empty() && trt::quantize_bvh4(bvh4, bvh4q);
        if (quant && (rc = upload((void**)&c->d_bvh4q, bvh4q.data(), sizeof(trt::Bvh4QNode) * bvh4q.size(),
                                  "upload quantized bvh4")) != TRT_OK) {
            free_scene(c);
            return rc;
        }
        if ((rc = upload((void**)&c->d_bvh, bvh.data(), sizeof(trt::BvhNode) * bvh.size(), "upload bvh")) != TRT_OK ||
            (!bvh4.empty() && (rc = upload((void**)&c->d_bvh4, bvh4.data(), sizeof(trt::Bvh4Node) * bvh4.size(),
                                            "upload bvh4")) != TRT_OK) ||
            (rc = upload((void**)&c->d_bvh_tris, bvh_tris.data(), sizeof(TriGeo) * bvh_tris.size(),
                         "upload bvh triangles")) != TRT_OK) {
            free_scene(c);
            return rc;
        }
    }
    if (env) {
        if ((rc = upload((void**)&c->d_env, env, (size_t)env_w * env_h * 4, "upload envmap")) != TRT_OK) {
            free_scene(c);
            return rc;
        }
        c->env_w = env_w;
        c->env_h = env_h;
    }
    size_t* sb = c->scene_bytes;
    std::memset(sb, 0, sizeof(c->scene_bytes));
    sb[trt::kSceneBatches] = std::max<size_t>(sizeof(BatchRec) * nmodel, 16);
    sb[trt::kSceneNodes] = std::max<size_t>(sizeof(float4) * nodes.size(), 16);
    sb[trt::kSceneGeo] = std::max<size_t>(sizeof(TriGeo) * ntri, 16);
    sb[trt::kSceneShade] = std::max<size_t>(sizeof(TriShade) * ntri, 16);
    sb[trt::kSceneMats] = sizeof(Mat) * mats.size();
    if (c->d_bvh) {
        sb[trt::kSceneBvh] = sizeof(trt::BvhNode) * bvh.size();
        sb[trt::kSceneBvhTris] = sizeof(TriGeo) * bvh_tris.size();
    }
    if (c->d_bvh4) sb[trt::kSceneBvh4] = sizeof(trt::Bvh4Node) * bvh4_n;
    if (c->d_bvh4q) sb[trt::kSceneBvh4Q] = sizeof(trt::Bvh4QNode) * bvh4_n;
    if (c->d_env) sb[trt::kSceneEnv] = (size_t)env_w * env_h * 4;
    c->nbatch = nmodel;
    c->top = top;
    std::memcpy(c->node_off, node_off, sizeof(node_off));
    c->ntri = ntri;
    c->nmat = (uint32_t)mats.size();
    c->ubo = *ubo;
    c->have_scene = true;
    return TRT_OK;
}

} // extern "C"

namespace {

// Builds the envmap pair rows (KArgs::envp) on `stream` when d_env changed since the last
// build.  Without them (TRT_ENV_PAIRROWS=0 in the environment) env_fetch reads d_env directly.
int ensure_envp(trt_ctx* c, const trt_params* p, hipStream_t stream) {
    if (!(p->flags & TRT_FLAG_ENVMAP) || !c->d_env || c->envp_ok) return TRT_OK;
    if (const char* e = std::getenv("TRT_ENV_PAIRROWS"))
        if (std::atoi(e) == 0) return TRT_OK;
    const size_t bytes = ((size_t)c->env_h + 2) * ((size_t)c->env_w + 3) * sizeof(uint2);
    if (bytes > c->envp_cap) {
        HIP_TRY(c, hipStreamSynchronize(stream));
        (void)hipFree(c->d_envp);
        c->d_envp = nullptr;
        c->envp_cap = 0;
        HIP_TRY(c, hipMalloc((void**)&c->d_envp, bytes));
        c->envp_cap = bytes;
    }
    HIP_TRY(c, trt::launch_envp(c->d_env, c->d_envp, c->env_w, c->env_h, stream));
    // once per envmap upload: wait for the build, since later frames may run on streams not
    // ordered after `stream` (trt_multi's two batch slots fork before the first batch builds)
    HIP_TRY(c, hipStreamSynchronize(stream));
    c->envp_ok = true;
    return TRT_OK;
}

int check_params(trt_ctx* c, const trt_params* p) {
    if (!p) return fail(c, TRT_ERR_INVALID, "trt_render: null params");
    if (!c->have_scene) return fail(c, TRT_ERR_NOSCENE, "trt_render: no scene uploaded");
    if (p->width == 0 || p->height == 0 || p->width > 65536 || p->height > 65536)
        return fail(c, TRT_ERR_INVALID, "trt_render: image size out of range");
    if (p->max_depth < 1 || p->max_depth > TRT_MAX_DEPTH_LIMIT)
        return fail(c, TRT_ERR_INVALID, "trt_render: max_depth must be 1..20");
    if (p->spp > 4096) return fail(c, TRT_ERR_INVALID, "trt_render: spp must be <= 4096");
    if (p->band_rows && p->band_count > 1 && p->band_index >= p->band_count)
        return fail(c, TRT_ERR_INVALID, "trt_render: band_index >= band_count");
    if ((p->flags & TRT_FLAG_BAND_IN_PLACE) && !(p->flags & TRT_FLAG_DEVICE_PTRS))
        return fail(c, TRT_ERR_INVALID, "trt_render: TRT_FLAG_BAND_IN_PLACE needs TRT_FLAG_DEVICE_PTRS");
    if ((p->flags & TRT_FLAG_ENVMAP) && !c->d_env)
        return fail(c, TRT_ERR_INVALID, "trt_render: TRT_FLAG_ENVMAP without an uploaded envmap");
    return TRT_OK;
}

// Everything of KArgs that does not depend on the UBO or the output pointers.
void fill_args(trt_ctx* c, const trt_params* p, KArgs& A) {
    std::memset(&A, 0, sizeof(A));
    A.width = p->width;
    A.height = p->height;
    A.rows = trt_output_rows(p);
    A.band_rows = p->band_rows;
    A.band_count = p->band_count;
    A.band_index = p->band_index;
    A.max_depth = p->max_depth;
    A.spp = p->spp ? p->spp : 1;
    // spp a power of two in [2, 64] and no replayed rays: one lane per sample (trace_samples;
    // TRT_SPP_LANES=0 keeps the per-pixel sample loop)
    A.spp_lanes = (A.spp >= 2u && A.spp <= 64u && (A.spp & (A.spp - 1u)) == 0u && !p->rays_in && c->spp_lanes) ? 1u : 0u;
    A.seed = p->seed;
    A.flags = p->flags;
    // dir_z = -1.0 * (HEIGHT / (2.0 * tan(fov / 2.0))) in double, main.cpp:1503
    A.dz = (float)(-1.0 * ((double)p->height / (2.0 * std::tan((double)p->fov / 2.0))));
    A.nbatch = c->nbatch;
    fill_ubo_args(A, c->ubo);
    A.nframes = 1;
    fill_frame(A.fr[0], c->ubo, nullptr, (p->flags & TRT_FLAG_BAND_IN_PLACE) != 0);
    A.batches = c->d_batches;
    A.geo = c->d_geo;
    A.shade = c->d_shade;
    A.mats = c->d_mats;
    A.env = c->d_env;
    A.envp = c->envp_ok ? c->d_envp : nullptr;
    A.env_w = c->env_w;
    A.env_h = c->env_h;
    A.counters = c->d_counters;
    A.nodes = c->d_nodes;
    A.bvh = c->d_bvh;
    A.bvh4 = c->d_bvh4;
    A.bvh4q = c->d_bvh4q;
    A.diag = reinterpret_cast<float4*>(c->diag);
    A.bvh_tris = c->d_bvh_tris;
    A.top = c->top;
    std::memcpy(A.node_off, c->node_off, sizeof(A.node_off));
    A.ntx = (A.width + 7u) / 8u;
    A.ntiles = A.ntx * ((A.rows + 7u) / 8u);
    // The BVH walk at 4 waves per SIMD (GEOM 3: <= 128 VGPRs, 16-entry LDS stack, quantized
    // nodes) hides more of the node-fetch latency than the 3-wave build.  Round 1 measured it
    // for large scenes only (C4 -13 %, C3 / shipped frame +1 %, profiles/r01_ab_occupancy.log);
    // since the traversal stack's index left scratch memory (round 3) it is ahead or equal
    // everywhere: C4 2.90 vs 3.38 ms, C3 -9 %, shipped frame and README scene within 1 %
    // (profiles/r03_ab_waves4_after_stack_fix.log), so it is the default for every BVH scene.
    // GEOM 3 kernels walk only the quantized nodes (trt_kernel.hip g3_quant_only): a scene whose
    // nodes did not quantize (or whose 4-wide stack would not fit) takes the GEOM 2 kernels.
    A.bvh_waves4 = c->d_bvh4q ? (c->bvh_waves4 >= 0 ? (uint32_t)c->bvh_waves4 : 1u) : 0u;
    A.xcd_rot = c->xcd_rot;
    A.xcd_skew = c->xcd_skew;
    A.xcd_inter = c->xcd_inter;
    {   // xcd_inter 2: a multiplier near 0.618 of the dealt chunk count, coprime to it (a
        // golden-ratio step spreads each XCD's chunks evenly over the image)
        const uint32_t tyn = (A.rows + 7u) / 8u;
        const uint32_t nfull = ((A.ntx / 2u) * (tyn / 2u) / 8u) * 8u;
        uint32_t m = nfull ? (uint32_t)(0.6180339887 * nfull) | 1u : 1u;
        auto gcd = [](uint32_t a, uint32_t b) { while (b) { const uint32_t t = a % b; a = b; b = t; } return a; };
        while (nfull && gcd(m, nfull) != 1u) m += 2u;
        A.xcd_mult = nfull ? m % nfull : 1u;
        if (A.xcd_mult == 0u || nfull >= 65536u) A.xcd_mult = 1u; // the kernel's k * mult stays in 32 bits
    }
    // Frame groups (trace_kernel): triangle-free frames (C2) 14.8 -> 13.85 us per frame at
    // 20-frame launches with pairs; mesh frames lose (C4 +2.5 %, C3 +10 %: their tiles' costs
    // vary more from frame to frame and a pair doubles the longest wave),
    // profiles/r03_ab_frame_pair.log
    A.frame_group = c->frame_group > 0 ? (uint32_t)c->frame_group : (c->nbatch == 0 ? 2u : 1u);
}

// Does this frame run deferred shadows?  Auto: mesh scenes with max_depth >= 8, whose deep
// refraction trees leave most lanes of a wave idle while a few trace their shadow rays.
// COUNT frames (the reference's counters) and spp > 1 frames run the per-pixel loop.
bool defer_frame(const trt_ctx* c, const trt_params* p, bool ignore_count = false) {
    if (p->spp > 1 || c->deferred_shadows == TRT_DEFER_OFF) return false;
    if ((p->flags & TRT_FLAG_COUNT) && !ignore_count) return false;
    if (c->deferred_shadows == TRT_DEFER_ON) return true;
    return c->nbatch > 0 && p->max_depth >= 8;
}

// The subtree-split window of a frame: 0 = off.  Auto: scenes with meshes (whose deep
// refraction trees make a few tiles run for milliseconds) with max_depth above the window.
uint32_t split_window(const trt_ctx* c, const trt_params* p) {
    const uint32_t D = p->max_depth;
    if ((p->spp > 1) || c->subtree_split == TRT_SPLIT_OFF) return 0;
    if ((size_t)trt_output_rows(p) * p->width >= (1u << (32 - trt::kTaskDepthBits))) return 0;
    uint32_t w;
    // experiment: a deferred frame traced one depth per launch (TRT_DEFER_WAVEFRONT=1)
    if (const char* e = std::getenv("TRT_DEFER_WAVEFRONT"))
        if (std::atoi(e) != 0 && defer_frame(c, p) && D > 1) return 1u;
    if (c->subtree_split == TRT_SPLIT_AUTO) {
        // measured (profiles/r01_split_sweep.log): -10..-16 % on the shipped depth-20 frame with
        // w = 4; +0..+25 % on depth-4 mesh frames (C3/C4) for any window, so only deep trees.
        // Deferred-shadow frames are not split: their trees hold no shadow rays, and a split
        // (exact, through LINK events) measured +11..+29 % on the shipped frame and +38..+69 %
        // on the README scene for windows 2..5 (profiles/r02_ab_defer_split.log).
        if (c->nbatch == 0 || D < 8 || defer_frame(c, p)) return 0;
        w = 4u;
    } else {
        w = (uint32_t)c->subtree_split;
    }
    return w < D ? w : 0u;
}

size_t env_cap(const char* name, size_t v) {
    if (const char* e = std::getenv(name)) return std::min<size_t>(v, (size_t)std::strtoull(e, nullptr, 10));
    return v;
}

// ---- deferred-frame scratch (one set per frames-in-flight slot) ----------------------------

// Deferred-frame sizes: event chunks (per tile:
// ceil((2^D - 1) / kEvRows) at depth <= 4, else 4 on average, at least 128 per stripe) and
// shadow queries (6 per pixel on average), both split into kDeferStripes equal stripes (tile t
// uses stripe hash(t)); ~1.2 KB per pixel at depth >= 5 (16 events of 64 B + 6 queries of 32 B).
// Every lane of a pool wave takes an event slot on every step of the wave's shared segment pool
// (idle lanes too, so the lanes stay on one row of one chunk), so a tile's event count is set by
// the pool's schedule, not bounded by 2^D - 1 per pixel; a tile that runs out re-traces its
// pixels in place (defer_fallback: the image stays exact, only slower).  Slot ids
// (chunk * kEvRows + row) * 64 + lane travel in 30 bits of a query.
constexpr size_t kPoolEvBytes = trt::kEvRows * 4 * 64 * sizeof(float4); // one chunk
size_t pool_chunks(size_t ntiles, uint32_t D) {
    const size_t per_tile = D <= 4 ? ((1u << D) - 1u + trt::kEvRows - 1u) / trt::kEvRows : 4u;
    constexpr size_t S = trt::kDeferStripes;
    const size_t tiles_per_stripe = (ntiles + S - 1) / S;
    return S * std::min<size_t>(std::max<size_t>(tiles_per_stripe * per_tile, D <= 4 ? 16u : 128u),
                                (1u << 30) / (trt::kEvRows * 64u) / S);
}
size_t shadow_qcap(size_t ntiles) {
    constexpr size_t S = trt::kDeferStripes;
    const size_t tiles_per_stripe = (ntiles + S - 1) / S;
    return S * std::min<size_t>(std::max<size_t>(6 * tiles_per_stripe * 64u, 1u << 12), 0xFFFFFFFFu / S);
}
struct DeferSizes {
    size_t chunks = 0, qcap = 0; // event chunks and shadow queries
    size_t bytes = 0;
};
DeferSizes defer_sizes(size_t ntiles, uint32_t D, size_t npx) {
    DeferSizes z;
    z.chunks = pool_chunks(ntiles, D);
    z.qcap = shadow_qcap(ntiles);
    z.bytes = z.chunks * kPoolEvBytes + z.qcap * 2 * sizeof(float4) + npx * (sizeof(uint2) + sizeof(uint32_t)) +
              sizeof(trt::DeferCtr);
    return z;
}

// A slot holds the scratch of `dframes` frames (a deferred launch group), each of the per-frame
// capacities below.
bool defer_bufs_fit(const trt_ctx::SplitBufs& b, const DeferSizes& z, size_t npx, uint32_t frames) {
    return z.chunks <= b.ev_chunks && z.qcap <= b.shq_cap && npx <= b.dnpx && frames <= b.dframes;
}

// Deferred frame loop shape: `group` frames per launch sequence on each of `slots` in-flight
// slots.  Explicit: TRT_DEFER_GROUP, or trt_set_frames_in_flight (then groups of 1, the
// reference's pacing when it is 2).  Auto, with the group's frames dealt block by block
// (defer_inter): with at least 16 hardware queues 8 slots of 3 frames (24 in flight: the shipped
// frame 320 -> 311 us, the README scene 155 -> 149 us against 16 slots of 1, at half the frame
// latency; profiles/r06t_ab_defer_shape_32q.jsonl); with fewer, defer_in_flight (16) frames over
// at most half the queues — a stream per slot, and slots sharing a queue serialise: with HIP's
// default 4 queues 2 slots of 8 frames (the shipped frame through the C++ host 0.82 -> 0.51 ms
// per frame; 2 x 12 and 6 x 4 within 2 %, profiles/r06t_shape_q4.log).  An explicit
// TRT_DEFER_IN_FLIGHT keeps the second rule at every queue count.
void defer_shape(const trt_ctx* c, uint32_t& group, uint32_t& slots) {
    const uint32_t T = std::max(c->defer_in_flight, 1u);
    if (c->frames_in_flight) {
        slots = c->frames_in_flight;
        group = c->defer_group ? c->defer_group : 1u;
        return;
    }
    if (c->defer_group) {
        group = c->defer_group;
        slots = std::max(1u, (T + group - 1) / group);
        return;
    }
    if (c->hw_queues >= 16u && !c->defer_in_flight_set) {
        slots = 8u;
        group = 3u;
        return;
    }
    slots = std::min(T, std::max(2u, c->hw_queues / 2u));
    group = (T + slots - 1) / slots;
}

// Device bytes one frames-in-flight slot needs for a group of `frames` deferred frames of these
// params (0 when the slot already holds enough).
size_t defer_slot_bytes(const trt_ctx* c, const trt_params* p, uint32_t slot, uint32_t frames) {
    const size_t npx = (size_t)trt_output_rows(p) * p->width;
    const size_t ntiles = ((p->width + 7u) / 8u) * ((trt_output_rows(p) + 7u) / 8u);
    const DeferSizes z = defer_sizes(ntiles * std::max(1u, c->defer_sub / 2u), p->max_depth, npx); // as prepare_defer
    return defer_bufs_fit(c->split[slot], z, npx, frames) ? 0 : z.bytes * frames;
}

// The automatic frames-in-flight count of a deferred loop, bounded by device memory: each slot
// holds its own scratch (defer_sizes: the shipped 1024x768 frame ~1 GB per slot), and the slots that would still need allocating may take
// at most half of the free device memory.
uint32_t fit_defer_slots(const trt_ctx* c, const trt_params* p, uint32_t want, uint32_t frames) {
    size_t freeb = 0, total = 0;
    if (hipMemGetInfo(&freeb, &total) != hipSuccess) return want;
    size_t need = 0;
    uint32_t n = 0;
    for (; n < want && n < TRT_BUILD_MAX_IN_FLIGHT; ++n) {
        need += defer_slot_bytes(c, p, n, frames);
        if (n > 0 && need > freeb / 2) break;
    }
    return std::max(1u, n);
}

void free_defer_bufs(trt_ctx::SplitBufs& b) {
    void* ps[] = {b.ev, b.shq, b.px_ev, b.fb};
    for (void* q : ps) (void)hipFree(q);
    (void)hipFree(b.dctr);
    b.ev = nullptr;
    b.shq = nullptr;
    b.px_ev = nullptr;
    b.fb = nullptr;
    b.dctr = nullptr;
    b.ev_chunks = b.shq_cap = b.dnpx = 0;
    b.dframes = 0;
}

// Allocates slot `slot`'s deferred-frame scratch for this frame and fills
// A's defer fields.
int prepare_defer(trt_ctx* c, const trt_params* p, KArgs& A, uint32_t slot) {
    auto& b = c->split[slot];
    const size_t npx = (size_t)trt_output_rows(p) * p->width;
    const uint32_t G = std::max(A.nframes, 1u); // frames of this launch, each with its own scratch
    // pass-A waves per tile (pool design): explicit (TRT_DEFER_PPW), else by the frames that
    // overlap: with few frames in flight a frame's latency — its deepest tiles' chains of walks —
    // sets the rate, and more waves per tile spread a deep tile's pixels (the shipped frame at 2
    // in flight: 1 wave 1.09, 2 waves 0.82 ms, profiles/r05j_ab_defer_ppw.jsonl; 4 waves a
    // further -2 % on both deep scenes at 2 in flight, 8 waves +12 % / -10 %, and at 4 in flight
    // 2 waves stay best, profiles/r06zb_ab_pass_a_waves_per_tile.jsonl); with many, the idle
    // lanes of the cheap tiles cost more than the overlap hides (at 16 in flight 0.32 -> 0.40 ms)
    const uint32_t ov = c->cur_in_flight * G;
    const uint32_t Sd = c->defer_sub ? c->defer_sub : ov <= 2u ? 4u : ov <= 4u ? 2u : 1u;
    // every pass-A wave takes its own event chunks (a row of 64 lanes per step, idle lanes'
    // slots unused): four waves per tile need twice the chunks of two (the shipped frame at two
    // waves peaks at 60 % of the capacity, profiles/r06z_defer_probe.jsonl)
    const DeferSizes z = defer_sizes(A.ntiles * std::max(1u, Sd / 2u), p->max_depth, npx);
    if (!defer_bufs_fit(b, z, npx, G)) {
        free_defer_bufs(b);
        hipError_t e = hipSuccess;
        auto alloc = [&](void** q, size_t bytes) {
            if (e == hipSuccess && bytes) e = hipMalloc(q, bytes);
        };
        if ((int)slot == test_fail_defer_slot()) e = hipErrorOutOfMemory;
        alloc((void**)&b.ev, G * z.chunks * kPoolEvBytes);
        alloc((void**)&b.shq, G * z.qcap * 2 * sizeof(float4));
        alloc((void**)&b.px_ev, G * npx * sizeof(uint2));
        alloc((void**)&b.fb, G * npx * sizeof(uint32_t));
        alloc((void**)&b.dctr, G * sizeof(trt::DeferCtr));
        if (e != hipSuccess) {
            free_defer_bufs(b);
            return hip_fail(c, e, "alloc deferred-frame buffers");
        }
        b.ev_chunks = z.chunks;
        b.shq_cap = z.qcap;
        b.dnpx = npx;
        b.dframes = G;
    }
    A.defer = 1;
    A.defer_sub = Sd;
    A.defer_inter = c->defer_inter;
    // test hooks: tiny capacities exercise the in-place fallback (tests/test_gpu_defer.py)
    A.ev_cap = (uint32_t)env_cap("TRT_DEFER_EVCAP", z.chunks / trt::kDeferStripes);
    A.shq_cap = (uint32_t)env_cap("TRT_DEFER_QCAP", z.qcap / trt::kDeferStripes);
    A.ev = b.ev;
    A.shq = b.shq;
    A.px_ev = b.px_ev;
    A.fb = b.fb;
    A.dctr = b.dctr;
    A.dframes = G;
    A.ev_fstride = b.ev_chunks * (kPoolEvBytes / sizeof(float4));
    A.shq_fstride = b.shq_cap * 2;
    A.px_fstride = (uint32_t)b.dnpx;
    b.used_ev_cap = A.ev_cap;
    b.used_shq_cap = A.shq_cap;
    return TRT_OK;
}

// Allocates slot `slot`'s split (or deferred-shadow) scratch for this frame size and fills A's
// split / defer fields; a frame on `stream` waits for the slot's previous frame when that ran
// on another stream.
int prepare_split(trt_ctx* c, const trt_params* p, KArgs& A, uint32_t slot, hipStream_t stream) {
    A.split_w = 0;
    A.split_d1 = A.max_depth;
    A.num_cus = c->num_cus;
    A.defer = 0;
    const bool defer = defer_frame(c, p);
    // A COUNT frame of a scene whose frames run deferred is traced unsplit, so its image is the
    // deferred frame's bit for bit (both are the reference's single running sum; a deferred
    // frame's subtree split keeps that order through LINK events).
    if (defer || !defer_frame(c, p, true)) A.split_w = split_window(c, p);
    if (!A.split_w && !defer) return TRT_OK;
    auto& b = c->split[slot];
    if (b.last && b.last != stream) HIP_TRY(c, hipStreamWaitEvent(stream, b.done, 0));
    if (defer) {
        const int rc = prepare_defer(c, p, A, slot);
        if (rc != TRT_OK) return rc;
    }
    if (!A.split_w) return TRT_OK;
    const size_t npx = (size_t)trt_output_rows(p) * p->width;
    if (npx > b.npx) {
        // queue capacity: 4 tasks per pixel per window edge (a full queue is not an error: the
        // child is traced in place, SplitCtr::overflow counts it; a deferred frame re-traces
        // the pixel in place)
        const size_t cap = std::min<size_t>(std::max<size_t>(4 * npx, 1u << 16), 1u << 28);
        auto drop = [&] {
            for (auto*& q : b.q) (void)hipFree(q), q = nullptr;
            for (auto*& q : b.qlink) (void)hipFree(q), q = nullptr;
            (void)hipFree(b.acc);
            (void)hipFree(b.spilled);
            b.acc = nullptr;
            b.spilled = nullptr;
            b.npx = 0;
            b.cap = 0;
        };
        drop();
        hipError_t e = hipMalloc((void**)&b.q[0], cap * sizeof(trt::Task));
        if (e == hipSuccess) e = hipMalloc((void**)&b.q[1], cap * sizeof(trt::Task));
        if (e == hipSuccess) e = hipMalloc((void**)&b.qlink[0], cap * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc((void**)&b.qlink[1], cap * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc((void**)&b.acc, npx * 4 * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMalloc((void**)&b.spilled, npx * sizeof(uint32_t));
        if (e == hipSuccess && !b.ctr) e = hipMalloc((void**)&b.ctr, sizeof(trt::SplitCtr));
        if (e != hipSuccess) {
            drop();
            return hip_fail(c, e, "alloc subtree-split buffers");
        }
        b.npx = npx;
        b.cap = (uint32_t)cap;
    }
    A.q_link_buf[0] = b.qlink[0];
    A.q_link_buf[1] = b.qlink[1];
    A.q_buf[0] = b.q[0];
    A.q_buf[1] = b.q[1];
    A.q_cap = b.cap;
    // test hook: a tiny queue exercises the in-place fallback (tests/test_gpu_split.py)
    if (const char* e = std::getenv("TRT_SPLIT_QCAP")) A.q_cap = std::min<uint32_t>(A.q_cap, (uint32_t)std::strtoul(e, nullptr, 10));
    A.acc = b.acc;
    A.spilled = b.spilled;
    A.ctr = b.ctr;
    return TRT_OK;
}

// After a split frame's launches on `stream`: the slot's fence.
int fence_split(trt_ctx* c, const KArgs& A, uint32_t slot, hipStream_t stream) {
    if (!A.split_w && !A.defer) return TRT_OK;
    auto& b = c->split[slot];
    if (!b.done) HIP_TRY(c, hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(b.done, stream));
    b.last = stream;
    return TRT_OK;
}

// trt_render's split slot: one per distinct stream among the last TRT_BUILD_MAX_IN_FLIGHT
// (so renders alternating between streams overlap), reused least recently first.
uint32_t render_slot(trt_ctx* c, hipStream_t s) {
    for (uint32_t k = 0; k < TRT_BUILD_MAX_IN_FLIGHT; ++k)
        if (c->render_slot_stream[k] == s) return k;
    const uint32_t k = c->render_slot_next;
    c->render_slot_next = (k + 1) % TRT_BUILD_MAX_IN_FLIGHT;
    c->render_slot_stream[k] = s;
    return k;
}

} // namespace

namespace trt {

int render_frame_list(trt_ctx* c, const trt_params* p, const FrameOut* frames, uint32_t nframes,
                      uint32_t time_every) {
    if (!c) return TRT_ERR_INVALID;
    int rc = check_params(c, p);
    if (rc != TRT_OK) return rc;
    if (!(p->flags & TRT_FLAG_DEVICE_PTRS))
        return fail(c, TRT_ERR_INVALID, "trt_render_frames: needs TRT_FLAG_DEVICE_PTRS");
    if (p->flags & TRT_FLAG_COUNT)
        return fail(c, TRT_ERR_INVALID, "trt_render_frames: COUNT is a per-frame trt_render flag");
    if (nframes && !frames) return fail(c, TRT_ERR_INVALID, "trt_render_frames: null frame list");
    HIP_TRY(c, hipSetDevice(c->device));
    const bool timing = time_every > 0;
    const uint32_t every = timing ? time_every : 1u;
    c->fev_frames = 0;
    c->fev_nframes.clear();
    if ((rc = ensure_envp(c, p, c->stream)) != TRT_OK) return rc;
    KArgs A;
    fill_args(c, p, A);
    A.rays_in = reinterpret_cast<const float*>(p->rays_in);
    auto ubo_of = [&](uint32_t i) -> const trt_ubo& { return frames[i].ubo ? *frames[i].ubo : c->ubo; };
    if (A.rows == 0 || nframes == 0) {
        if (nframes) c->ubo = ubo_of(nframes - 1);
        return TRT_OK;
    }
    // Plain frames (no subtree split, no deferred shadows: the same decision prepare_split
    // makes) go out several per launch; the others one per launch (per-slot scratch).
    const bool defer = defer_frame(c, p);
    const bool split = (defer || !defer_frame(c, p, true)) && split_window(c, p) != 0;
    const bool plain = !defer && !split;
    // Frames in flight (main.cpp:45, MAX_FRAMES_IN_FLIGHT): launch j runs on slot j % n.  Slot 0
    // is the context's stream, slots 1..n-1 are context-owned streams forked from it here and
    // joined back into it below, so to the caller all frames complete on its stream.  A plain
    // loop needs no second slot: one multi-frame launch keeps the GPU full from its first frame
    // to its last, so a 20-frame loop is one launch and drains once (C2 at 20 frames: 20.5 us per
    // frame against 25.0 with one launch per frame on 4 slots; at 1000 frames 15.6 vs 15.9,
    // profiles/r03_ab_frame_batch.log); with n slots set explicitly the frames are spread over
    // n launches.  Per-frame launch sequences (split / deferred-shadow frames) keep the slots
    // busy instead: auto 4, or defer_in_flight (16) for deferred-shadow frames (8 vs 16 in round
    // 4: the shipped frame 0.42 -> 0.35 ms, the README scene 0.24 -> 0.17 ms,
    // profiles/r04z_ab_deferred_in_flight.jsonl; round 2: the shipped frame 1.45 -> 0.56 ms at
    // 8, profiles/r02_ab_queues_deep.log).
    uint32_t want = c->frames_in_flight ? c->frames_in_flight : plain ? 1u : defer ? c->defer_in_flight : 4u;
    // auto: no more deferred slots than device memory holds (each slot owns its scratch)
    // deferred frames (not split) go out in groups of frames per launch sequence (defer_shape)
    uint32_t group = 1;
    if (defer && !split) {
        uint32_t slots = want;
        defer_shape(c, group, slots);
        group = std::min(group, trt::kMaxLaunchFrames);
        want = slots;
    }
    if (!c->frames_in_flight && defer) want = fit_defer_slots(c, p, want, group);
    const uint32_t cap = plain ? (c->frame_batch ? c->frame_batch : trt::kMaxLaunchFrames) : group;
    const uint32_t per_launch = std::max(1u, std::min(cap, (nframes + want - 1) / want));
    // launches: runs of consecutive frames sharing every UBO field but camPos
    std::vector<uint32_t> first{0};
    for (uint32_t i = 1; i < nframes; ++i)
        if (i - first.back() >= per_launch || !same_but_camera(ubo_of(i), ubo_of(first.back()))) first.push_back(i);
    const uint32_t nl = (uint32_t)first.size();
    first.push_back(nframes);
    if (timing) {
        const uint32_t ntimed = (nl + every - 1) / every; // launches 0, every, 2*every, ...
        while (c->fev.size() < 2 * (size_t)ntimed) {
            hipEvent_t e;
            HIP_TRY(c, hipEventCreate(&e));
            c->fev.push_back(e);
        }
    }
    uint32_t nfl = std::min(want, nl);
    c->cur_in_flight = nfl;
    std::vector<hipStream_t> sv{c->stream};
    // every slot's stream is made on first use of the in-flight count, not only the ones this
    // call needs: creating a stream takes milliseconds and must not land in a later, longer
    // call (a timed loop after a short warmup)
    while (c->aux.size() + 1 < want) {
        hipStream_t s;
        HIP_TRY(c, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        HIP_TRY(c, trt::touch_stream(s, c->d_counters)); // its hardware queue exists from now on
        c->aux.push_back(s);
        hipEvent_t e;
        HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->aux_ev.push_back(e);
    }
    if (nfl > 1) {
        if (!c->fork_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
        HIP_TRY(c, hipEventRecord(c->fork_ev, c->stream));
        for (uint32_t k = 0; k + 1 < nfl; ++k) {
            HIP_TRY(c, hipStreamWaitEvent(c->aux[k], c->fork_ev, 0));
            sv.push_back(c->aux[k]);
        }
    }
    for (uint32_t j = 0; j < nl; ++j) {
        const uint32_t i0 = first[j], n = first[j + 1] - i0;
        c->ubo = ubo_of(i0);
        fill_ubo_args(A, c->ubo);
        A.nframes = n;
        for (uint32_t k = 0; k < n; ++k) fill_frame(A.fr[k], ubo_of(i0 + k), frames[i0 + k].out8, frames[i0 + k].in_place);
        uint32_t slot = j % nfl;
        if ((rc = prepare_split(c, p, A, slot, sv[slot])) != TRT_OK) {
            // auto count: a slot whose scratch does not fit in device memory is dropped, with the
            // slots after it, and the launch goes to a slot that has its scratch; any other
            // failure is the caller's
            if (c->frames_in_flight || slot == 0 || rc != TRT_ERR_OOM) return rc;
            (void)hipGetLastError(); // the failed hipMalloc's sticky error: not the next launch's
            c->err.clear();
            nfl = slot;
            c->cur_in_flight = nfl;
            slot = j % nfl;
            if ((rc = prepare_split(c, p, A, slot, sv[slot])) != TRT_OK) return rc;
        }
        hipStream_t st = sv[slot];
        const bool timed = timing && j % every == 0;
        const size_t k = 2 * (size_t)(j / every);
        if (timed) HIP_TRY(c, hipEventRecord(c->fev[k], st));
        HIP_TRY(c, trt::launch_trace(A, st, false));
        if ((rc = fence_split(c, A, slot, st)) != TRT_OK) return rc;
        if (timed) {
            HIP_TRY(c, hipEventRecord(c->fev[k + 1], st));
            c->fev_nframes.push_back(n);
            c->fev_frames = j / every + 1;
        }
    }
    c->ubo = ubo_of(nframes - 1);
    for (uint32_t k = 0; k + 1 < nfl; ++k) {
        HIP_TRY(c, hipEventRecord(c->aux_ev[k], c->aux[k]));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->aux_ev[k], 0));
    }
    return TRT_OK;
}

} // namespace trt

extern "C" int trt_render_frames(trt_ctx* c, const trt_params* p, const trt_ubo* ubos, uint32_t nframes,
                                 uint8_t* out8, size_t frame_stride, uint32_t time_every) {
    if (!c) return TRT_ERR_INVALID;
    if (!p) return fail(c, TRT_ERR_INVALID, "trt_render_frames: null params");
    std::vector<trt::FrameOut> fl(nframes);
    const bool in_place = (p->flags & TRT_FLAG_BAND_IN_PLACE) != 0;
    for (uint32_t i = 0; i < nframes; ++i)
        fl[i] = trt::FrameOut{ubos ? &ubos[i] : nullptr, out8 ? out8 + (size_t)i * frame_stride : nullptr, in_place};
    // TRT_FLAG_TIMING: events around every time_every-th launch (0 or 1: every launch)
    return trt::render_frame_list(c, p, fl.data(), nframes, (p->flags & TRT_FLAG_TIMING) ? std::max(time_every, 1u) : 0u);
}

extern "C" int trt_set_frame_batch(trt_ctx* c, uint32_t n) {
    if (!c) return TRT_ERR_INVALID;
    if (n > TRT_MAX_FRAME_BATCH)
        return fail(c, TRT_ERR_INVALID, "trt_set_frame_batch: n must be 0 (auto) or in [1, TRT_MAX_FRAME_BATCH]");
    c->frame_batch = n;
    return TRT_OK;
}

extern "C" int trt_frame_times(trt_ctx* c, float* ms, uint32_t n) {
    if (!c || (!ms && n)) return TRT_ERR_INVALID;
    if (n > c->fev_frames) return fail(c, TRT_ERR_INVALID, "trt_frame_times: more launches than were timed");
    HIP_TRY(c, hipSetDevice(c->device));
    for (uint32_t i = 0; i < n; ++i) {
        HIP_TRY(c, hipEventSynchronize(c->fev[2 * i + 1]));
        HIP_TRY(c, hipEventElapsedTime(&ms[i], c->fev[2 * i], c->fev[2 * i + 1]));
        ms[i] /= (float)std::max(c->fev_nframes[i], 1u);
    }
    return TRT_OK;
}

extern "C" uint32_t trt_timed_launches(trt_ctx* c, uint32_t* frames_out, uint32_t cap) {
    if (!c) return 0;
    for (uint32_t i = 0; frames_out && i < cap && i < c->fev_frames; ++i) frames_out[i] = c->fev_nframes[i];
    return c->fev_frames;
}

extern "C" {

int trt_render(trt_ctx* c, const trt_params* p, uint8_t* out8, float* out32, trt_stats* st) {
    if (!c) return TRT_ERR_INVALID;
    int rc = check_params(c, p);
    if (rc != TRT_OK) return rc;
    HIP_TRY(c, hipSetDevice(c->device));

    const bool dev = (p->flags & TRT_FLAG_DEVICE_PTRS) != 0;
    const bool count = (p->flags & TRT_FLAG_COUNT) != 0 && st;
    const bool timing = (p->flags & TRT_FLAG_TIMING) != 0 && st;
    const uint32_t rows = trt_output_rows(p);
    const size_t npx = (size_t)rows * p->width;

    if ((rc = ensure_envp(c, p, c->stream)) != TRT_OK) return rc;
    KArgs A;
    fill_args(c, p, A);

    if (p->rays_in) {
        if (dev) {
            A.rays_in = reinterpret_cast<const float*>(p->rays_in);
        } else {
            const size_t bytes = sizeof(trt_ray) * (size_t)p->width * p->height;
            if ((rc = ensure(c, &c->d_rays, &c->caprays, bytes, "alloc rays")) != TRT_OK) return rc;
            HIP_TRY(c, hipMemcpyAsync(c->d_rays, p->rays_in, bytes, hipMemcpyHostToDevice, c->stream));
            A.rays_in = reinterpret_cast<const float*>(c->d_rays);
        }
    }
    if (out8) {
        if (dev) {
            A.fr[0].out8 = reinterpret_cast<uint32_t*>(out8);
        } else {
            if ((rc = ensure(c, &c->d_out8, &c->cap8, npx * 4, "alloc rgba8")) != TRT_OK) return rc;
            A.fr[0].out8 = reinterpret_cast<uint32_t*>(c->d_out8);
        }
    }
    if (out32) {
        if (dev) {
            A.out32 = out32;
        } else {
            if ((rc = ensure(c, &c->d_out32, &c->cap32, npx * 16, "alloc rgba32f")) != TRT_OK) return rc;
            A.out32 = reinterpret_cast<float*>(c->d_out32);
        }
    }
    const uint32_t slot = render_slot(c, c->stream);
    c->cur_in_flight = 1u; // one frame: its latency is the rate
    if ((rc = prepare_split(c, p, A, slot, c->stream)) != TRT_OK) return rc;
    if (count) HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, 32 * sizeof(unsigned long long), c->stream));
    if (timing) HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
    if (npx > 0) HIP_TRY(c, trt::launch_trace(A, c->stream, count));
    if ((rc = fence_split(c, A, slot, c->stream)) != TRT_OK) return rc;
    if (timing) HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
    if (out8 && !dev)
        HIP_TRY(c, hipMemcpyAsync(out8, c->d_out8, npx * 4, hipMemcpyDeviceToHost, c->stream));
    if (out32 && !dev)
        HIP_TRY(c, hipMemcpyAsync(out32, c->d_out32, npx * 16, hipMemcpyDeviceToHost, c->stream));
    unsigned long long cnt[32] = {0};
    if (count)
        HIP_TRY(c, hipMemcpyAsync(cnt, c->d_counters, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
    if (!dev || count || timing) HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (st) {
        st->primary_rays = cnt[0];
        st->secondary_rays = cnt[1];
        st->shadow_rays = cnt[2];
        st->misses = cnt[3];
        st->tri_nearest = cnt[4];
        st->sphere_tests = cnt[5];
        st->batch_tests = cnt[6];
        st->batch_hits = cnt[7];
        st->tri_tests = cnt[8];
        st->node_tests = cnt[9];
        st->tri_past_a = cnt[10];
        st->tri_past_u = cnt[11];
        st->tri_past_v = cnt[12];
        st->shadow_skipped = cnt[13];
        st->skipped_sphere_tests = cnt[14];
        st->skipped_box_tests = cnt[15];
        st->skipped_tri_tests = cnt[16];
        st->skipped_tri_past_a = cnt[17];
        st->skipped_tri_past_u = cnt[18];
        st->skipped_tri_past_v = cnt[19];
        st->kernel_ms = 0.0;
        if (timing) {
            float ms = 0.0f;
            HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
            st->kernel_ms = ms;
        }
    }
    return TRT_OK;
}

} // extern "C"

// ---- envmap JPEG: host entropy decode + GPU reconstruction ----------------

namespace trt {
namespace jpeg {
const Image* image_of(const trt_jpeg* j);
}
} // namespace trt

extern "C" int trt_jpeg_decode(trt_ctx* c, const trt_jpeg* j, uint8_t* out, uint32_t flags) {
    if (!c) return TRT_ERR_INVALID;
    const trt::jpeg::Image* im = trt::jpeg::image_of(j);
    if (!im) return fail(c, TRT_ERR_INVALID, "trt_jpeg_decode: nothing parsed");
    if (!out) return fail(c, TRT_ERR_INVALID, "trt_jpeg_decode: null output");
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t bytes = (size_t)im->width * im->height * 4;
    uint8_t* dst = out;
    if (!(flags & TRT_FLAG_DEVICE_PTRS)) {
        int rc = ensure(c, &c->d_out8, &c->cap8, bytes, "jpeg output");
        if (rc != TRT_OK) return rc;
        dst = static_cast<uint8_t*>(c->d_out8);
    }
    HIP_TRY(c, trt::jpeg::reconstruct(*im, dst, c->stream));
    if (!(flags & TRT_FLAG_DEVICE_PTRS)) {
        HIP_TRY(c, hipMemcpyAsync(out, dst, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return TRT_OK;
}

extern "C" int trt_upload_envmap_jpeg(trt_ctx* c, const uint8_t* data, size_t len) {
    if (!c) return TRT_ERR_INVALID;
    trt_jpeg* j = nullptr;
    int rc = trt_jpeg_create(&j);
    if (rc != TRT_OK) return fail(c, rc, "trt_upload_envmap_jpeg: out of memory");
    rc = trt_jpeg_parse(j, data, len);
    if (rc != TRT_OK) {
        std::string msg = std::string("trt_upload_envmap_jpeg: ") + trt_jpeg_last_error(j);
        trt_jpeg_destroy(j);
        return fail(c, rc, msg);
    }
    const trt::jpeg::Image* im = trt::jpeg::image_of(j);
    hipError_t e = hipSetDevice(c->device);
    uint32_t* d = nullptr;
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d), (size_t)im->width * im->height * 4);
    if (e == hipSuccess) e = trt::jpeg::reconstruct(*im, reinterpret_cast<uint8_t*>(d), c->stream);
    if (e != hipSuccess) {
        (void)hipFree(d);
        trt_jpeg_destroy(j);
        return hip_fail(c, e, "trt_upload_envmap_jpeg");
    }
    (void)hipFree(c->d_env);
    c->d_env = d;
    c->envp_ok = false;
    c->env_w = (uint32_t)im->width;
    c->env_h = (uint32_t)im->height;
    c->scene_bytes[trt::kSceneEnv] = (size_t)im->width * im->height * 4;
    trt_jpeg_destroy(j);
    return TRT_OK;
}

// ---- scene export / adoption (the RCCL scene broadcast of trt_multi.cpp) --------------------

namespace trt {

void** scene_buf(trt_ctx* c, int k) {
    switch (k) {
    case kSceneBatches: return reinterpret_cast<void**>(&c->d_batches);
    case kSceneNodes: return reinterpret_cast<void**>(&c->d_nodes);
    case kSceneBvh: return reinterpret_cast<void**>(&c->d_bvh);
    case kSceneBvh4: return reinterpret_cast<void**>(&c->d_bvh4);
    case kSceneBvhTris: return reinterpret_cast<void**>(&c->d_bvh_tris);
    case kSceneGeo: return reinterpret_cast<void**>(&c->d_geo);
    case kSceneShade: return reinterpret_cast<void**>(&c->d_shade);
    case kSceneMats: return reinterpret_cast<void**>(&c->d_mats);
    case kSceneBvh4Q: return reinterpret_cast<void**>(&c->d_bvh4q);
    default: return reinterpret_cast<void**>(&c->d_env);
    }
}

void scene_header(const trt_ctx* c, SceneHeader& h) {
    std::memset(&h, 0, sizeof(h));
    h.magic = kSceneMagic;
    h.nbatch = c->nbatch;
    h.ntri = c->ntri;
    h.nmat = c->nmat;
    h.env_w = c->env_w;
    h.env_h = c->env_h;
    h.top = c->top;
    std::memcpy(h.node_off, c->node_off, sizeof(h.node_off));
    for (int k = 0; k < kSceneBufs; ++k) h.bytes[k] = c->scene_bytes[k];
    h.ubo = c->ubo;
}

int scene_adopt(trt_ctx* c, const SceneHeader& h) {
    if (h.magic != kSceneMagic) return fail(c, TRT_ERR_INVALID, "scene broadcast: bad header");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    free_scene(c);
    for (int k = 0; k < kSceneBufs; ++k) {
        if (!h.bytes[k]) continue;
        void** p = scene_buf(c, k);
        hipError_t e = hipMalloc(p, h.bytes[k]);
        if (e != hipSuccess) {
            free_scene(c);
            return hip_fail(c, e, "scene broadcast: alloc");
        }
        c->scene_bytes[k] = h.bytes[k];
    }
    c->nbatch = h.nbatch;
    c->ntri = h.ntri;
    c->nmat = h.nmat;
    c->env_w = h.env_w;
    c->env_h = h.env_h;
    c->top = h.top;
    std::memcpy(c->node_off, h.node_off, sizeof(c->node_off));
    c->ubo = h.ubo;
    c->have_scene = true;
    return TRT_OK;
}

} // namespace trt

// ---- diagnostics (not part of include/trt/abi.h; tools/shadow_exp.py) ----------------------

// Ray-dump buffer of TRT_DIAG_DUMP_SHADOW builds (device pointer, or NULL).
// diagnostic: the first 16 words of slot `slot`'s deferred-frame counters (nfb + pad, where
// defer_resolve records a log it could not finish)
extern "C" int trt_diag_defer_pad(trt_ctx* c, uint32_t slot, uint32_t* out16) {
    if (!c || !out16 || slot >= TRT_BUILD_MAX_IN_FLIGHT || !c->split[slot].dctr) return TRT_ERR_INVALID;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(out16, c->split[slot].dctr, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return TRT_OK;
}

extern "C" int trt_diag_set_buffer(trt_ctx* c, void* dev_ptr) {
    if (!c) return TRT_ERR_INVALID;
    c->diag = dev_ptr;
    return TRT_OK;
}

// counters[k] of the last counting pass (k < 32).
extern "C" unsigned long long trt_diag_counter(trt_ctx* c, uint32_t k) {
    unsigned long long v = 0;
    if (!c || k >= 32 || hipSetDevice(c->device) != hipSuccess) return 0;
    if (hipMemcpy(&v, c->d_counters + k, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    return v;
}

// Traces n shadow queries (2 float4 each, device) into occ (device, one uint32 each) on the
// context's stream with the frame params' traversal (BVH build, waves).
extern "C" int trt_diag_shadow_batch(trt_ctx* c, const trt_params* p, const void* rays, uint32_t n, void* occ) {
    if (!c) return TRT_ERR_INVALID;
    int rc = check_params(c, p);
    if (rc != TRT_OK) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = ensure_envp(c, p, c->stream)) != TRT_OK) return rc;
    KArgs A;
    fill_args(c, p, A);
    HIP_TRY(c, trt::launch_shadow_batch(A, static_cast<const float4*>(rays), n, static_cast<uint32_t*>(occ), c->stream));
    return TRT_OK;
}

// Diagnostic (tests/test_bvh_layout.py): the BVH2 the upload builds — nodes and the BVH-ordered
// leaf triangle records (meta: triangle, batch, ni) — copied out when the capacities suffice;
// counts[0] = nodes, counts[1] = leaf references.
extern "C" int trt_diag_bvh_export(const trt_triangle* tris, uint32_t ntri, const trt_model* models, uint32_t nmodel,
                                   trt::BvhNode* nodes_out, uint32_t cap_nodes, TriGeo* tris_out, uint32_t cap_tris,
                                   uint64_t counts[2]) {
    if (!counts || (ntri && !tris) || (nmodel && !models)) return TRT_ERR_INVALID;
    std::vector<trt::BvhNode> bvh;
    std::vector<TriGeo> bvh_tris;
    if (!nmodel || !trt::build_bvh(tris, ntri, models, nmodel, bvh, bvh_tris)) return TRT_ERR_INVALID;
    counts[0] = bvh.size();
    counts[1] = bvh_tris.size();
    if (nodes_out && bvh.size() <= cap_nodes) std::memcpy(nodes_out, bvh.data(), bvh.size() * sizeof(trt::BvhNode));
    if (tris_out && bvh_tris.size() <= cap_tris) std::memcpy(tris_out, bvh_tris.data(), bvh_tris.size() * sizeof(TriGeo));
    return TRT_OK;
}

// Host-only check of the BVH pipeline of trt_upload_scene (no GPU): BVH2 build, 4-wide
// collapse and quantization.  out[0] BVH2 nodes, out[1] BVH4 nodes, out[2] quantized (0/1),
// out[3] BVH2 depth (levels of the deepest leaf, root = 1), out[4] worst-case BVH4 stack,
// out[5] leaf triangles.  Returns TRT_ERR_INVALID when no BVH is built (overlapping batch ranges).
extern "C" int trt_diag_bvh_build(const trt_triangle* tris, uint32_t ntri, const trt_model* models, uint32_t nmodel,
                                  uint64_t out[6]) {
    if (!out || (ntri && !tris) || (nmodel && !models)) return TRT_ERR_INVALID;
    for (int i = 0; i < 6; ++i) out[i] = 0;
    std::vector<trt::BvhNode> bvh;
    std::vector<TriGeo> bvh_tris;
    if (!nmodel || !trt::build_bvh(tris, ntri, models, nmodel, bvh, bvh_tris)) return TRT_ERR_INVALID;
    std::vector<trt::Bvh4Node> bvh4;
    out[0] = bvh.size();
    out[4] = trt::collapse_bvh4(bvh, bvh4);
    out[1] = bvh4.size();
    std::vector<trt::Bvh4QNode> q;
    out[2] = (!bvh4.empty() && trt::quantize_bvh4(bvh4, q)) ? 1 : 0;
    out[3] = trt::bvh_depth(bvh);
    out[5] = bvh_tris.size();
    return TRT_OK;
}
