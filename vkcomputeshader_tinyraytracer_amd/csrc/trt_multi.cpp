// trt_multi.cpp — one frame row-tiled over the GPUs of a node, gathered over RCCL (xGMI).
//
// The reference renders every frame on one GPU through one VkQueue (main.cpp:722-724,
// dispatch main.cpp:2108-2131, submit main.cpp:2181-2205).  Here the frame's rows are dealt to
// the devices in interleaved bands (row y belongs to band group (y / B) % G_total, so the
// costly image centre is spread over every device), each device renders its band groups with
// the single-GPU kernel (trt_render with band_* params) into a compact RGBA8 buffer, and one
// grouped ncclSend / ncclRecv moves the compact buffers to the frame's root device, where a
// re-interleave kernel writes the frame.  The scene is uploaded once on rank 0 and broadcast
// (ncclBroadcast of the packed device bindings), so a C++ host builds it only once.
//
// Two ways to create the communicator:
//   * trt_multi_create:      one process drives N devices (ncclCommInitAll), the SURVEY §8(b)
//                            single-process form;
//   * trt_multi_create_rank: one process per GPU (ncclCommInitRank with an id exchanged out of
//                            band), the layout torch.distributed / the bench uses.
// Pipelining: batches of frames alternate between two buffer slots; each slot has its own
// render stream per device, and the gathers run on a per-device communication stream, so a
// batch's gather + re-interleave overlaps the next batch's render (the reference's
// MAX_FRAMES_IN_FLIGHT = 2, main.cpp:45).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/trt/abi.h"
#include "trt_ctx.h"

namespace trt {
hipError_t launch_interleave(const uint32_t* gather, uint32_t* out, uint32_t width, uint32_t height,
                             uint32_t band_rows, uint32_t groups, uint32_t max_rows, uint32_t nframes,
                             size_t frame_stride_px, hipStream_t stream, uint32_t skip_lo, uint32_t skip_hi);
}

struct trt_multi {
    struct Dev {
        int device = 0;
        uint32_t rank = 0;
        trt_ctx* ctx = nullptr;
        ncclComm_t comm = nullptr;
        hipStream_t comm_stream = nullptr;
        hipStream_t render[2] = {nullptr, nullptr};
        hipEvent_t rendered[2] = {nullptr, nullptr};
        hipEvent_t gathered[2] = {nullptr, nullptr};
        bool gathered_valid[2] = {false, false};
        hipEvent_t fork = nullptr, join = nullptr;
        uint8_t* local[2] = {nullptr, nullptr}; // this device's compact band groups of a batch
        size_t local_cap[2] = {0, 0};
        uint8_t* gather[2] = {nullptr, nullptr}; // all compact buffers of a batch (as root)
        size_t gather_cap[2] = {0, 0};
        uint8_t* frame = nullptr; // trt_render_multi with host output: the root's frame
        size_t frame_cap = 0;
        void* scratch = nullptr;  // scene header / counters
    };
    std::vector<Dev> devs;
    uint32_t nranks = 1;
    uint32_t groups = 1; // band groups per rank
    uint64_t batch_seq = 0;
    bool have_scene = false;
    std::string err;
};

namespace {

constexpr size_t kScratchBytes = 4096;
static_assert(sizeof(trt::SceneHeader) <= kScratchBytes, "scene header fits the scratch buffer");

int mfail(trt_multi* m, int code, const std::string& msg) {
    if (m) m->err = msg;
    return code;
}

#define MHIP(m, expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return mfail((m), TRT_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define MNCCL(m, expr)                                                                           \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) return mfail((m), TRT_ERR_HIP, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)
#define MTRY(m, ctx, expr)                                                                       \
    do {                                                                                         \
        int rc_ = (expr);                                                                        \
        if (rc_ != TRT_OK) return mfail((m), rc_, std::string(#expr ": ") + trt_last_error(ctx)); \
    } while (0)

int init_dev(trt_multi* m, trt_multi::Dev& d) {
    int rc = trt_create(&d.ctx, d.device);
    if (rc != TRT_OK) return mfail(m, rc, "trt_create(device " + std::to_string(d.device) + ") failed");
    MHIP(m, hipSetDevice(d.device));
    MHIP(m, hipStreamCreateWithFlags(&d.comm_stream, hipStreamNonBlocking));
    for (int s = 0; s < 2; ++s) {
        MHIP(m, hipStreamCreateWithFlags(&d.render[s], hipStreamNonBlocking));
        MHIP(m, hipEventCreateWithFlags(&d.rendered[s], hipEventDisableTiming));
        MHIP(m, hipEventCreateWithFlags(&d.gathered[s], hipEventDisableTiming));
    }
    MHIP(m, hipEventCreateWithFlags(&d.fork, hipEventDisableTiming));
    MHIP(m, hipEventCreateWithFlags(&d.join, hipEventDisableTiming));
    MHIP(m, hipMalloc(&d.scratch, kScratchBytes));
    return TRT_OK;
}

void free_dev(trt_multi::Dev& d) {
    (void)hipSetDevice(d.device);
    if (d.comm_stream) (void)hipStreamSynchronize(d.comm_stream);
    for (int s = 0; s < 2; ++s) {
        if (d.render[s]) {
            (void)hipStreamSynchronize(d.render[s]);
            (void)hipStreamDestroy(d.render[s]);
        }
        if (d.rendered[s]) (void)hipEventDestroy(d.rendered[s]);
        if (d.gathered[s]) (void)hipEventDestroy(d.gathered[s]);
        (void)hipFree(d.local[s]);
        (void)hipFree(d.gather[s]);
    }
    if (d.fork) (void)hipEventDestroy(d.fork);
    if (d.join) (void)hipEventDestroy(d.join);
    (void)hipFree(d.frame);
    (void)hipFree(d.scratch);
    if (d.comm) (void)ncclCommDestroy(d.comm);
    if (d.comm_stream) (void)hipStreamDestroy(d.comm_stream);
    if (d.ctx) trt_destroy(d.ctx);
}

int grow(trt_multi* m, int device, uint8_t** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap && *p) return TRT_OK;
    MHIP(m, hipSetDevice(device));
    MHIP(m, hipDeviceSynchronize()); // the old buffer may still be read by an in-flight batch
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    MHIP(m, hipMalloc(reinterpret_cast<void**>(p), bytes));
    *cap = bytes;
    return TRT_OK;
}

// Band parameters of global band group g (of NG).
trt_params group_params(const trt_params* p, uint32_t band_rows, uint32_t NG, uint32_t g) {
    trt_params q = *p;
    q.flags |= TRT_FLAG_DEVICE_PTRS;
    if (NG > 1) {
        q.band_rows = band_rows;
        q.band_count = NG;
        q.band_index = g;
    } else {
        q.band_rows = q.band_count = q.band_index = 0;
    }
    return q;
}

int check_common(trt_multi* m, const trt_params* p, uint32_t band_rows, int root) {
    if (!m) return TRT_ERR_INVALID;
    if (!p) return mfail(m, TRT_ERR_INVALID, "null params");
    if (!m->have_scene) return mfail(m, TRT_ERR_NOSCENE, "no scene uploaded (trt_multi_upload_scene)");
    if (band_rows == 0) return mfail(m, TRT_ERR_INVALID, "band_rows must be >= 1");
    if (p->band_rows && p->band_count > 1)
        return mfail(m, TRT_ERR_INVALID, "params must describe the whole frame (band_* = 0)");
    if (p->rays_in) return mfail(m, TRT_ERR_INVALID, "rays_in replay is a single-GPU (trt_render) feature");
    if (root != TRT_ROOT_ROTATE && (root < 0 || (uint32_t)root >= m->nranks))
        return mfail(m, TRT_ERR_INVALID, "root must be a rank or TRT_ROOT_ROTATE");
    return TRT_OK;
}

// One batch of `nf` frames: every local device renders its band groups of each frame into its
// compact buffer (render stream of the slot), the compact buffers go to the batch's root over
// RCCL (communication stream), and the root re-interleaves them into out + f * stride.
int run_batch(trt_multi* m, const trt_params* p, const trt_ubo* ubos, uint32_t nf, uint32_t band_rows,
              uint32_t root, bool rotate, uint8_t* const* out8, size_t frame_stride) {
    const uint32_t N = m->nranks, G = m->groups, NG = N * G;
    const uint32_t W = p->width, H = p->height;
    uint32_t max_rows = 0;
    std::vector<uint32_t> rows(NG);
    for (uint32_t g = 0; g < NG; ++g) {
        trt_params q = group_params(p, band_rows, NG, g);
        rows[g] = trt_output_rows(&q);
        max_rows = std::max(max_rows, rows[g]);
    }
    const size_t blk = (size_t)max_rows * W * 4; // one compact band-group buffer
    const int slot = (int)(m->batch_seq & 1u);
    ++m->batch_seq;
    // both slots grow together, and with a rotating root every device sizes its gather
    // buffers, so no batch after the first one of a size allocates (grow synchronizes the
    // device before it frees a buffer an in-flight batch may read)
    for (auto& d : m->devs)
        for (int s = 0; s < 2; ++s) {
            if (grow(m, d.device, &d.local[s], &d.local_cap[s], blk * G * nf) != TRT_OK) return TRT_ERR_HIP;
            if ((rotate || d.rank == root) && grow(m, d.device, &d.gather[s], &d.gather_cap[s], blk * NG * nf) != TRT_OK)
                return TRT_ERR_HIP;
        }
    // render
    size_t di = 0;
    for (auto& d : m->devs) {
        uint8_t* frame_out = (d.rank == root && out8) ? out8[di] : nullptr;
        ++di;
        MHIP(m, hipSetDevice(d.device));
        hipStream_t rs = d.render[slot];
        if (d.gathered_valid[slot]) MHIP(m, hipStreamWaitEvent(rs, d.gathered[slot], 0));
        hipStream_t keep = d.ctx->stream;
        d.ctx->stream = rs;
        // a band group's frames are 1/N of a frame each: the auto in-flight count of a tiled
        // batch is 8 (C2 at 1 rank, 64 frames per gather: 24.4 -> 19.6 us per frame against 4,
        // profiles/r02_multi_probe_inflight.log)
        const uint32_t keep_fl = d.ctx->frames_in_flight;
        if (!keep_fl) d.ctx->frames_in_flight = TRT_MAX_FRAMES_IN_FLIGHT;
        // the batch's frames of each band group through the context's frame loop, so they run
        // with its frames in flight (frame f's group v lands at local + (f * G + v) * blk)
        for (uint32_t v = 0; v < G; ++v) {
            const uint32_t g = d.rank * G + v;
            if (!rows[g]) continue;
            trt_params q = group_params(p, band_rows, NG, g);
            q.flags &= ~(TRT_FLAG_COUNT | TRT_FLAG_TIMING);
            q.flags |= TRT_FLAG_DEVICE_PTRS;
            // the root's own groups: rendered in place into the output frames when there are
            // any (no send, no re-interleave), else straight into the gather buffer
            const bool own = d.rank == root;
            uint8_t* dst = d.local[slot] + v * blk;
            size_t stride = G * blk;
            if (own && frame_out) {
                q.flags |= TRT_FLAG_BAND_IN_PLACE;
                dst = frame_out;
                stride = frame_stride;
            } else if (own) {
                dst = d.gather[slot] + (size_t)g * blk;
                stride = NG * blk;
            }
            const int rc = trt_render_frames(d.ctx, &q, ubos, nf, dst, stride, 0);
            if (rc != TRT_OK) {
                d.ctx->stream = keep;
                d.ctx->frames_in_flight = keep_fl;
                return mfail(m, rc, std::string("band render: ") + trt_last_error(d.ctx));
            }
        }
        if (ubos) d.ctx->ubo = ubos[nf - 1];
        d.ctx->stream = keep;
        d.ctx->frames_in_flight = keep_fl;
        MHIP(m, hipEventRecord(d.rendered[slot], rs));
        MHIP(m, hipStreamWaitEvent(d.comm_stream, d.rendered[slot], 0));
    }
    // gather: frame f, group g of rank r lands at gather + (f * NG + g) * blk on the root
    MNCCL(m, ncclGroupStart());
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        for (uint32_t f = 0; f < nf; ++f) {
            if (d.rank != root) {
                for (uint32_t v = 0; v < G; ++v) {
                    const uint32_t g = d.rank * G + v;
                    if (rows[g])
                        MNCCL(m, ncclSend(d.local[slot] + (f * G + v) * blk, (size_t)rows[g] * W * 4, ncclUint8,
                                          (int)root, d.comm, d.comm_stream));
                }
                continue;
            }
            for (uint32_t g = 0; g < NG; ++g)
                if (rows[g] && g / G != root)
                    MNCCL(m, ncclRecv(d.gather[slot] + (f * NG + g) * blk, (size_t)rows[g] * W * 4, ncclUint8,
                                      (int)(g / G), d.comm, d.comm_stream));
        }
    }
    MNCCL(m, ncclGroupEnd());
    size_t li = 0;
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        if (d.rank == root && out8 && out8[li]) {
            MHIP(m, trt::launch_interleave(reinterpret_cast<const uint32_t*>(d.gather[slot]),
                                           reinterpret_cast<uint32_t*>(out8[li]), W, H, band_rows, NG, max_rows, nf,
                                           frame_stride / 4, d.comm_stream, root * G, root * G + G));
        }
        MHIP(m, hipEventRecord(d.gathered[slot], d.comm_stream));
        d.gathered_valid[slot] = true;
        ++li;
    }
    return TRT_OK;
}

// The call's streams fork from each context's current stream and join back into it.
int fork_all(trt_multi* m) {
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        MHIP(m, hipEventRecord(d.fork, d.ctx->stream));
        MHIP(m, hipStreamWaitEvent(d.comm_stream, d.fork, 0));
        for (int s = 0; s < 2; ++s) MHIP(m, hipStreamWaitEvent(d.render[s], d.fork, 0));
    }
    return TRT_OK;
}

int join_all(trt_multi* m) {
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        for (hipStream_t s : {d.render[0], d.render[1], d.comm_stream}) {
            MHIP(m, hipEventRecord(d.join, s));
            MHIP(m, hipStreamWaitEvent(d.ctx->stream, d.join, 0));
        }
    }
    return TRT_OK;
}

} // namespace

extern "C" {

int trt_multi_create(trt_multi** out, const int* devices, uint32_t ndev) {
    if (!out) return TRT_ERR_INVALID;
    *out = nullptr;
    if (!devices || ndev == 0) return TRT_ERR_INVALID;
    trt_multi* m = new (std::nothrow) trt_multi();
    if (!m) return TRT_ERR_OOM;
    m->nranks = ndev;
    m->devs.resize(ndev);
    std::vector<ncclComm_t> comms(ndev, nullptr);
    std::vector<int> devlist(devices, devices + ndev);
    int rc = TRT_OK;
    for (uint32_t i = 0; i < ndev && rc == TRT_OK; ++i) {
        m->devs[i].device = devices[i];
        m->devs[i].rank = i;
        rc = init_dev(m, m->devs[i]);
    }
    if (rc == TRT_OK && ncclCommInitAll(comms.data(), (int)ndev, devlist.data()) != ncclSuccess) rc = TRT_ERR_HIP;
    if (rc != TRT_OK) {
        trt_multi_destroy(m);
        return rc;
    }
    for (uint32_t i = 0; i < ndev; ++i) m->devs[i].comm = comms[i];
    *out = m;
    return TRT_OK;
}

int trt_multi_unique_id(uint8_t* id) {
    if (!id) return TRT_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == TRT_MULTI_ID_BYTES, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return TRT_ERR_HIP;
    std::memcpy(id, &u, sizeof(u));
    return TRT_OK;
}

int trt_multi_create_rank(trt_multi** out, int device, uint32_t nranks, uint32_t rank, const uint8_t* id) {
    if (!out) return TRT_ERR_INVALID;
    *out = nullptr;
    if (!id || nranks == 0 || rank >= nranks) return TRT_ERR_INVALID;
    trt_multi* m = new (std::nothrow) trt_multi();
    if (!m) return TRT_ERR_OOM;
    m->nranks = nranks;
    m->devs.resize(1);
    m->devs[0].device = device;
    m->devs[0].rank = rank;
    int rc = init_dev(m, m->devs[0]);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (rc == TRT_OK && (hipSetDevice(device) != hipSuccess ||
                         ncclCommInitRank(&m->devs[0].comm, (int)nranks, u, (int)rank) != ncclSuccess))
        rc = TRT_ERR_HIP;
    if (rc != TRT_OK) {
        trt_multi_destroy(m);
        return rc;
    }
    *out = m;
    return TRT_OK;
}

int trt_multi_destroy(trt_multi* m) {
    if (!m) return TRT_ERR_INVALID;
    for (auto& d : m->devs) free_dev(d);
    delete m;
    return TRT_OK;
}

const char* trt_multi_last_error(const trt_multi* m) { return m ? m->err.c_str() : "null multi context"; }

uint32_t trt_multi_ranks(const trt_multi* m) { return m ? m->nranks : 0; }

uint32_t trt_multi_local_count(const trt_multi* m) { return m ? (uint32_t)m->devs.size() : 0; }

trt_ctx* trt_multi_context(trt_multi* m, uint32_t local) {
    return (m && local < m->devs.size()) ? m->devs[local].ctx : nullptr;
}

int trt_multi_set_band_groups(trt_multi* m, uint32_t groups_per_rank) {
    if (!m) return TRT_ERR_INVALID;
    if (groups_per_rank < 1 || groups_per_rank > 64)
        return mfail(m, TRT_ERR_INVALID, "trt_multi_set_band_groups: groups_per_rank must be in [1, 64]");
    m->groups = groups_per_rank;
    return TRT_OK;
}

int trt_multi_upload_scene(trt_multi* m, const trt_ubo* ubo, const trt_triangle* tris, uint32_t ntri,
                           const trt_model* models, uint32_t nmodel, const uint8_t* env, uint32_t env_w,
                           uint32_t env_h) {
    if (!m) return TRT_ERR_INVALID;
    m->have_scene = false;
    // 1. rank 0 builds the device bindings from the AoS records (BVH, SoA repack, envmap)
    for (auto& d : m->devs) {
        if (d.rank != 0) continue;
        MTRY(m, d.ctx, trt_upload_scene(d.ctx, ubo, tris, ntri, models, nmodel, env, env_w, env_h));
        trt::SceneHeader h;
        trt::scene_header(d.ctx, h);
        MHIP(m, hipSetDevice(d.device));
        MHIP(m, hipMemcpy(d.scratch, &h, sizeof(h), hipMemcpyHostToDevice));
    }
    // 2. the header, then every binding, broadcast from rank 0 (ncclBroadcast over xGMI)
    MNCCL(m, ncclGroupStart());
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        MNCCL(m, ncclBroadcast(d.scratch, d.scratch, sizeof(trt::SceneHeader), ncclUint8, 0, d.comm, d.comm_stream));
    }
    MNCCL(m, ncclGroupEnd());
    trt::SceneHeader h{};
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        MHIP(m, hipStreamSynchronize(d.comm_stream));
        MHIP(m, hipMemcpy(&h, d.scratch, sizeof(h), hipMemcpyDeviceToHost));
        if (d.rank != 0) MTRY(m, d.ctx, trt::scene_adopt(d.ctx, h));
    }
    MNCCL(m, ncclGroupStart());
    for (int k = 0; k < trt::kSceneBufs; ++k) {
        if (!h.bytes[k]) continue;
        for (auto& d : m->devs) {
            MHIP(m, hipSetDevice(d.device));
            void* p = *trt::scene_buf(d.ctx, k);
            MNCCL(m, ncclBroadcast(p, p, h.bytes[k], ncclUint8, 0, d.comm, d.comm_stream));
        }
    }
    MNCCL(m, ncclGroupEnd());
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        MHIP(m, hipStreamSynchronize(d.comm_stream));
    }
    m->have_scene = true;
    return TRT_OK;
}

int trt_multi_update_ubo(trt_multi* m, const trt_ubo* ubo) {
    if (!m || !ubo) return mfail(m, TRT_ERR_INVALID, "trt_multi_update_ubo: null argument");
    for (auto& d : m->devs) MTRY(m, d.ctx, trt_update_ubo(d.ctx, ubo));
    return TRT_OK;
}

int trt_render_multi(trt_multi* m, const trt_params* p, uint32_t band_rows, int root, uint8_t* const* out8,
                     trt_stats* st) {
    int rc = check_common(m, p, band_rows, root);
    if (rc != TRT_OK) return rc;
    if (root == TRT_ROOT_ROTATE) root = (int)(m->batch_seq % m->nranks);
    const bool dev_out = (p->flags & TRT_FLAG_DEVICE_PTRS) != 0;
    const size_t frame_bytes = (size_t)p->width * p->height * 4;
    // host output: the root renders into its own device frame and copies it out
    std::vector<uint8_t*> outs(m->devs.size(), nullptr);
    size_t li = 0;
    for (auto& d : m->devs) {
        if ((int)d.rank == root && out8 && out8[li]) {
            if (dev_out) {
                outs[li] = out8[li];
            } else {
                if (grow(m, d.device, &d.frame, &d.frame_cap, frame_bytes) != TRT_OK) return TRT_ERR_HIP;
                outs[li] = d.frame;
            }
        }
        ++li;
    }
    if ((rc = fork_all(m)) != TRT_OK) return rc;
    if ((rc = run_batch(m, p, nullptr, 1, band_rows, (uint32_t)root, false, outs.data(), 0)) != TRT_OK) return rc;
    if ((rc = join_all(m)) != TRT_OK) return rc;
    li = 0;
    for (auto& d : m->devs) {
        if (!dev_out && outs[li]) {
            MHIP(m, hipSetDevice(d.device));
            MHIP(m, hipMemcpyAsync(out8[li], outs[li], frame_bytes, hipMemcpyDeviceToHost, d.ctx->stream));
            MHIP(m, hipStreamSynchronize(d.ctx->stream));
        }
        ++li;
    }
    if (st) {
        // Counters: a separate counting pass of every band group (trt_render COUNT), summed over
        // the devices of this process and then over the ranks (ncclAllReduce).
        std::memset(st, 0, sizeof(*st));
        if (p->flags & TRT_FLAG_COUNT) {
            const uint32_t NG = m->nranks * m->groups;
            for (auto& d : m->devs) {
                uint64_t sum[20] = {0};
                for (uint32_t v = 0; v < m->groups; ++v) {
                    trt_params q = group_params(p, band_rows, NG, d.rank * m->groups + v);
                    q.flags &= ~(TRT_FLAG_DEVICE_PTRS | TRT_FLAG_TIMING);
                    trt_stats s{};
                    MTRY(m, d.ctx, trt_render(d.ctx, &q, nullptr, nullptr, &s));
                    const uint64_t vk[20] = {s.primary_rays, s.secondary_rays, s.shadow_rays, s.misses, s.tri_nearest,
                                             s.sphere_tests, s.batch_tests, s.batch_hits, s.tri_tests, s.node_tests,
                                             s.tri_past_a, s.tri_past_u, s.tri_past_v, s.shadow_skipped,
                                             s.skipped_sphere_tests, s.skipped_box_tests, s.skipped_tri_tests,
                                             s.skipped_tri_past_a, s.skipped_tri_past_u, s.skipped_tri_past_v};
                    for (int k = 0; k < 20; ++k) sum[k] += vk[k];
                }
                MHIP(m, hipSetDevice(d.device));
                MHIP(m, hipMemcpy(d.scratch, sum, sizeof(sum), hipMemcpyHostToDevice));
            }
            MNCCL(m, ncclGroupStart());
            for (auto& d : m->devs) {
                MHIP(m, hipSetDevice(d.device));
                MNCCL(m, ncclAllReduce(d.scratch, d.scratch, 20, ncclUint64, ncclSum, d.comm, d.comm_stream));
            }
            MNCCL(m, ncclGroupEnd());
            uint64_t tot[20] = {0};
            auto& d0 = m->devs[0];
            MHIP(m, hipSetDevice(d0.device));
            MHIP(m, hipStreamSynchronize(d0.comm_stream));
            MHIP(m, hipMemcpy(tot, d0.scratch, sizeof(tot), hipMemcpyDeviceToHost));
            for (auto& d : m->devs) {
                MHIP(m, hipSetDevice(d.device));
                MHIP(m, hipStreamSynchronize(d.comm_stream));
            }
            st->primary_rays = tot[0];
            st->secondary_rays = tot[1];
            st->shadow_rays = tot[2];
            st->misses = tot[3];
            st->tri_nearest = tot[4];
            st->sphere_tests = tot[5];
            st->batch_tests = tot[6];
            st->batch_hits = tot[7];
            st->tri_tests = tot[8];
            st->node_tests = tot[9];
            st->tri_past_a = tot[10];
            st->tri_past_u = tot[11];
            st->tri_past_v = tot[12];
            st->shadow_skipped = tot[13];
            st->skipped_sphere_tests = tot[14];
            st->skipped_box_tests = tot[15];
            st->skipped_tri_tests = tot[16];
            st->skipped_tri_past_a = tot[17];
            st->skipped_tri_past_u = tot[18];
            st->skipped_tri_past_v = tot[19];
        }
    }
    return TRT_OK;
}

int trt_render_multi_frames(trt_multi* m, const trt_params* p, const trt_ubo* ubos, uint32_t nframes,
                            uint32_t band_rows, int root, uint32_t frames_per_gather, uint8_t* const* out8,
                            size_t frame_stride) {
    int rc = check_common(m, p, band_rows, root);
    if (rc != TRT_OK) return rc;
    if (!(p->flags & TRT_FLAG_DEVICE_PTRS))
        return mfail(m, TRT_ERR_INVALID, "trt_render_multi_frames: needs TRT_FLAG_DEVICE_PTRS");
    if (p->flags & (TRT_FLAG_COUNT | TRT_FLAG_TIMING))
        return mfail(m, TRT_ERR_INVALID, "trt_render_multi_frames: COUNT/TIMING are trt_render_multi flags");
    if (frame_stride % 4) return mfail(m, TRT_ERR_INVALID, "frame_stride must be a multiple of 4");
    const uint32_t F = std::max(frames_per_gather, 1u);
    if ((rc = fork_all(m)) != TRT_OK) return rc;
    std::vector<uint8_t*> outs(m->devs.size());
    for (uint32_t i0 = 0; i0 < nframes; i0 += F) {
        const uint32_t nf = std::min(F, nframes - i0);
        const uint32_t r = root == TRT_ROOT_ROTATE ? (uint32_t)(m->batch_seq % m->nranks) : (uint32_t)root;
        for (size_t li = 0; li < m->devs.size(); ++li)
            outs[li] = (out8 && out8[li]) ? out8[li] + (size_t)i0 * frame_stride : nullptr;
        if ((rc = run_batch(m, p, ubos ? ubos + i0 : nullptr, nf, band_rows, r, root == TRT_ROOT_ROTATE, outs.data(),
                            frame_stride)) != TRT_OK)
            return rc;
    }
    return join_all(m);
}

int trt_multi_synchronize(trt_multi* m) {
    if (!m) return TRT_ERR_INVALID;
    for (auto& d : m->devs) {
        MHIP(m, hipSetDevice(d.device));
        MHIP(m, hipStreamSynchronize(d.ctx->stream));
    }
    return TRT_OK;
}

} // extern "C"
