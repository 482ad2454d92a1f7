// trt_multi.cpp — frames row-tiled over the GPUs of a node, gathered over RCCL (xGMI).
//
// The reference renders every frame on one GPU through one VkQueue (main.cpp:722-724,
// dispatch main.cpp:2108-2131, submit main.cpp:2181-2205).  Here a frame's rows are dealt to
// the devices in interleaved bands (row y belongs to band group (y / B) % G_total, so the
// costly image centre is spread over every device: trt_bands.h), each device traces its band
// groups of a batch of frames with the single-GPU kernel (multi-frame launches with band_*
// params) into compact RGBA8 buffers, one grouped ncclSend / ncclRecv moves every frame's
// compact buffers to that frame's root (the plan of band_plan.cpp: frame i's root is rank
// i % N when the root rotates, so every device's links ingest at once), and a re-interleave
// kernel writes the frames there.  The root traces its own bands straight into its frames
// (in place), so they never travel.  The scene is uploaded once on rank 0 and broadcast
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
//
// Failure handling: every argument check and every allocation happens before a collective,
// and allocations are agreed on by all ranks (a status all-reduce), so one rank's failure is
// every rank's error instead of a hang.  An RCCL group is always closed (NcclGroup).  A failure
// inside a collective section leaves the communicators aborted and the context unusable.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/trt/abi.h"
#include "band_plan.h"
#include "trt_ctx.h"

namespace trt {
hipError_t launch_interleave(const uint32_t* gather, uint32_t* out, uint32_t width, uint32_t height,
                             uint32_t band_rows, uint32_t groups, uint32_t groups_per_rank, uint32_t max_rows,
                             uint32_t nframes, size_t frame_stride_px, hipStream_t stream, uint32_t skip_lo,
                             uint32_t skip_hi);
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
        uint8_t* gather[2] = {nullptr, nullptr}; // the compact buffers of the frames it roots
        size_t gather_cap[2] = {0, 0};
        uint8_t* frame = nullptr; // trt_render_multi with host output: the root's frame
        size_t frame_cap = 0;
        void* scratch = nullptr;  // scene header / counters / status words
    };
    std::vector<Dev> devs;
    uint32_t nranks = 1;
    uint32_t groups = 1; // band groups per rank
    uint64_t batch_seq = 0;
    uint64_t frame_seq = 0; // frames of trt_render_multi (its rotating root)
    bool have_scene = false;
    bool self_gather = false;
    bool broken = false; // a collective failed midway: the communicators are aborted
    size_t frame_agreed = 0; // host-output frame bytes every rank's devices hold (agreed)
    // Test hook (TRT_TEST_FAIL_GROW=k at creation): the k-th buffer growth of this context
    // fails as if hipMalloc had, so tests can drive the failure paths on one GPU.
    uint32_t grow_calls = 0, fail_grow_at = 0;
    int open_groups = 0; // RCCL groups opened by this context and not yet closed
    std::string err;
};

namespace {

// Failure injection (tests only): TRT_TEST_FAIL_GROW=k makes the k-th buffer growth of a new
// context fail, but only together with the test-only switch TRT_ENABLE_TEST_HOOKS=1, so a
// deployment that happens to set the first variable gets no injected failures.
uint32_t test_fail_grow_at() {
    const char* on = std::getenv("TRT_ENABLE_TEST_HOOKS");
    if (!on || std::strcmp(on, "1") != 0) return 0;
    const char* e = std::getenv("TRT_TEST_FAIL_GROW");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
}

constexpr size_t kScratchBytes = 4096;
static_assert(sizeof(trt::SceneHeader) <= kScratchBytes, "scene header fits the scratch buffer");

int mfail(trt_multi* m, int code, const std::string& msg) {
    if (m) m->err = msg;
    return code;
}

// A failure inside a collective section: other ranks may be blocked in the collective, so the
// communicators are aborted (their pending operations fail instead of waiting forever) and the
// context refuses further work.
int poison(trt_multi* m, int code, const std::string& msg) {
    // close the open group (if any) before the communicators it references go away
    for (; m->open_groups > 0; --m->open_groups) (void)ncclGroupEnd();
    for (auto& d : m->devs)
        if (d.comm) {
            (void)ncclCommAbort(d.comm);
            d.comm = nullptr;
        }
    m->broken = true;
    return mfail(m, code, msg + " (communicators aborted; destroy this context)");
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
// inside a collective section (a group is open, or peers wait on this rank)
#define CHIP(m, expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return poison((m), TRT_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define CNCCL(m, expr)                                                                           \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) return poison((m), TRT_ERR_HIP, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)
#define MTRY(m, ctx, expr)                                                                       \
    do {                                                                                         \
        int rc_ = (expr);                                                                        \
        if (rc_ != TRT_OK) return mfail((m), rc_, std::string(#expr ": ") + trt_last_error(ctx)); \
    } while (0)

// An RCCL group that is closed on every path out of its scope (poison() closes it first when
// it aborts the communicators).
struct NcclGroup {
    trt_multi* m;
    bool open = false;
    explicit NcclGroup(trt_multi* mm) : m(mm) {}
    ncclResult_t start() {
        const ncclResult_t r = ncclGroupStart();
        open = r == ncclSuccess;
        if (open) ++m->open_groups;
        return r;
    }
    ncclResult_t end() {
        open = false;
        --m->open_groups;
        return ncclGroupEnd();
    }
    ~NcclGroup() {
        if (open && m->open_groups > 0) {
            --m->open_groups;
            (void)ncclGroupEnd();
        }
    }
};

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
    for (hipStream_t s : {d.comm_stream, d.render[0], d.render[1]}) MHIP(m, trt::touch_stream(s, d.scratch));
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

// Grows *p to `bytes` (the device is synchronized first: an in-flight batch may read the old
// buffer).  Returns false on failure (error text in m->err).
bool grow(trt_multi* m, int device, uint8_t** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap && *p) return true;
    if (m->fail_grow_at && ++m->grow_calls == m->fail_grow_at) {
        (void)hipSetDevice(device);
        (void)hipDeviceSynchronize();
        (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
        m->err = "multi-GPU buffer allocation: injected failure (TRT_TEST_FAIL_GROW)";
        return false;
    }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) {
        (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
        e = hipMalloc(reinterpret_cast<void**>(p), bytes);
    }
    if (e != hipSuccess) {
        m->err = std::string("multi-GPU buffer allocation: ") + hipGetErrorString(e);
        return false;
    }
    *cap = bytes;
    return true;
}

// Frees both slots of a device's batch and gather buffers (capacities 0).
void release_batch_buffers(trt_multi::Dev& d) {
    if (hipSetDevice(d.device) == hipSuccess) (void)hipDeviceSynchronize();
    for (int s = 0; s < 2; ++s) {
        (void)hipFree(d.local[s]);
        (void)hipFree(d.gather[s]);
        d.local[s] = d.gather[s] = nullptr;
        d.local_cap[s] = d.gather_cap[s] = 0;
    }
}

// Sum over every device of every rank of `local` (one int per device of this process); the
// collective that makes a local failure everybody's error.  Runs on the comm streams.
int agree(trt_multi* m, const std::vector<int>& local, int& total) {
    {
        NcclGroup grp(m);
        CNCCL(m, grp.start());
        for (size_t i = 0; i < m->devs.size(); ++i) {
            auto& d = m->devs[i];
            CHIP(m, hipSetDevice(d.device));
            int32_t* w = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(d.scratch) + kScratchBytes - 64);
            CHIP(m, hipMemcpyAsync(w, &local[i], sizeof(int32_t), hipMemcpyHostToDevice, d.comm_stream));
            CNCCL(m, ncclAllReduce(w, w, 1, ncclInt32, ncclSum, d.comm, d.comm_stream));
        }
        CNCCL(m, grp.end());
    }
    total = 0;
    auto& d0 = m->devs[0];
    CHIP(m, hipSetDevice(d0.device));
    int32_t v = 0;
    CHIP(m, hipMemcpyAsync(&v, static_cast<uint8_t*>(d0.scratch) + kScratchBytes - 64, sizeof(v), hipMemcpyDeviceToHost,
                           d0.comm_stream));
    for (auto& d : m->devs) {
        CHIP(m, hipSetDevice(d.device));
        CHIP(m, hipStreamSynchronize(d.comm_stream));
    }
    total = v;
    return TRT_OK;
}

// Band parameters of global band group g (of NG).
trt_params group_params(const trt_params* p, uint32_t band_rows, uint32_t NG, uint32_t g) {
    trt_params q = *p;
    q.flags |= TRT_FLAG_DEVICE_PTRS;
    q.flags &= ~TRT_FLAG_BAND_IN_PLACE;
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
    if (m->broken) return mfail(m, TRT_ERR_HIP, "multi context unusable after a failed collective: " + m->err);
    if (!p) return mfail(m, TRT_ERR_INVALID, "null params");
    if (!m->have_scene) return mfail(m, TRT_ERR_NOSCENE, "no scene uploaded (trt_multi_upload_scene)");
    if (band_rows == 0) return mfail(m, TRT_ERR_INVALID, "band_rows must be >= 1");
    if (p->band_rows && p->band_count > 1)
        return mfail(m, TRT_ERR_INVALID, "params must describe the whole frame (band_* = 0)");
    if (p->rays_in) return mfail(m, TRT_ERR_INVALID, "rays_in replay is a single-GPU (trt_render) feature");
    if (p->width == 0 || p->height == 0) return mfail(m, TRT_ERR_INVALID, "empty frame");
    if (root != TRT_ROOT_ROTATE && (root < 0 || (uint32_t)root >= m->nranks))
        return mfail(m, TRT_ERR_INVALID, "root must be a rank or TRT_ROOT_ROTATE");
    return TRT_OK;
}

// One batch of `nf` frames (frame f's root: trt_frame_root(rot0 + f, N, root)).  Every local
// device traces its band groups of every frame (render stream of the slot) — a frame it roots
// straight into out8[local] + f * frame_stride, the others compactly into its batch buffer —
// the plan's transfers move the compact buffers to the roots over RCCL (communication stream),
// and each root re-interleaves its frames.  out8[local] may be null: that device's frames are
// not written.
int run_batch(trt_multi* m, const trt_params* p, const trt_ubo* ubos, uint32_t nf, uint32_t band_rows, int root,
              uint32_t rot0, uint8_t* const* out8, size_t frame_stride) {
    const uint32_t N = m->nranks, G = m->groups;
    const uint32_t W = p->width, H = p->height;
    trt_band_layout L{};
    std::vector<trt_band_xfer> plan;
    if (trt::build_band_plan(W, H, band_rows, N, G, rot0, nf, root, m->self_gather ? TRT_PLAN_SELF_GATHER : 0u, L,
                             &plan) != TRT_OK)
        return mfail(m, TRT_ERR_INVALID, "band plan: invalid batch");
    const uint32_t NG = L.groups;
    const size_t blk = L.block_bytes;
    const int slot = (int)(m->batch_seq & 1u);
    ++m->batch_seq;
    // Buffers: every device sizes its batch buffer and a gather buffer for a root of every frame
    // (so the decision depends only on the batch shape, the same on every rank), both slots
    // together; when anything grows the ranks agree on the outcome before the first collective.
    // The decision looks at both slots of both buffers, and a failed agreement frees them on
    // every rank, so after a failure every rank grows (and agrees) again on the next call: the
    // ranks' capacities never diverge (a half-grown slot would be traced into or skip the
    // all-reduce its peers enter).
    const size_t need_local = L.local_bytes, need_gather = (size_t)nf * NG * blk;
    bool grows = false;
    for (auto& d : m->devs)
        for (int s = 0; s < 2; ++s)
            grows = grows || need_local > d.local_cap[s] || need_gather > d.gather_cap[s] ||
                    (need_local && !d.local[s]) || (need_gather && !d.gather[s]);
    if (grows) {
        std::vector<int> bad(m->devs.size(), 0);
        std::string why;
        for (size_t i = 0; i < m->devs.size(); ++i) {
            auto& d = m->devs[i];
            for (int s = 0; s < 2 && !bad[i]; ++s)
                if (!grow(m, d.device, &d.local[s], &d.local_cap[s], need_local) ||
                    !grow(m, d.device, &d.gather[s], &d.gather_cap[s], need_gather)) {
                    bad[i] = 1;
                    why = m->err;
                }
        }
        int total = 0;
        const int rc = agree(m, bad, total);
        if (rc != TRT_OK) return rc;
        if (total) {
            for (auto& d : m->devs) release_batch_buffers(d);
            return mfail(m, TRT_ERR_OOM, why.empty() ? "a peer rank failed to allocate its batch buffers" : why);
        }
    }
    std::vector<uint32_t> froot(nf), fslot, fj;
    for (uint32_t f = 0; f < nf; ++f) froot[f] = trt_frame_root(rot0 + f, N, root);
    trt::band_plan_slots(N, rot0, nf, root, fslot, fj);
    // render
    std::vector<trt::FrameOut> fl(nf);
    for (size_t li = 0; li < m->devs.size(); ++li) {
        auto& d = m->devs[li];
        MHIP(m, hipSetDevice(d.device));
        hipStream_t rs = d.render[slot];
        if (d.gathered_valid[slot]) MHIP(m, hipStreamWaitEvent(rs, d.gathered[slot], 0));
        hipStream_t keep = d.ctx->stream;
        d.ctx->stream = rs;
        for (uint32_t v = 0; v < G; ++v) {
            const uint32_t g = d.rank * G + v;
            trt_params q = group_params(p, band_rows, NG, g);
            q.flags &= ~(TRT_FLAG_COUNT | TRT_FLAG_TIMING);
            if (!trt_output_rows(&q)) continue;
            for (uint32_t f = 0; f < nf; ++f) {
                const trt_ubo* u = ubos ? &ubos[f] : nullptr;
                if (froot[f] == d.rank && !m->self_gather) // own frame: in place, never travels
                    fl[f] = trt::FrameOut{u, (out8 && out8[li]) ? out8[li] + (size_t)f * frame_stride : nullptr, true};
                else // frames ordered by root: the J blocks for one root are contiguous
                    fl[f] = trt::FrameOut{u, d.local[slot] + ((size_t)fslot[f] * G + v) * blk, false};
            }
            const int rc = trt::render_frame_list(d.ctx, &q, fl.data(), nf, 0);
            if (rc != TRT_OK) {
                d.ctx->stream = keep;
                // peers are about to enter the exchange with this rank: abort, don't strand them
                return poison(m, rc, std::string("band render: ") + trt_last_error(d.ctx));
            }
        }
        d.ctx->stream = keep;
        MHIP(m, hipEventRecord(d.rendered[slot], rs));
        MHIP(m, hipStreamWaitEvent(d.comm_stream, d.rendered[slot], 0));
    }
    // gather: the plan's transfers (one per sender-root pair), in list order on both ends
    if (!plan.empty()) {
        NcclGroup grp(m);
        CNCCL(m, grp.start());
        for (auto& d : m->devs) {
            CHIP(m, hipSetDevice(d.device));
            for (const trt_band_xfer& x : plan) {
                if (x.src == d.rank)
                    CNCCL(m, ncclSend(d.local[slot] + x.src_offset, x.bytes, ncclUint8, (int)x.dst, d.comm, d.comm_stream));
                if (x.dst == d.rank)
                    CNCCL(m, ncclRecv(d.gather[slot] + x.dst_offset, x.bytes, ncclUint8, (int)x.src, d.comm, d.comm_stream));
            }
        }
        CNCCL(m, grp.end());
    }
    // re-interleave: a root's frames of the batch are f0, f0 + step, ... (rotation) or all;
    // sender q's blocks of its j-th frame at ((q * J + j) * G + v) * blk
    for (size_t li = 0; li < m->devs.size(); ++li) {
        auto& d = m->devs[li];
        MHIP(m, hipSetDevice(d.device));
        uint32_t f0 = nf, cnt = 0;
        for (uint32_t f = 0; f < nf; ++f)
            if (froot[f] == d.rank) {
                if (f0 == nf) f0 = f;
                ++cnt;
            }
        if (cnt && out8 && out8[li]) {
            const uint32_t step = root == TRT_ROOT_ROTATE ? N : 1u;
            const uint32_t lo = m->self_gather ? 0u : d.rank * G, hi = m->self_gather ? 0u : d.rank * G + G;
            MHIP(m, trt::launch_interleave(reinterpret_cast<const uint32_t*>(d.gather[slot]),
                                           reinterpret_cast<uint32_t*>(out8[li] + (size_t)f0 * frame_stride), W, H,
                                           band_rows, NG, G, L.max_rows, cnt, (size_t)step * frame_stride / 4,
                                           d.comm_stream, lo, hi));
        }
        MHIP(m, hipEventRecord(d.gathered[slot], d.comm_stream));
        d.gathered_valid[slot] = true;
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
    m->fail_grow_at = test_fail_grow_at();
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
    m->fail_grow_at = test_fail_grow_at();
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

int trt_multi_set_self_gather(trt_multi* m, int on) {
    if (!m) return TRT_ERR_INVALID;
    m->self_gather = on != 0;
    return TRT_OK;
}

int trt_multi_upload_scene(trt_multi* m, const trt_ubo* ubo, const trt_triangle* tris, uint32_t ntri,
                           const trt_model* models, uint32_t nmodel, const uint8_t* env, uint32_t env_w,
                           uint32_t env_h) {
    if (!m) return TRT_ERR_INVALID;
    if (m->broken) return mfail(m, TRT_ERR_HIP, "multi context unusable after a failed collective: " + m->err);
    m->have_scene = false;
    // 1. rank 0 builds the device bindings from the AoS records (BVH, SoA repack, envmap); a
    //    failure there travels as a header with magic 0, so every rank returns an error
    int rc0 = TRT_OK;
    std::string why;
    for (auto& d : m->devs) {
        if (d.rank != 0) continue;
        trt::SceneHeader h{};
        rc0 = trt_upload_scene(d.ctx, ubo, tris, ntri, models, nmodel, env, env_w, env_h);
        if (rc0 == TRT_OK) trt::scene_header(d.ctx, h);
        else why = std::string("trt_upload_scene on rank 0: ") + trt_last_error(d.ctx);
        MHIP(m, hipSetDevice(d.device));
        MHIP(m, hipMemcpy(d.scratch, &h, sizeof(h), hipMemcpyHostToDevice));
    }
    // 2. the header broadcast from rank 0 (ncclBroadcast over xGMI)
    {
        NcclGroup grp(m);
        CNCCL(m, grp.start());
        for (auto& d : m->devs) {
            CHIP(m, hipSetDevice(d.device));
            CNCCL(m, ncclBroadcast(d.scratch, d.scratch, sizeof(trt::SceneHeader), ncclUint8, 0, d.comm, d.comm_stream));
        }
        CNCCL(m, grp.end());
    }
    trt::SceneHeader h{};
    std::vector<int> bad(m->devs.size(), 0);
    for (size_t i = 0; i < m->devs.size(); ++i) {
        auto& d = m->devs[i];
        CHIP(m, hipSetDevice(d.device));
        CHIP(m, hipStreamSynchronize(d.comm_stream));
        CHIP(m, hipMemcpy(&h, d.scratch, sizeof(h), hipMemcpyDeviceToHost));
        if (h.magic != trt::kSceneMagic) return mfail(m, rc0 != TRT_OK ? rc0 : TRT_ERR_INVALID,
                                                      why.empty() ? "rank 0 failed to build the scene" : why);
        if (d.rank != 0 && trt::scene_adopt(d.ctx, h) != TRT_OK) {
            bad[i] = 1;
            why = std::string("scene adoption: ") + trt_last_error(d.ctx);
        }
    }
    // 3. every rank agrees that every device holds buffers for the bindings
    int total = 0;
    const int rc = agree(m, bad, total);
    if (rc != TRT_OK) return rc;
    if (total) return mfail(m, TRT_ERR_OOM, why.empty() ? "a peer rank failed to allocate the scene" : why);
    // 4. every binding broadcast from rank 0
    {
        NcclGroup grp(m);
        CNCCL(m, grp.start());
        for (int k = 0; k < trt::kSceneBufs; ++k) {
            if (!h.bytes[k]) continue;
            for (auto& d : m->devs) {
                CHIP(m, hipSetDevice(d.device));
                void* p = *trt::scene_buf(d.ctx, k);
                CNCCL(m, ncclBroadcast(p, p, h.bytes[k], ncclUint8, 0, d.comm, d.comm_stream));
            }
        }
        CNCCL(m, grp.end());
    }
    for (auto& d : m->devs) {
        CHIP(m, hipSetDevice(d.device));
        CHIP(m, hipStreamSynchronize(d.comm_stream));
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
    const uint32_t r = trt_frame_root((uint32_t)(m->frame_seq++ % m->nranks), m->nranks, root);
    const bool dev_out = (p->flags & TRT_FLAG_DEVICE_PTRS) != 0;
    const size_t frame_bytes = (size_t)p->width * p->height * 4;
    // host output: the root renders into its own device frame and copies it out.  Every rank
    // may root a frame (rotation), so every device holds that frame buffer, and its growth is
    // agreed on by all ranks before the exchange (the same decision on every rank: the frame
    // size and the output mode, not who roots this frame).
    if (!dev_out && frame_bytes > m->frame_agreed) {
        std::vector<int> bad(m->devs.size(), 0);
        std::string why;
        for (size_t li = 0; li < m->devs.size(); ++li)
            if (!grow(m, m->devs[li].device, &m->devs[li].frame, &m->devs[li].frame_cap, frame_bytes)) {
                bad[li] = 1;
                why = m->err;
            }
        int total = 0;
        if ((rc = agree(m, bad, total)) != TRT_OK) return rc;
        if (total) {
            for (auto& d : m->devs) {
                if (hipSetDevice(d.device) == hipSuccess) (void)hipDeviceSynchronize();
                (void)hipFree(d.frame);
                d.frame = nullptr;
                d.frame_cap = 0;
            }
            m->frame_agreed = 0;
            return mfail(m, TRT_ERR_OOM, why.empty() ? "a peer rank failed to allocate its frame buffer" : why);
        }
        m->frame_agreed = frame_bytes;
    }
    std::vector<uint8_t*> outs(m->devs.size(), nullptr);
    for (size_t li = 0; li < m->devs.size(); ++li) {
        auto& d = m->devs[li];
        if (d.rank == r && out8 && out8[li]) outs[li] = dev_out ? out8[li] : d.frame;
    }
    if ((rc = fork_all(m)) != TRT_OK) return rc;
    if ((rc = run_batch(m, p, nullptr, 1, band_rows, (int)r, 0, outs.data(), 0)) != TRT_OK) return rc;
    if ((rc = join_all(m)) != TRT_OK) return rc;
    for (size_t li = 0; li < m->devs.size(); ++li) {
        auto& d = m->devs[li];
        if (!dev_out && outs[li]) {
            MHIP(m, hipSetDevice(d.device));
            MHIP(m, hipMemcpyAsync(out8[li], outs[li], frame_bytes, hipMemcpyDeviceToHost, d.ctx->stream));
            MHIP(m, hipStreamSynchronize(d.ctx->stream));
        }
    }
    if (st) {
        // Counters: a separate counting pass of every band group (trt_render COUNT), summed over
        // the devices of this process and then over the ranks (ncclAllReduce).
        std::memset(st, 0, sizeof(*st));
        if (p->flags & TRT_FLAG_COUNT) {
            const uint32_t NG = m->nranks * m->groups;
            // word 20: local failures (a failed counting pass still joins the all-reduce)
            std::string why;
            for (auto& d : m->devs) {
                uint64_t sum[21] = {0};
                for (uint32_t v = 0; v < m->groups && !sum[20]; ++v) {
                    trt_params q = group_params(p, band_rows, NG, d.rank * m->groups + v);
                    q.flags &= ~(TRT_FLAG_DEVICE_PTRS | TRT_FLAG_TIMING);
                    trt_stats s{};
                    if (trt_render(d.ctx, &q, nullptr, nullptr, &s) != TRT_OK) {
                        sum[20] = 1;
                        why = std::string("counting pass: ") + trt_last_error(d.ctx);
                        break;
                    }
                    const uint64_t vk[20] = {s.primary_rays, s.secondary_rays, s.shadow_rays, s.misses, s.tri_nearest,
                                             s.sphere_tests, s.batch_tests, s.batch_hits, s.tri_tests, s.node_tests,
                                             s.tri_past_a, s.tri_past_u, s.tri_past_v, s.shadow_skipped,
                                             s.skipped_sphere_tests, s.skipped_box_tests, s.skipped_tri_tests,
                                             s.skipped_tri_past_a, s.skipped_tri_past_u, s.skipped_tri_past_v};
                    for (int k = 0; k < 20; ++k) sum[k] += vk[k];
                }
                CHIP(m, hipSetDevice(d.device));
                CHIP(m, hipMemcpy(d.scratch, sum, sizeof(sum), hipMemcpyHostToDevice));
            }
            {
                NcclGroup grp(m);
                CNCCL(m, grp.start());
                for (auto& d : m->devs) {
                    CHIP(m, hipSetDevice(d.device));
                    CNCCL(m, ncclAllReduce(d.scratch, d.scratch, 21, ncclUint64, ncclSum, d.comm, d.comm_stream));
                }
                CNCCL(m, grp.end());
            }
            uint64_t tot[21] = {0};
            auto& d0 = m->devs[0];
            CHIP(m, hipSetDevice(d0.device));
            CHIP(m, hipStreamSynchronize(d0.comm_stream));
            CHIP(m, hipMemcpy(tot, d0.scratch, sizeof(tot), hipMemcpyDeviceToHost));
            for (auto& d : m->devs) {
                CHIP(m, hipSetDevice(d.device));
                CHIP(m, hipStreamSynchronize(d.comm_stream));
            }
            if (tot[20]) return mfail(m, TRT_ERR_HIP, why.empty() ? "a peer rank's counting pass failed" : why);
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
    const uint32_t F = std::min(std::max(frames_per_gather, 1u), TRT_MAX_FRAME_BATCH);
    if (m->nranks == 1 && !m->self_gather) {
        // One rank: nothing travels and nothing is re-interleaved, so the tiled loop is the frame
        // loop — each band group traced in place on the context's stream, no batch streams, no
        // events (each cross-stream hop costs ~10 us of GPU latency and a few HIP calls).
        auto& d = m->devs[0];
        const uint32_t NG = m->groups;
        std::vector<trt::FrameOut> fl(nframes);
        for (uint32_t v = 0; v < NG; ++v) {
            trt_params q = group_params(p, band_rows, NG, v);
            q.flags &= ~(TRT_FLAG_COUNT | TRT_FLAG_TIMING);
            if (!trt_output_rows(&q)) continue;
            for (uint32_t i = 0; i < nframes; ++i)
                fl[i] = trt::FrameOut{ubos ? &ubos[i] : nullptr,
                                      (out8 && out8[0]) ? out8[0] + (size_t)i * frame_stride : nullptr, NG > 1};
            if ((rc = trt::render_frame_list(d.ctx, &q, fl.data(), nframes, 0)) != TRT_OK)
                return mfail(m, rc, std::string("band render: ") + trt_last_error(d.ctx));
        }
        return TRT_OK;
    }
    if ((rc = fork_all(m)) != TRT_OK) return rc;
    std::vector<uint8_t*> outs(m->devs.size());
    for (uint32_t i0 = 0; i0 < nframes; i0 += F) {
        const uint32_t nf = std::min(F, nframes - i0);
        for (size_t li = 0; li < m->devs.size(); ++li)
            outs[li] = (out8 && out8[li]) ? out8[li] + (size_t)i0 * frame_stride : nullptr;
        if ((rc = run_batch(m, p, ubos ? ubos + i0 : nullptr, nf, band_rows, root, i0, outs.data(), frame_stride)) !=
            TRT_OK)
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
