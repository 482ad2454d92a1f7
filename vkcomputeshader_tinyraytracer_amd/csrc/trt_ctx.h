// trt_ctx.h — the context behind the C-ABI's opaque trt_ctx (internal to libtrt).
//
// Shared by trt_runtime.cpp (the single-GPU ABI) and trt_multi.cpp (the multi-GPU frame
// tiling over RCCL, which broadcasts a context's scene bindings to the other devices).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/trt/abi.h"
#include "trt_device.h"

// Frames-in-flight slots of a context: a private build-time knob (the public
// TRT_MAX_FRAMES_IN_FLIGHT of abi.h is fixed and bounds it).
#ifndef TRT_BUILD_MAX_IN_FLIGHT
#define TRT_BUILD_MAX_IN_FLIGHT TRT_MAX_FRAMES_IN_FLIGHT
#endif
static_assert(TRT_BUILD_MAX_IN_FLIGHT >= 1u && TRT_BUILD_MAX_IN_FLIGHT <= TRT_MAX_FRAMES_IN_FLIGHT,
              "TRT_BUILD_MAX_IN_FLIGHT must lie in [1, TRT_MAX_FRAMES_IN_FLIGHT]");

struct trt_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    trt_ubo ubo{};
    bool have_scene = false;

    trt::BatchRec* d_batches = nullptr;
    float4* d_nodes = nullptr; // implicit 8-ary hierarchy over the batches
    trt::BvhNode* d_bvh = nullptr;  // per-ray BVH over the triangles (null: batch walk only)
    trt::Bvh4Node* d_bvh4 = nullptr; // the same, 4-wide
    trt::Bvh4QNode* d_bvh4q = nullptr; // the same, 4-wide with quantized child boxes
    trt::TriGeo* d_bvh_tris = nullptr;
    uint32_t node_off[11] = {0};
    uint32_t top = 0;
    trt::TriGeo* d_geo = nullptr;
    trt::TriShade* d_shade = nullptr;
    trt::Mat* d_mats = nullptr;
    uint32_t* d_env = nullptr;
    // envmap footprint layout derived from d_env (trt_kernel.hip env_fetch): (H + 2) x (W + 3)
    // texel pairs, rebuilt lazily before the first render after d_env changes
    uint2* d_envp = nullptr;
    size_t envp_cap = 0;
    bool envp_ok = false;
    uint32_t nbatch = 0, ntri = 0, nmat = 0, env_w = 0, env_h = 0;

    void* d_out8 = nullptr;
    size_t cap8 = 0;
    void* d_out32 = nullptr;
    size_t cap32 = 0;
    void* d_rays = nullptr;
    size_t caprays = 0;
    unsigned long long* d_counters = nullptr;
    uint32_t num_cus = 256;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::vector<hipEvent_t> fev; // per-launch event pairs of the last timed trt_render_frames
    std::vector<uint32_t> fev_nframes; // frames traced by each timed launch
    uint32_t frames_in_flight = TRT_FRAMES_IN_FLIGHT_DEFAULT;
    uint32_t frame_batch = TRT_FRAME_BATCH_AUTO; // frames per launch of a plain frame loop
    // block -> tile dealing of multi-frame launches (trt_kernel.hip xcd_tile): rotation of the
    // XCD chunk classes every 2^(xcd_rot - 1) frames (0 = fixed), per-chunk-row skew (0 = none);
    // TRT_XCD_ROT / TRT_XCD_SKEW env
    uint32_t xcd_rot = trt::kDefaultXcdRot, xcd_skew = trt::kDefaultXcdSkew, xcd_inter = trt::kDefaultXcdInter;
    int frame_group = -1; // TRT_FRAME_GROUP (1 or 2); -1 = auto: 2 for triangle-free scenes, else 1
    int bvh_waves4 = -1; // TRT_BVH_WAVES4 env: 0 / 1 forces the BVH build, -1 = by scene size
    uint32_t defer_in_flight = 16; // auto frames in flight of deferred-shadow loops (TRT_DEFER_IN_FLIGHT env)
    bool defer_in_flight_set = false; // TRT_DEFER_IN_FLIGHT given: it shapes the loop at every queue count (defer_shape)
    // frames per deferred launch group of a frame loop: TRT_DEFER_GROUP env, 0 = auto (by the
    // hardware queues: render_frame_list)
    uint32_t defer_inter = 2;   // TRT_DEFER_INTER: a frame group's blocks dealt frame by frame: 0 = off, 1 = pass A, 2 = passes A, B, C
    uint32_t defer_group = 0;
    // hardware queues HIP gives this process: GPU_MAX_HW_QUEUES at trt_create (HIP's default 4
    // when unset); the library only reads it
    uint32_t hw_queues = 4;
    int subtree_split = TRT_SPLIT_AUTO;
    int deferred_shadows = TRT_DEFER_AUTO;
    // pass-A waves per tile of a deferred frame: 0 = auto (2 when <= 4 frames overlap, else 1),
    // TRT_DEFER_PPW = 64 / 32 / 16 pixels per wave forces 1 / 2 / 4
    uint32_t defer_sub = 0;
    uint32_t cur_in_flight = 1; // frames in flight of the current render call
    bool spp_lanes = true;      // spp > 1 frames: one lane per sample (TRT_SPP_LANES)
    // Subtree-split scratch, one set per frames-in-flight slot (concurrent frames must not share
    // task queues): two task queues, per-pixel fixed-point colours, the split-pixel list and
    // the counters.
    struct SplitBufs {
        trt::Task* q[2] = {nullptr, nullptr};
        uint32_t* qlink[2] = {nullptr, nullptr}; // deferred split: LINK slot per task
        unsigned long long* acc = nullptr;
        uint32_t* spilled = nullptr;
        trt::SplitCtr* ctr = nullptr;
        size_t npx = 0;  // pixels the buffers hold
        uint32_t cap = 0; // tasks per queue
        // Deferred-shadow scratch (trt_set_deferred_shadows): event chunks, the shadow query
        // queue, per-pixel tree roots, the fallback list and the counters.
        float4* ev = nullptr;
        float4* shq = nullptr;
        uint2* px_ev = nullptr;
        uint32_t* fb = nullptr;
        trt::DeferCtr* dctr = nullptr;
        size_t ev_chunks = 0, shq_cap = 0, dnpx = 0;
        uint32_t dframes = 0; // frames the deferred scratch holds (a launch group), each of the sizes above
        // per-stripe capacities the slot's last deferred frame ran with (trt_defer_stats)
        size_t used_ev_cap = 0, used_shq_cap = 0;
        // The stream of the slot's last frame and an event after it: a frame on another
        // stream waits for it before reusing the scratch (trt_render on alternating
        // streams, e.g. dist.PipelinedTiles, must not race on the task queues).
        hipStream_t last = nullptr;
        hipEvent_t done = nullptr;
    };
    SplitBufs split[TRT_BUILD_MAX_IN_FLIGHT];
    hipStream_t render_slot_stream[TRT_BUILD_MAX_IN_FLIGHT] = {}; // trt_render: stream -> slot (LRU)
    uint32_t render_slot_next = 0;
    std::vector<hipStream_t> aux; // frames-in-flight streams (frame i -> stream i % n)
    std::vector<hipEvent_t> aux_ev;
    hipEvent_t fork_ev = nullptr;
    uint32_t fev_frames = 0;
    // bytes of each scene binding on the device (trt::kSceneBuf* order), for the broadcast
    size_t scene_bytes[10] = {0};
    void* diag = nullptr; // diagnostic builds: ray-dump buffer (trt_diag_set_buffer)
};

namespace trt {

// A 4-byte fill on a new stream (then a sync), so its hardware queue is created now instead of
// at its first frame.
hipError_t touch_stream(hipStream_t s, void* scratch);

// One frame of a frame loop: its UBO (null: the context's current one), its RGBA8 image (a
// device pointer, or null) and whether a band launch writes its rows at their frame rows.
struct FrameOut {
    const trt_ubo* ubo;
    uint8_t* out8;
    bool in_place;
};
// The frame loop behind trt_render_frames and the multi-GPU band renders: plain frames go
// out as multi-frame launches (up to kMaxLaunchFrames frames sharing everything but camPos and
// the output), split / deferred-shadow frames one launch sequence per frame; launches rotate
// over the frames-in-flight streams forked from and joined back into the context's stream.
// Only enqueues.  time_every > 0: HIP events bracket every time_every-th launch.
int render_frame_list(trt_ctx* c, const trt_params* p, const FrameOut* frames, uint32_t n, uint32_t time_every);

// The scene bindings of a context in a fixed order (the RCCL scene broadcast walks them).
enum SceneBuf : int {
    kSceneBatches = 0, kSceneNodes, kSceneBvh, kSceneBvh4, kSceneBvhTris, kSceneGeo, kSceneShade,
    kSceneMats, kSceneEnv, kSceneBvh4Q, kSceneBufs
};
static_assert(kSceneBufs == sizeof(trt_ctx::scene_bytes) / sizeof(size_t), "one byte count per scene binding");
void** scene_buf(trt_ctx* c, int k);

// Everything besides the device buffers that trt_upload_scene derives (fixed size, broadcast
// as bytes from the root device to the others).
struct SceneHeader {
    uint32_t magic;
    uint32_t nbatch, ntri, nmat, env_w, env_h, top, pad;
    uint32_t node_off[11];
    uint32_t pad2;
    uint64_t bytes[kSceneBufs];
    trt_ubo ubo;
};
constexpr uint32_t kSceneMagic = 0x54525453u; // "STRT"

// Fills h from a context with an uploaded scene.
void scene_header(const trt_ctx* c, SceneHeader& h);
// Drops c's scene and allocates empty device buffers of h's sizes (filled by the caller,
// e.g. by ncclBroadcast), then adopts h's scalars.  Returns TRT_OK or an error code.
int scene_adopt(trt_ctx* c, const SceneHeader& h);

} // namespace trt
