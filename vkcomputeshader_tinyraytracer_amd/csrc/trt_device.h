// trt_device.h — device-side data layout and launch arguments of the CDNA4 tracer.
//
// The reference binds AoS std140 records (Triangle 144 B, Model 96 B; shader.comp:19-38)
// and reads a whole 144-byte Triangle per test (shader.comp:345).  On gfx950 the hot loops
// are wave-uniform walks over batches and their triangles, so the layouts below are
// shaped for the SCALAR memory path: one batch record (32 B) and one triangle geometry
// record (48 B) are each a single s_load_dwordx8 / dwordx4 stream shared by the 64 lanes,
// and everything a test does not need (materials, vertex normals) lives in separate
// arrays read once per closest hit.
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

namespace trt {

// One AABB batch (Model, shader.comp:29-38): bbox + triangle range + smooth flag.
struct alignas(32) BatchRec {
    float bmin[3];
    float bmax[3];
    int32_t start;
    int32_t count_ni; // count | (normal_interp != 0) << 31
};
static_assert(sizeof(BatchRec) == 32, "BatchRec is one s_load_dwordx8");

// Triangle geometry for the Moller-Trumbore test: v0 and the two edges, pre-subtracted
// on the host with the same float subtraction the shader performs (shader.comp:230-231).
struct alignas(16) TriGeo {
    float v0[3];
    float e1[3];
    float e2[3];
    float pad[3];
};
static_assert(sizeof(TriGeo) == 48, "TriGeo is 3 x dwordx4");

// Per-triangle shading data, read once per closest hit.
struct alignas(16) TriShade {
    float n0[3];
    float n1[3];
    float n2[3];
    uint32_t material; // index into the deduplicated material table
    uint32_t pad[2];
};
static_assert(sizeof(TriShade) == 48, "TriShade is 3 x dwordx4");

// BVH2 node over triangles (bvh_build.cpp): both children's boxes live in the parent, so a
// visit is one 64 B load and two slab tests.  child[k]: node index, or a leaf
// (kBvhLeafBit | (count - 1) << kBvhCountShift | first) into the BVH-ordered triangle array.
constexpr uint32_t kBvhLeafBit = 0x80000000u;
constexpr uint32_t kBvhCountShift = 27u;
constexpr uint32_t kBvhFirstMask = (1u << kBvhCountShift) - 1u;
constexpr uint32_t kBvhLeafMin = 2u, kBvhLeafMax = 4u; // SAH sweep: profiles/r01_ab_sah.log
constexpr int kBvhSahDepth = 32;  // below this depth only median splits
constexpr int kBvhStack = 64;     // traversal stack >= max depth (32 + log2(2^27))
struct alignas(16) BvhNode {
    float lo0[3], hi0[3], lo1[3], hi1[3];
    uint32_t child[2];
    uint32_t pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode is 64 B");

// 4-wide node collapsed from the BVH2 (bvh_build.cpp): one visit resolves two BVH2 levels,
// halving the dependent node fetches per query.  Child boxes SoA (lo_x[4] ...), 128 B = 8 x
// dwordx4; an unused slot has child == kBvh4None.
constexpr uint32_t kBvh4None = 0xFFFFFFFFu;
// Box of an unused slot: NaN on every axis.  Every slab product is then NaN, the NaN-ignoring
// min/max give tnear = tfar = NaN, and `tnear <= tfar` fails for any ray and any distance bound.
constexpr float kBvh4EmptyCoord = __builtin_nanf("");
struct alignas(16) Bvh4Node {
    float lox[4], loy[4], loz[4];
    float hix[4], hiy[4], hiz[4];
    uint32_t child[4];
    uint32_t pad[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node is 128 B");

// The same 4-wide node with its child boxes quantized to 8 bits per plane (Ylitie et al.,
// "Efficient incoherent ray traversal on GPUs through compressed wide BVHs", HPG 2017): a grid
// of origin p and power-of-two step s = 2^(e - 127) per axis; child i's box is
// [p + qlo_i * s, p + qhi_i * s], rounded outward by at least one step beyond the padded box
// (bvh_build.cpp quantize_bvh4), so it stays conservative.  64 B = 4 x dwordx4 per visit
// instead of 8.  Byte i of qlo[a] / qhi[a] belongs to child i; an unused slot has qlo = 255,
// qhi = 0 on every axis (an inverted box, which the sign-ordered slab test never enters).
struct alignas(16) Bvh4QNode {
    float p[3];
    uint32_t exps;   // e_x | e_y << 8 | e_z << 16 (biased exponents of the steps)
    uint32_t qlo[3]; // per axis, 4 x u8 lower planes
    uint32_t qhi[3]; // per axis, 4 x u8 upper planes
    uint32_t pad[2];
    uint32_t child[4];
};
static_assert(sizeof(Bvh4QNode) == 64, "Bvh4QNode is 64 B");


struct Mat {
    float albedo[4];
    float kd[3];
    float spec_exp;
    float ior;
    float pad[3];
};
static_assert(sizeof(Mat) == 48, "Mat is 48 B");

// Subtree split (trt_set_subtree_split): a segment at a depth-window edge handed to any lane
// of a later launch instead of being traced by its pixel's lane.  32 B = 2 x dwordx4.
struct alignas(16) Task {
    float o[3];
    float dx;
    float dy, dz;
    float thr;
    uint32_t px_depth; // output pixel << 5 | depth
};
static_assert(sizeof(Task) == 32, "Task is 32 B");
constexpr uint32_t kTaskDepthBits = 5u;
constexpr uint32_t kMaxSplitRounds = 20u; // a window of 1 at max_depth 20 (deferred frames)
// Device counters of one frame's split launches (one set per frames-in-flight slot).
struct SplitCtr {
    uint32_t spilled;                  // pixels finished by finalize_spilled
    uint32_t overflow;                 // children traced in place because a queue was full
    uint32_t produced[kMaxSplitRounds + 1]; // tasks written by launch r (0 = the tile kernel)
    uint32_t head[kMaxSplitRounds + 1];     // dequeue head of launch r's output (read by r + 1)
};

// Deferred-shadow frame (trt_set_deferred_shadows).  Pass A traces every pixel's Whitted tree
// without its shadow rays and logs one colour event per traced segment; the shadow queries go
// to one dense queue that pass B traces with every lane busy; pass C sums each pixel's events
// in the reference's pop order.  The events of a pixel form its segment TREE: an event names
// the children its segment made (tag bits) and each child, wherever and whenever it is traced,
// writes its own event's slot into its parent's plane 3 (z = reflection child, w = refraction
// child).  So pass A may trace a pixel's segments in any order and on any lane of the wave (the
// lanes share their pending segments, defer_walk), and pass C walks the tree in the pop order
// of shader.comp:530-575 (node, reflection subtree, refraction subtree).  A chunk holds kEvRows
// events of the 64 lanes of a wave, laid out [row][plane][lane] (4 x 16 B planes per event,
// coalesced across lanes); a slot is (chunk * kEvRows + row) * 64 + lane.
//   plane 0: kd.xyz, tag            (tag & kEvTagConst: xyz = the event's colour term)
//   plane 1: diffuse terms[3], albedo.x
//   plane 2: specular terms[3], albedo.y
//   plane 3: throughput, occluded-light bits (pass B), reflection child, refraction child
constexpr uint32_t kEvRows = 4u;
constexpr uint32_t kEvNone = 0xFFFFFFFFu;      // px_ev.x of a pixel re-traced by defer_fallback
constexpr uint32_t kEvTagConst = 0x80000000u;  // tag bit: colour term known in pass A
constexpr uint32_t kEvTagRefl = 1u << 3;       // tag bit: the segment made a reflection child
constexpr uint32_t kEvTagRefr = 1u << 4;       // tag bit: ... a refraction (or TIR) child
constexpr uint32_t kEvRoot = 0xFFFFFFFFu;      // parent link of a root segment
constexpr uint32_t kMaxTreeDepth = 20u;        // MAX_DEPTH: pass C's stack of refraction children
// The event pool and the query queue are split into kDeferStripes stripes (tile t allocates
// from stripe hash(t), each with its own counter on its own 64-B line): one counter
// for a whole 4K frame serialises ~10^6 wave-aggregated atomics in one L2 channel (measured:
// a 4K depth-4 frame 2.5x slower).  Pass B walks the stripes with a static grid, no atomics.
constexpr uint32_t kDeferStripes = 128u;
constexpr uint32_t kCtrStride = 16u; // uint32 per counter line
struct DeferCtr {
    uint32_t nfb;                                  // pixels handed to defer_fallback
    uint32_t pad[kCtrStride - 1];
    uint32_t chunks[kDeferStripes * kCtrStride];   // [s * kCtrStride]: chunks taken from stripe s
    uint32_t nq[kDeferStripes * kCtrStride];       // [s * kCtrStride]: queries appended to stripe s
};

struct SphereArg {
    float c[3];
    float r;
    Mat m;
};

// One frame of a launch.  A plain frame loop (trt_render_frames) traces up to
// kMaxLaunchFrames frames per launch: block b renders tile b % ntiles of frame b / ntiles, so
// one frame's slow tiles (the glass sphere) overlap the next frame's tiles inside one grid —
// no stream switch, no launch gap, one drain per launch instead of per frame.  The frames of
// a launch share every UBO field but the camera position (the reference's interactive loop
// moves only camPos, main.cpp:391-403, 2165-2179) and each writes its own image.
constexpr uint32_t kMaxLaunchFrames = 64;
// Tile dealing of multi-frame launches (trt_kernel.hip xcd_tile, trt_ctx xcd_rot / xcd_skew)
constexpr uint32_t kDefaultXcdRot = 1, kDefaultXcdSkew = 0, kDefaultXcdInter = 1;
struct FrameRec {
    float cam[3];      // UBO camPos (main.cpp:2170)
    uint32_t in_place; // band launch: rows written at their frame rows (TRT_FLAG_BAND_IN_PLACE)
    uint32_t* out8;    // packed RGBA8 of this frame (binding 3), or null
};
static_assert(sizeof(FrameRec) == 24, "FrameRec is 24 B");

// Kernel arguments: the UBO (binding 0) travels in the kernarg segment, i.e. in SGPRs.
struct KArgs {
    uint32_t width, height;
    uint32_t rows;      // rows this launch renders (compact output rows)
    uint32_t band_rows; // 0 = no banding
    uint32_t band_count, band_index;
    uint32_t max_depth, spp, seed, flags;
    float dz;
    uint32_t nbatch;
    uint32_t nframes;   // frames of this launch (fr[0 .. nframes-1]), >= 1
    float light[3][3];
    SphereArg sph[4];
    const BatchRec* __restrict__ batches;
    const TriGeo* __restrict__ geo;
    const TriShade* __restrict__ shade;
    const Mat* __restrict__ mats;
    const uint32_t* __restrict__ env; // RGBA8 texels
    // Pair rows: entry (r, c) of (env_h + 2) x (env_w + 3) is the texels (x, y0), (x, y1) with
    // x = clamp(c - 1), y0 = clamp(r - 1), y1 = clamp(r): a bilinear footprint is the 16 bytes at
    // (yf + 1, xf + 1) — one load (clamp-to-edge included) instead of two rows' lines.
    const uint2* __restrict__ envp;
    uint32_t env_w, env_h;
    const float* __restrict__ rays_in; // Ray records (8 floats), or null
    float* __restrict__ out32;         // float4 per pixel (rayOut, binding 2; single-frame launches), or null
    unsigned long long* __restrict__ counters; // trt_stats counters, in order (COUNT build)
    const BvhNode* __restrict__ bvh;  // per-lane BVH over triangles, or null (batch walk)
    const Bvh4Node* __restrict__ bvh4; // the same BVH collapsed to 4-wide nodes
    const Bvh4QNode* __restrict__ bvh4q; // ... with quantized child boxes (same node indices)
    const TriGeo* __restrict__ bvh_tris; // BVH-ordered geometry; pad = (triangle, batch, ni)
    const float4* __restrict__ nodes; // batch hierarchy: per node (lo.xyz, -), (hi.xyz, -)
    uint32_t node_off[11];            // first node of level L (L = 1..top) in `nodes`
    uint32_t top;                     // levels above the batches: 8^top >= nbatch
    uint32_t ntx;                     // 8x8 tiles per output row
    uint32_t ntiles;              // 8x8 tiles in the launch
    uint32_t bvh_waves4;          // BVH walk: the 4-waves-per-SIMD build (GEOM 3)
    uint32_t xcd_rot, xcd_skew;   // multi-frame tile dealing (xcd_tile): rotation period, row skew
    uint32_t xcd_inter;           // ... frames interleaved per chunk group (inter_tile); 2: no rotation, permuted classes
    uint32_t xcd_mult;            // ... xcd_inter 2: chunk permutation multiplier (coprime to the dealt chunks)
    uint32_t frame_group;         // ... 2: each workgroup traces its tile in two consecutive frames
    // subtree split: this launch traces depths < split_d1; children at depth split_d1 become
    // tasks (split_d1 >= max_depth: no split).  split_w: the window (0 = split off).
    uint32_t split_w, split_d1;
    uint32_t q_cap;                   // task capacity of each queue
    uint32_t num_cus;
    Task* __restrict__ q_out;         // tasks this launch produces
    const Task* __restrict__ q_in;    // tasks this launch consumes (trace_tasks)
    Task* __restrict__ q_buf[2];      // the two queues of the slot (ping-pong)
    uint32_t* __restrict__ q_link_out; // deferred split: per task of q_out, its parent link (slot << 1 | refr)
    const uint32_t* __restrict__ q_link_in;
    uint32_t* __restrict__ q_link_buf[2];
    uint32_t* __restrict__ q_out_n;   // produced count of q_out
    const uint32_t* __restrict__ q_in_n;
    uint32_t* __restrict__ q_in_head;
    SplitCtr* __restrict__ ctr;
    unsigned long long* __restrict__ acc; // per output pixel: fixed-point colour (r, g, b, -)
    uint32_t* __restrict__ spilled;   // output pixels finished by finalize_spilled
    float4* __restrict__ diag;        // diagnostic builds only (TRT_DIAG_DUMP_SHADOW): ray dump
    // deferred shadows (defer != 0): event log, shadow query queue, per-pixel log heads
    uint32_t defer;
    uint32_t ev_cap;                  // event chunks per stripe (stripe s: chunks [s * ev_cap, ...))
    uint32_t shq_cap;                 // queries per stripe (stripe s: queries [s * shq_cap, ...))
    float4* __restrict__ ev;          // chunks of kEvRows x 4 planes x 64 lanes float4
    float4* __restrict__ shq;         // per query: (origin, max distance), (direction, slot << 2 | light)
    uint2* __restrict__ px_ev;        // per output pixel: (root event slot or kEvNone, 0)
    uint32_t* __restrict__ fb;        // output pixels re-traced with in-place shadows
    DeferCtr* __restrict__ dctr;
    uint32_t defer_sub;               // pass A waves per 8x8 tile (1, 2, 4, 8: trace_tile)
    // frames of a deferred launch (trt_render_frames groups consecutive frames): frame f's
    // scratch is ev + f * ev_fstride, shq + f * shq_fstride, px_ev / fb + f * px_fstride, dctr + f
    uint32_t dframes;
    uint32_t defer_inter;             // a group's blocks frame by frame: 1 = pass A (trace_kernel), 2 = passes A, B, C
    uint32_t px_fstride;
    size_t ev_fstride, shq_fstride;
    uint32_t spp_lanes;               // spp > 1: one lane per sample (trace_samples), spp waves per tile
    FrameRec fr[kMaxLaunchFrames];    // camera + output of each frame of the launch
};
static_assert(sizeof(KArgs) <= 4096, "KArgs fits the 4 KB kernel-argument limit");

} // namespace trt
