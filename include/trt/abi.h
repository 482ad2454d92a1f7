/*
 * trt/abi.h — the C-ABI drop-in for the reference's compute-shader hot path.
 *
 * The reference's "operator boundary" is a Vulkan descriptor set with seven bindings
 * (main.cpp:1218-1274) plus one vkCmdDispatch per frame (main.cpp:2108-2131).  Each
 * entry point below replaces one piece of that boundary:
 *
 *   trt_create / trt_destroy   <- device + pipeline setup (main.cpp:547-725, 1394-1427)
 *                                 and teardown (main.cpp:440-526)
 *   trt_upload_scene           <- createShaderStorageBuffers() (main.cpp:1494-1647:
 *                                 binding 5 triangles, binding 6 models), createUniformBuffers()
 *                                 (main.cpp:1650-1664, binding 0) and the background texture
 *                                 upload + sampler (main.cpp:928-1111, binding 4)
 *   trt_update_ubo             <- updateUniformBuffer() (main.cpp:2165-2179)
 *   trt_render                 <- recordComputeCommandBuffer() + vkQueueSubmit
 *                                 (main.cpp:2108-2131, 2181-2205); binding 1 (rayIn) is
 *                                 trt_params.rays_in, binding 2 (rayOut.resultColor) is
 *                                 out_rgba32f, binding 3 (storage image) is out_rgba8.
 *
 * Conventions: every function returns 0 (TRT_OK) or a negative TRT_ERR_* code and never
 * throws; trt_last_error() returns the message of the last failure on that context.  The
 * caller owns every host array (copied during the call).  The context owns its device
 * buffers until trt_destroy().  Calls on one context are serialised by the caller; use one
 * context per GPU.
 */
#ifndef TRT_ABI_H
#define TRT_ABI_H

#include <stddef.h>
#include <stdint.h>

#include "scene_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TRT_ABI_VERSION 4

/* status codes */
#define TRT_OK 0
#define TRT_ERR_INVALID (-1) /* bad argument (null pointer, size, depth, band) */
#define TRT_ERR_HIP (-2)     /* HIP runtime failure (no device, launch, copy) */
#define TRT_ERR_NOSCENE (-3) /* trt_render before trt_upload_scene */
#define TRT_ERR_OOM (-4)     /* host or device allocation failed */
#define TRT_ERR_IO (-5)      /* file could not be read or parsed */

/* trt_params.flags */
#define TRT_FLAG_SPHERES (1u << 0)     /* draw_sphere, shader.comp:83 (false in the shipped shader) */
#define TRT_FLAG_FLOOR (1u << 1)       /* draw_floor, shader.comp:84 */
#define TRT_FLAG_CHECKER (1u << 2)     /* checker floor colour, shader.comp:312 (commented out upstream) */
#define TRT_FLAG_ENVMAP (1u << 3)      /* miss -> envmap, shader.comp:455-456; else BACKGROUND_COLOR :77 */
#define TRT_FLAG_ROW_QUIRK (1u << 4)   /* the pix++ off-by-one of main.cpp:1501-1502 */
#define TRT_FLAG_DEVICE_PTRS (1u << 5) /* out_rgba8 / out_rgba32f / rays_in are device pointers */
#define TRT_FLAG_COUNT (1u << 6)       /* fill trt_stats ray counters */
#define TRT_FLAG_TIMING (1u << 7)      /* fill trt_stats.kernel_ms (waits for the frame) */
#define TRT_FLAG_BATCH_WALK (1u << 8)  /* trace meshes by walking the batch list in the reference's
                                          order (shader.comp:338) instead of the per-ray BVH; same
                                          image, and batch/triangle work counters equal the
                                          reference's */
#define TRT_FLAG_SRGB_OUT (1u << 9)    /* out_rgba8 = the frame as displayed: sRGB-encoded
                                          (the B8G8R8A8_SRGB swapchain, main.cpp:2341, that
                                          shader.frag writes the sampled image to); out_rgba32f
                                          stays rayOut */
#define TRT_FLAG_BAND_IN_PLACE (1u << 10) /* with band params: each rendered row is written at its
                                          row of a full width*height image instead of compactly
                                          (several bands render into one frame); needs
                                          TRT_FLAG_DEVICE_PTRS */

/* The shipped shader: floor on, spheres off, envmap background, host ray quirk. */
#define TRT_FLAGS_REFERENCE (TRT_FLAG_FLOOR | TRT_FLAG_ENVMAP | TRT_FLAG_ROW_QUIRK)

#define TRT_MAX_DEPTH_LIMIT 20u /* MAX_DEPTH of shader.comp:75 */

typedef struct trt_params {
    uint32_t width, height; /* image size; WIDTH/HEIGHT of main.cpp:35-36 & shader.comp:79-80 */
    uint32_t max_depth;     /* MAX_DEPTH (shader.comp:75): segments of depth 0..max_depth-1; 1..20 */
    uint32_t spp;           /* samples per pixel; 1 = the reference's pixel-centre rays */
    uint32_t seed;          /* jitter seed (spp > 1 only) */
    uint32_t flags;         /* TRT_FLAG_* */
    float fov;              /* vertical field of view in radians (main.cpp:1498: 1.05f) */
    uint32_t band_rows;     /* row-band sharding: 0 = whole image; else rows r with */
    uint32_t band_count;    /*   (r / band_rows) % band_count == band_index are rendered and */
    uint32_t band_index;    /*   written compactly, in row order */
    const trt_ray* rays_in; /* optional binding-1 replay (width*height rays), or NULL */
} trt_params;

typedef struct trt_stats {
    uint64_t primary_rays;   /* root segments traced (W*H*spp over the rendered rows) */
    uint64_t secondary_rays; /* reflection/refraction/TIR segments that reach scene_intersect */
    uint64_t shadow_rays;    /* shadow_intersect calls */
    /* Per-stage work, the units of the algorithmic-byte roofline: */
    uint64_t misses;         /* segments with no hit (background lookups) */
    uint64_t tri_nearest;    /* segments whose closest hit is a triangle */
    uint64_t sphere_tests;   /* ray_sphere_intersect calls (scene + shadow) */
    uint64_t batch_tests;    /* ray_aabb_intersect calls (scene + shadow) */
    uint64_t batch_hits;     /* ... that passed */
    uint64_t tri_tests;      /* ray_triangle_intersect calls (scene + shadow) */
    uint64_t node_tests;     /* hierarchy-node box tests in front of the batch tests (0 in the
                                reference's linear loop; batch_tests then counts only the batch
                                boxes actually reached) */
    double kernel_ms;        /* device time of the frame (TRT_FLAG_TIMING) */
    /* Moller-Trumbore stages reached (shader.comp:223-270; the per-stage FP32 work of the VALU
     * roofline, SURVEY §8d: 22 / 34 / 52 / 59 flops at exit after a / u / v / t): */
    uint64_t tri_past_a;     /* triangle tests past the parallel test (u computed) */
    uint64_t tri_past_u;     /* ... past the u test (v computed) */
    uint64_t tri_past_v;     /* ... past the v test (t computed) */
    /* Shadow queries a frame does not trace: the light's diffuse and specular terms both vanish
     * from the colour (zero term or zero albedo weight), so lit or shadowed it adds exactly
     * nothing (shader.comp:495-505).  The counting pass traces them (every counter above is the
     * reference's work) and reports them and the work inside them here: */
    uint64_t shadow_skipped;
    uint64_t skipped_sphere_tests, skipped_box_tests, skipped_tri_tests;
    uint64_t skipped_tri_past_a, skipped_tri_past_u, skipped_tri_past_v;
} trt_stats;

typedef struct trt_ctx trt_ctx;

const char* trt_version(void);

/* Creates a context on HIP device `hip_device` (a fresh non-blocking stream). */
int trt_create(trt_ctx** out, int hip_device);
int trt_destroy(trt_ctx* ctx);
const char* trt_last_error(const trt_ctx* ctx);

/* Launch subsequent work on an external hipStream_t (e.g. a torch.cuda.Stream); NULL
 * restores the context's own stream (the legacy null stream cannot be selected). */
int trt_set_stream(trt_ctx* ctx, void* hip_stream);

/* Uploads the bindings of one scene.  ntri/nmodel may be 0 (the reference cannot bind a
 * zero-size SSBO; this boundary can), env may be NULL when TRT_FLAG_ENVMAP is never set.
 * Triangle materials are kept per triangle as in binding 5. */
int trt_upload_scene(trt_ctx* ctx, const trt_ubo* ubo, const trt_triangle* tris, uint32_t ntri,
                     const trt_model* models, uint32_t nmodel, const uint8_t* env_rgba8,
                     uint32_t env_w, uint32_t env_h);

/* Per-frame UBO update (spheres, lights, camera). */
int trt_update_ubo(trt_ctx* ctx, const trt_ubo* ubo);

/* Renders one frame.  out_rgba8: rows*width*4 bytes (RGBA8 = floor(255*c + 0.5), a = 255);
 * out_rgba32f: rows*width*4 floats (rayOut.resultColor = (c, 1)).  Either may be NULL.
 * rows = trt_output_rows(p).  Host pointers unless TRT_FLAG_DEVICE_PTRS; with device
 * pointers and no COUNT/TIMING flag the call only enqueues work on the stream. */
int trt_render(trt_ctx* ctx, const trt_params* p, uint8_t* out_rgba8, float* out_rgba32f,
               trt_stats* st);

/* Frames in flight of trt_render_frames (the reference's MAX_FRAMES_IN_FLIGHT = 2,
 * main.cpp:45: per-frame command buffers, UBOs and rayOut buffers, main.cpp:1518-1664, with
 * no barrier between consecutive compute submissions).  Frame i of a trt_render_frames call
 * runs on in-flight slot i % n: slot 0 is the context's stream, slots 1..n-1 are streams the
 * context owns, forked from and joined back into its stream inside the call, so frame i+1's
 * workgroups fill the GPU while frame i's slowest tiles finish.  n in [1, 32], or 0 = auto
 * (the default): 4, or for deferred-shadow frames, whose depth-20 trees leave the longest
 * tails, a shape by the hardware queues (below; measured: profiles/r02_ab_queues_*.log,
 * profiles/r04z_ab_deferred_in_flight.jsonl, profiles/r06t_ab_defer_shape_32q.jsonl).  With n
 * set, deferred frames go one per launch on the n slots.  Each slot is a HIP stream, so the process
 * needs as many hardware queues: the library leaves GPU_MAX_HW_QUEUES to the host (HIP's
 * default is 4; the Python package and bench.py raise it to 32 before HIP initialises, see
 * INTEGRATION.md) and only reads it: with auto in-flight, a deferred loop runs slots tracing
 * launch groups of several consecutive frames each, on at most half the queues: 8 slots x 3
 * frames with >= 16 queues, 2 x 8 with HIP's default 4. */
#define TRT_FRAMES_IN_FLIGHT_DEFAULT 0u
#define TRT_FRAMES_IN_FLIGHT_AUTO 0u
/* Fixed by the ABI (a host cannot change it): the upper bound of n.  The library's own slot
 * count is the private build-time TRT_BUILD_MAX_IN_FLIGHT (csrc/trt_ctx.h, default and maximum:
 * this value); its range checks use that count. */
#define TRT_MAX_FRAMES_IN_FLIGHT 32u
int trt_set_frames_in_flight(trt_ctx* ctx, uint32_t n);

/* Frames per launch of trt_render_frames.  The reference records one vkCmdDispatch per frame
 * (main.cpp:2122-2124).  Here consecutive frames of a plain frame loop (no subtree split, no
 * deferred shadows) whose UBOs differ only in camPos — the reference's interactive loop moves
 * only the camera, main.cpp:391-403 — are traced by ONE launch of ntiles x n workgroups: frame
 * k of the launch owns blocks [k * ntiles, (k + 1) * ntiles), so a frame's slowest tiles overlap
 * the next frame's tiles inside one grid and the GPU drains once per launch instead of once per
 * frame.  n in [1, TRT_MAX_FRAME_BATCH]: 1 = one launch per frame (the reference's dispatch per
 * frame); 0 = auto (the default): up to TRT_MAX_FRAME_BATCH frames per launch.  Split frames
 * launch one frame at a time; deferred-shadow frames in launch groups of their own (above),
 * each frame of a group with its own scratch. */
#define TRT_FRAME_BATCH_AUTO 0u
#define TRT_MAX_FRAME_BATCH 64u
int trt_set_frame_batch(trt_ctx* ctx, uint32_t n);

/* Subtree split (load balance of deep refraction trees).  The reference traces a pixel's whole
 * Whitted tree depth-first in one invocation (shader.comp:423-583); in mesh scenes at depth 20
 * a few pixels' trees hold hundreds of segments and one 8x8 tile then runs for milliseconds
 * while the rest of the GPU idles.  With a window of w depths the frame is traced in depth
 * windows: a segment at depth k*w is handed to a task queue and traced by any lane of the
 * next launch.  Rays, hits and counters are unchanged; the colour of a split pixel is the
 * sum of its subtrees' colours (each summed in the reference's pop order) added in 32.32
 * fixed point — deterministic, and within a few ulp of the reference's single running sum
 * (well inside the RGBA8 +-1 bar).  Pixels whose tree stays within the first window are
 * bit-identical to the unsplit frame.  spp > 1 frames are never split.
 * window: TRT_SPLIT_AUTO (default: w = 4 for mesh scenes with max_depth >= 8, else off),
 * TRT_SPLIT_OFF, or 2..5. */
#define TRT_SPLIT_AUTO 0
#define TRT_SPLIT_OFF 1
int trt_set_subtree_split(trt_ctx* ctx, int window);

/* Deferred shadow rays (the reference traces a hit's three shadow rays in place inside the
 * pixel's DFS, shader.comp:483-507).  A deferred frame runs in three passes: (A) every pixel's
 * Whitted tree without shadow rays, logging one colour event per segment in the reference's
 * pop order, with the shadow queries appended to one dense queue; (B) the queue traced with
 * every lane of every wave busy (in the per-pixel loop a wave runs the shadow rays of only the
 * lanes that sit at a hit); (C) each pixel's events summed in logged order with the shader's
 * own arithmetic.  The image is bit-identical to the per-pixel loop without subtree split (the
 * reference's single running sum), rays and counters are unchanged, and a pixel whose log does
 * not fit the scratch is re-traced in place.  With an explicit subtree-split window (above) a
 * deferred frame's subtrees are traced by other lanes into logs of their own, reached through
 * LINK events at the place of their events, so the sum keeps the reference order (no
 * fixed-point sums); TRT_SPLIT_AUTO does not split deferred frames.  COUNT and spp > 1 frames
 * always run the per-pixel loop (a COUNT frame of a scene that would defer runs unsplit, so its
 * image equals the deferred frame's).
 * mode: TRT_DEFER_AUTO (default: mesh scenes with max_depth >= 8, unless a subtree-split
 * window 2..5 was set explicitly), TRT_DEFER_OFF, TRT_DEFER_ON. */
#define TRT_DEFER_AUTO 0
#define TRT_DEFER_OFF 1
#define TRT_DEFER_ON 2
int trt_set_deferred_shadows(trt_ctx* ctx, int mode);

/* Counters of the last deferred frame rendered on `slot` (0 .. TRT_MAX_FRAMES_IN_FLIGHT-1;
 * trt_render uses one slot per stream): out[0] event chunks taken, out[1] shadow queries
 * appended, out[2] pixels re-traced in place, out[3] chunk capacity, out[4] query capacity (of
 * the slot's allocation).  Waits for the context's stream. */
int trt_defer_stats(trt_ctx* ctx, uint32_t slot, uint64_t out[5]);

/* The reference's frame loop (mainLoop -> drawFrame, main.cpp:405-438, 2181-2205) in one
 * call: for each of `nframes` frames, updateUniformBuffer with ubos[i] (or the current UBO
 * when ubos is NULL) and trace the frame into out_rgba8 + i * frame_stride bytes.  Plain
 * frames are traced several per launch (trt_set_frame_batch); launches rotate over the
 * frames-in-flight streams (trt_set_frames_in_flight), so frames may run concurrently: give
 * concurrent frames distinct images (frame_stride >= rows*width*4) unless they are identical —
 * frame_stride 0 makes every frame write the same image, like the reference's single storage
 * image (binding 3, main.cpp:865-926).  Requires TRT_FLAG_DEVICE_PTRS; only enqueues; all
 * frames have completed on the context's stream when work enqueued after the call runs.  With
 * TRT_FLAG_TIMING a HIP event pair brackets every `time_every`-th launch (0 or 1: every
 * launch) on its stream (the span includes any overlap with launches on the other streams);
 * trt_frame_times() reads them. */
int trt_render_frames(trt_ctx* ctx, const trt_params* p, const trt_ubo* ubos, uint32_t nframes,
                      uint8_t* out_rgba8, size_t frame_stride, uint32_t time_every);

/* Device time per frame (ms) of each launch timed by the last timed trt_render_frames call:
 * the launch's event span divided by the frames it traced (waits for them); n <= the number
 * of timed launches, trt_timed_launches(). */
int trt_frame_times(trt_ctx* ctx, float* ms, uint32_t n);
/* Launches timed by the last timed trt_render_frames call, and (frames_out, may be NULL) the
 * frames each traced. */
uint32_t trt_timed_launches(trt_ctx* ctx, uint32_t* frames_out, uint32_t cap);

/* Waits for all work enqueued on the context's stream. */
int trt_synchronize(trt_ctx* ctx);

/* Rows written by trt_render for these params (H, or the band's share). */
uint32_t trt_output_rows(const trt_params* p);

/* Fills `p` with the reference defaults: 1024x768, depth 20, spp 1, fov 1.05,
 * TRT_FLAGS_REFERENCE. */
void trt_params_default(trt_params* p);

/* ---- multi-GPU frame tiling over RCCL (SURVEY §8(b) trt_render_multi, §8(e)) ----------
 * Replaces the single-queue dispatch + submit (main.cpp:2108-2131, 2181-2205) with one frame
 * row-tiled over the GPUs of a node: rows are dealt in interleaved bands of `band_rows` rows
 * to ranks * groups_per_rank band groups (row y -> group (y / band_rows) % (ranks * groups);
 * group g is rendered by rank g / groups_per_rank), every device renders its groups with the
 * single-GPU kernel into compact RGBA8 buffers, one grouped ncclSend / ncclRecv moves them to
 * the frame's root device over xGMI, and a re-interleave kernel assembles the frame there.
 * The result is bit-identical to trt_render of the whole frame.  The scene is built once, on
 * rank 0, and its device bindings are broadcast (ncclBroadcast) to the other devices.
 * Output arrays `out_rgba8` have one entry per device of THIS process (trt_multi_local_count);
 * only the root's entry is written (the others may be NULL). */
typedef struct trt_multi trt_multi;

#define TRT_MULTI_ID_BYTES 128 /* ncclUniqueId */
#define TRT_ROOT_ROTATE (-1)   /* root of frame i = rank i % ranks (every device's xGMI links
                                  ingest frames at once) */

/* One process drives `ndev` devices (ncclCommInitAll); rank i = devices[i]. */
int trt_multi_create(trt_multi** out, const int* devices, uint32_t ndev);
/* One process per GPU: every rank passes the same id (made by trt_multi_unique_id on one rank
 * and exchanged out of band, e.g. MPI or torch.distributed), ncclCommInitRank. */
int trt_multi_unique_id(uint8_t* id /* TRT_MULTI_ID_BYTES */);
int trt_multi_create_rank(trt_multi** out, int hip_device, uint32_t nranks, uint32_t rank, const uint8_t* id);
int trt_multi_destroy(trt_multi* m);
const char* trt_multi_last_error(const trt_multi* m);
uint32_t trt_multi_ranks(const trt_multi* m);       /* world size */
uint32_t trt_multi_local_count(const trt_multi* m); /* devices driven by this process */
/* The per-device context of local device i (its stream, split and frames-in-flight knobs). */
trt_ctx* trt_multi_context(trt_multi* m, uint32_t local);
/* Band groups per rank (default 1); more groups = finer interleave of the image over ranks. */
int trt_multi_set_band_groups(trt_multi* m, uint32_t groups_per_rank);
/* trt_upload_scene on rank 0 + broadcast of its device bindings; on the other ranks of a
 * one-process-per-GPU run the arrays are ignored (may be NULL).  Collective. */
int trt_multi_upload_scene(trt_multi* m, const trt_ubo* ubo, const trt_triangle* tris, uint32_t ntri,
                           const trt_model* models, uint32_t nmodel, const uint8_t* env_rgba8,
                           uint32_t env_w, uint32_t env_h);
int trt_multi_update_ubo(trt_multi* m, const trt_ubo* ubo);
/* One frame (p describes the whole frame; band_* must be 0) gathered on rank `root` (or
 * TRT_ROOT_ROTATE).  out_rgba8[i]: width*height*4 bytes, a device pointer on local device i
 * with TRT_FLAG_DEVICE_PTRS (then the call only enqueues on each context's stream), else a
 * host pointer (synchronous).  TRT_FLAG_COUNT: st = counters summed over all ranks (a
 * separate counting pass).  Collective. */
int trt_render_multi(trt_multi* m, const trt_params* p, uint32_t band_rows, int root,
                     uint8_t* const* out_rgba8, trt_stats* st);
/* The frame loop of trt_render_frames, tiled: frames i = 0..nframes-1 (UBO ubos[i], or the
 * current one) in batches of `frames_per_gather` frames.  Each device traces its band groups of
 * a batch's frames (multi-frame launches, trt_set_frame_batch), then ONE grouped ncclSend /
 * ncclRecv moves every frame's bands to that frame's root (trt_band_plan) and each root
 * re-interleaves its frames: frame i lands at out_rgba8[local index of its root] + i *
 * frame_stride on rank trt_frame_root(i, ranks, root) — with TRT_ROOT_ROTATE frame i goes to rank
 * i % ranks, so every device ingests at once and every rank's entry must be set; with a fixed
 * root only the root's entry is written.  Two batches are in flight: a batch's gather +
 * re-interleave overlaps the next batch's render.  Requires TRT_FLAG_DEVICE_PTRS; only
 * enqueues (complete on each context's stream).  Collective. */
int trt_render_multi_frames(trt_multi* m, const trt_params* p, const trt_ubo* ubos, uint32_t nframes,
                            uint32_t band_rows, int root, uint32_t frames_per_gather,
                            uint8_t* const* out_rgba8, size_t frame_stride);
/* Waits for every context stream of this process. */
int trt_multi_synchronize(trt_multi* m);
/* Test / diagnostic: with on != 0 the root's own band groups also travel through the gather
 * (an ncclSend to itself and the re-interleave) instead of being rendered in place, so the
 * whole exchange runs on a one-GPU communicator.  Same image; slower. */
int trt_multi_set_self_gather(trt_multi* m, int on);

/* ---- the exchange plan of a tiled batch ---------------------------------------------------
 * The data movement trt_render_multi_frames performs for a batch of `nframes` frames starting
 * at frame `first_frame` of the call, as a list of transfers, so a host with its own transport
 * (MPI, torch.distributed, ...) can run the same exchange; trt_multi.cpp executes exactly this
 * plan over RCCL (ncclSend / ncclRecv in list order on both ends, one group).  Frame i's root is
 * trt_frame_root(i, nranks, root): `root`, or i % nranks for TRT_ROOT_ROTATE.  Rank q renders
 * band groups q * G .. q * G + G - 1 (G = groups_per_rank) of every frame.  One transfer per
 * (sender, root) pair carries all of the batch's frames that root owns:
 *   - the batch frames are ordered by root; rank r's J_r frames (batch order) start at frame
 *     slot off_r = the number of batch frames rooted by ranks < r;
 *   - a sender stores group v of the j-th frame of root r at ((off_r + j) * G + v) * block_bytes
 *     of its batch buffer, so the J_r * G blocks for root r are contiguous;
 *   - root r receives sender q's blocks at (q * J_r * G) * block_bytes of its gather buffer, i.e.
 *     group v of its j-th frame at ((q * J_r + j) * G + v) * block_bytes;
 *   - compact row k of band group g is frame row trt_band_frame_row(k, band_rows, groups, g).
 * Blocks are block_bytes each (padded to the largest group).  Without TRT_PLAN_SELF_GATHER the
 * root's own groups do not travel (it renders them in place).  Pure host arithmetic. */
typedef struct trt_band_layout {
    uint32_t groups;       /* band groups NG = nranks * groups_per_rank */
    uint32_t max_rows;     /* compact rows of the largest group */
    uint64_t block_bytes;  /* one compact group buffer: max_rows * width * 4 */
    uint64_t local_bytes;  /* a rank's batch buffer: nframes * groups_per_rank * block_bytes */
    uint64_t gather_bytes; /* the largest gather buffer of a root: frames rooted * groups * block_bytes */
} trt_band_layout;
typedef struct trt_band_xfer {
    uint32_t src, dst;   /* sending rank, receiving rank (the root of the carried frames) */
    uint32_t frames;     /* J_dst: the batch frames dst roots (all of them travel together) */
    uint32_t groups;     /* band groups per frame (groups_per_rank) */
    uint32_t first_slot; /* off_dst: their first frame slot in the sender's buffer */
    uint32_t pad;
    uint64_t src_offset; /* bytes into the sender's batch buffer: off_dst * G * block_bytes */
    uint64_t dst_offset; /* bytes into the root's gather buffer: src * J_dst * G * block_bytes */
    uint64_t bytes;      /* J_dst * G * block_bytes */
} trt_band_xfer;
#define TRT_PLAN_SELF_GATHER 1u
uint32_t trt_frame_root(uint32_t frame, uint32_t nranks, int root);
uint32_t trt_band_frame_row(uint32_t k, uint32_t band_rows, uint32_t groups, uint32_t g);
/* Fills *layout and up to `cap` transfers (xfers may be NULL to count them); *count = the
 * number of transfers of the plan. */
int trt_band_plan(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t nranks, uint32_t groups_per_rank,
                  uint32_t first_frame, uint32_t nframes, int root, uint32_t flags, trt_band_layout* layout,
                  trt_band_xfer* xfers, uint32_t cap, uint32_t* count);

/* ---- host scene build (main.cpp:192-252, 1529-1580, 2290-2335) -------------------- */

typedef struct trt_scene trt_scene;

int trt_scene_create(trt_scene** out);
void trt_scene_destroy(trt_scene* s);
const char* trt_scene_last_error(const trt_scene* s);

/* Triangles per AABB batch (main.cpp:1549: 64). */
int trt_scene_set_batch_size(trt_scene* s, uint32_t batch_size);

/* One modelList entry (config.hpp:97-101) from an already-triangulated mesh: positions
 * (xyz floats, nverts) and indices (3 per triangle, file order).  Applies
 * M = T * Rz * Ry * Rx * S (transformTriangles, main.cpp:192-216), smooth vertex
 * normals when normal_interp == 1 (computeVertexNormals, main.cpp:218-252), then splits
 * into batches with AABBs (main.cpp:1548-1566). */
int trt_scene_add_mesh(trt_scene* s, const float* positions, uint32_t nverts,
                       const uint32_t* indices, uint32_t ntris, const trt_material* mat,
                       const float scale[3], const float rotation_deg[3],
                       const float translation[3], int normal_interp);

/* The same from an OBJ file (loadObjAsTriangles, main.cpp:2290-2335, with tinyobjloader's
 * triangulation rules). */
int trt_scene_add_obj(trt_scene* s, const char* path, const trt_material* mat,
                      const float scale[3], const float rotation_deg[3],
                      const float translation[3], int normal_interp);

uint32_t trt_scene_triangle_count(const trt_scene* s);
uint32_t trt_scene_model_count(const trt_scene* s);
const trt_triangle* trt_scene_triangles(const trt_scene* s);
const trt_model* trt_scene_models(const trt_scene* s);

/* ---- envmap JPEG ---------------------------------------------------------
 * The reference reads its envmap with stb_image v2.22, stbi_load(path, ..., STBI_rgb_alpha)
 * (main.cpp:928-949), then uploads it as binding 4.  This path decodes the same files to the
 * same RGBA8 bytes: the entropy decode (Huffman, baseline and progressive scans) runs on the
 * host into coefficient planes (trt_jpeg_*), and dequantisation, IDCT, chroma upsampling and
 * colour conversion run on the GPU (trt_jpeg_decode), straight into device memory. */

/* colour model of the RGBA output (stb's load_jpeg_image) */
#define TRT_JPEG_GRAY 0
#define TRT_JPEG_YCBCR 1
#define TRT_JPEG_RGB 2  /* component ids 'R','G','B', or Adobe transform 0 without JFIF */
#define TRT_JPEG_CMYK 3 /* 4 components, Adobe transform 0 */
#define TRT_JPEG_YCCK 4 /* 4 components, Adobe transform 2 */

typedef struct trt_jpeg trt_jpeg;

typedef struct trt_jpeg_info {
    uint32_t width, height;
    uint32_t components;  /* 1, 3 or 4 */
    uint32_t progressive; /* SOF2 */
    int32_t color;        /* TRT_JPEG_* */
    uint32_t hmax, vmax;  /* largest sampling factors */
    uint32_t h[4], v[4];  /* per-component sampling factors */
    uint32_t blocks_w[4], blocks_h[4]; /* MCU-padded block grid of each coefficient plane */
} trt_jpeg_info;

int trt_jpeg_create(trt_jpeg** out);
void trt_jpeg_destroy(trt_jpeg* j);
const char* trt_jpeg_last_error(const trt_jpeg* j);

/* Parses `len` bytes of a JPEG file and entropy-decodes every scan (host). */
int trt_jpeg_parse(trt_jpeg* j, const uint8_t* data, size_t len);
int trt_jpeg_get_info(const trt_jpeg* j, trt_jpeg_info* info);

/* Raw (not dequantised) coefficients of component c: blocks_w * blocks_h blocks of 64
 * int16 in natural (row-major) order; and its 64-entry quantisation table.  NULL if c is
 * out of range or nothing was parsed. */
const int16_t* trt_jpeg_coefficients(const trt_jpeg* j, uint32_t c);
const uint16_t* trt_jpeg_quant(const trt_jpeg* j, uint32_t c);

/* GPU reconstruction of a parsed JPEG into width * height * 4 bytes of RGBA8 (alpha 255), the
 * buffer stbi_load(..., STBI_rgb_alpha) returns.  Host pointer unless TRT_FLAG_DEVICE_PTRS.
 * Synchronous. */
int trt_jpeg_decode(trt_ctx* ctx, const trt_jpeg* j, uint8_t* out_rgba8, uint32_t flags);

/* Binding 4 from JPEG bytes (the reference's stbi_load + texture upload, main.cpp:928-1111):
 * replaces the context's envmap.  Call after trt_upload_scene (which replaces every
 * binding). */
int trt_upload_envmap_jpeg(trt_ctx* ctx, const uint8_t* data, size_t len);

/* ---- frame files (the reference only presents, main.cpp:2181-2205) ------- */

/* Binary PPM (P6, RGB; alpha dropped) of a host RGBA8 frame, e.g. trt_render's out_rgba8. */
int trt_write_ppm(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height);

/* 8-bit RGBA PNG (zlib deflate) of a host RGBA8 frame. */
int trt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* TRT_ABI_H */
