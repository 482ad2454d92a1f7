/*
 * oracle/trt_oracle.h — TEST INFRASTRUCTURE ONLY (see trt_oracle.c header).
 *
 * CPU restatement of the reference hot path (VulkanComputeShaderApplication/shaders/
 * shader.comp:1-602 + the host ray generation of main.cpp:1496-1506).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 */
#ifndef TRT_ORACLE_H
#define TRT_ORACLE_H

#include "../include/trt/abi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MODE_FAST 0    /* volume stack removed (proven inert) */
#define ORC_MODE_LITERAL 1 /* shader.comp as written: PathSegment copies + volume stack */
/* fast mode + the kernel's subtree split with window W (2..5; trt_set_subtree_split) */
#define ORC_MODE_SPLIT(W) (16 + (W))

typedef struct orc_scene {
    const trt_ubo* ubo;
    const trt_triangle* tris;
    uint32_t ntri;
    const trt_model* models;
    uint32_t nmodel;
    const uint8_t* env; /* RGBA8, env_w * env_h texels, row 0 = v = 0 */
    uint32_t env_w, env_h;
} orc_scene;

/* Renders the rows selected by p (band fields honoured) into compact outputs; host pointers
 * only (TRT_FLAG_DEVICE_PTRS is rejected).  nthreads <= 0 -> all hardware threads.
 * Returns 0 or a negative TRT_ERR_* code. */
int orc_render(const orc_scene* scene, const trt_params* p, int mode, int nthreads,
               uint8_t* out_rgba8, float* out_rgba32f, trt_stats* st);

/* Single-ray probes used by the known-answer tests (shader.comp line refs in the .c). */
int orc_ray_aabb(const float o[3], const float d[3], const float bmin[3], const float bmax[3]);
int orc_ray_triangle(const float o[3], const float d[3], const float v0[3], const float v1[3],
                     const float v2[3], const float n0[3], const float n1[3], const float n2[3],
                     int normal_interp, float* t, float normal[3]);
int orc_ray_sphere(const float o[3], const float d[3], const float center_radius[4], float* t);
void orc_custom_refract(const float I[3], const float N[3], float eta_out, float eta_in,
                        float out[3]);
void orc_direction_to_uv(const float d[3], float uv[2]);
void orc_sample_env(const uint8_t* env, uint32_t w, uint32_t h, const float uv[2],
                    float rgb[3]);
void orc_primary_dir(const trt_params* p, uint32_t x, uint32_t y, uint32_t sample,
                     float d[3]);
/* cast_ray for one root ray; returns the clamped linear colour (before gamma). */
void orc_cast_ray(const orc_scene* scene, const trt_params* p, int mode, const float o[3],
                  const float d[3], float rgb[3], trt_stats* st);

#ifdef __cplusplus
}
#endif

#endif
