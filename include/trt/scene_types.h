/*
 * trt/scene_types.h — byte layouts of the reference's GPU-visible scene records.
 *
 * These are the std140 records the reference binds to its compute descriptor set
 * (main.cpp:1218-1274, shader.comp:40-71).  Every struct here is layout-identical
 * to the reference so that a caller can hand over the very arrays it used to fill
 * its SSBOs/UBO:
 *
 *   trt_material  <- Material            geometry.hpp:5-10,   shader.comp:3-7    (48 B)
 *   trt_sphere    <- Sphere              geometry.hpp:12-16,  shader.comp:9-12   (64 B)
 *   trt_triangle  <- Triangle            geometry.hpp:18-27,  shader.comp:19-27  (144 B)
 *   trt_model     <- Model (a 64-tri batch record)
 *                                        geometry.hpp:30-46,  shader.comp:29-38  (96 B)
 *   trt_ubo       <- UniformBufferObject main.cpp:145-157,    shader.comp:40-51  (352 B)
 *   trt_ray       <- Ray                 main.cpp:159-187,    shader.comp:14-17  (32 B)
 *
 * Plain C, no GPU types: included by the C-ABI (abi.h), the HIP runtime and the
 * CPU oracle alike.
 */
#ifndef TRT_SCENE_TYPES_H
#define TRT_SCENE_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct trt_vec4 { float x, y, z, w; } trt_vec4;
typedef struct trt_ivec4 { int32_t x, y, z, w; } trt_ivec4;

/* albedo = (diffuse weight, specular weight, reflection weight, refraction weight);
 * diffuse_specular = (kd.rgb, specular exponent); refractive.x = index of refraction. */
typedef struct trt_material {
    trt_vec4 albedo;
    trt_vec4 diffuse_specular;
    trt_vec4 refractive;
} trt_material;

typedef struct trt_sphere {
    trt_vec4 center_radius; /* xyz centre, w radius */
    trt_material material;
} trt_sphere;

typedef struct trt_triangle {
    trt_vec4 v0, v1, v2; /* xyz position, w = 1 */
    trt_material material;
    trt_vec4 v0_norm, v1_norm, v2_norm; /* smoothed vertex normals, w = 0 */
} trt_triangle;

/* One AABB-culled triangle batch.  params0 = (start, count, normal_interp, 0). */
typedef struct trt_model {
    trt_ivec4 params0;
    trt_vec4 bboxMin;
    trt_vec4 bboxMax;
    trt_material material;
} trt_model;

typedef struct trt_ubo {
    trt_sphere sphere0, sphere1, sphere2, sphere3;
    trt_vec4 light0, light1, light2; /* xyz position, w intensity (unused by the shader) */
    trt_vec4 camPos;                 /* xyz ray origin */
    trt_vec4 bboxMin, bboxMax;       /* written by the host, never read by the shader */
} trt_ubo;

typedef struct trt_ray {
    trt_vec4 dir;         /* xyz primary direction, w = 1 */
    trt_vec4 resultColor; /* rgb after gamma, a = 1 */
} trt_ray;

#ifdef __cplusplus
} /* extern "C" */
#define TRT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define TRT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

TRT_STATIC_ASSERT(sizeof(trt_material) == 48, "Material is 48 B (std140)");
TRT_STATIC_ASSERT(sizeof(trt_sphere) == 64, "Sphere is 64 B (std140)");
TRT_STATIC_ASSERT(sizeof(trt_triangle) == 144, "Triangle is 144 B (std140)");
TRT_STATIC_ASSERT(sizeof(trt_model) == 96, "Model is 96 B (std140)");
TRT_STATIC_ASSERT(sizeof(trt_ubo) == 352, "UniformBufferObject is 352 B (std140)");
TRT_STATIC_ASSERT(sizeof(trt_ray) == 32, "Ray is 32 B (std140)");

#endif /* TRT_SCENE_TYPES_H */
