/*
 * rt_types.h — scene / camera / ray records shared by the host library, the
 * HIP kernels and the CPU oracle.
 *
 * Every struct is byte-compatible with the reference's host/device structs in
 * clrt/ocl/geometry.h:63-163 (and seed_value_t in clrt/ocl/rng.h:9-12), so a
 * caller that already fills the reference's `Sphere` / `Camera` arrays can hand
 * them to rt_set_spheres / rt_set_camera unchanged.  Offsets are pinned by the
 * static asserts at the bottom.
 *
 * Plain C, no HIP types: this header is part of the C-ABI boundary.
 */
#ifndef RT_TYPES_H
#define RT_TYPES_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* clrt/ocl/geometry.h:59 — origin offset / epsilon used everywhere. */
#define RT_SMALL_F 1e-4f
/* clrt/ocl/raytracer.cl:16-17 — half-extents of the enclosing box. */
#define RT_BOX_WIDTH 6u
#define RT_BOX_HEIGHT 5u
/* clrt/ocl/rtcommon.h:9 — shadow samples per emissive sphere (sphere path). */
#define RT_LIGHT_SAMPLES 2u

/* clrt/ocl/geometry.h:63-67 */
typedef struct rt_vec3 {
    float x, y, z;
} rt_vec3;

/* clrt/ocl/geometry.h:37-47 (host float4 union) / OpenCL float4 — 16 B aligned. */
typedef struct rt_float4 {
    float x, y, z, w;
}
#if defined(__GNUC__) || defined(__clang__)
__attribute__((aligned(16)))
#endif
rt_float4;

/* clrt/ocl/geometry.h:72-83 */
typedef struct rt_ray {
    rt_vec3 o;
    rt_vec3 d;
    float tmin;
    float tmax;
    rt_vec3 propagation;
    rt_vec3 extinction;
    uint32_t diffuse_bounce;
} rt_ray;

/* clrt/ocl/geometry.h:88-95 */
typedef struct rt_triangle {
    rt_vec3 v0;
    rt_vec3 e1;
    rt_vec3 e2;
} rt_triangle;

/* clrt/ocl/geometry.h:100-109 */
typedef struct rt_hit_info {
    rt_vec3 hit_pt;
    rt_vec3 surface_normal;
} rt_hit_info;

/* clrt/ocl/geometry.h:118-123 — view carries |view| = (W/2)/tan(fov/2). */
typedef struct rt_camera {
    rt_float4 view;
    rt_float4 up;
    rt_float4 right;
    rt_float4 position;
} rt_camera;

/* clrt/ocl/geometry.h:130-151 */
typedef struct rt_material {
    rt_vec3 diffuse;
    float kd;
    rt_vec3 extinction;
    float kt;
    rt_vec3 emission;
    float emission_power;
    float ks;
    float specExp;
    float ior;
    float refExp;
} rt_material;

/* clrt/ocl/geometry.h:156-163 */
typedef struct rt_sphere {
    rt_material mat;
    rt_vec3 center;
    float radius;
} rt_sphere;

/* clrt/ocl/rng.h:9-12 */
typedef struct rt_seed {
    uint32_t x;
    uint32_t y;
} rt_seed;

#ifdef __cplusplus
}
#define RT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

RT_STATIC_ASSERT(sizeof(rt_vec3) == 12, "vec3 is 12 B");
RT_STATIC_ASSERT(sizeof(rt_ray) == 60, "ray_t is 60 B");
RT_STATIC_ASSERT(offsetof(rt_ray, tmin) == 24, "ray_t.tmin @24");
RT_STATIC_ASSERT(offsetof(rt_ray, propagation) == 32, "ray_t.propagation @32");
RT_STATIC_ASSERT(offsetof(rt_ray, diffuse_bounce) == 56, "ray_t.diffuse_bounce @56");
RT_STATIC_ASSERT(sizeof(rt_triangle) == 36, "triangle_t is 36 B");
RT_STATIC_ASSERT(sizeof(rt_hit_info) == 24, "hit_info_t is 24 B");
RT_STATIC_ASSERT(sizeof(rt_camera) == 64, "Camera is 64 B");
RT_STATIC_ASSERT(offsetof(rt_camera, position) == 48, "Camera.position @48");
RT_STATIC_ASSERT(sizeof(rt_material) == 64, "material_t is 64 B");
RT_STATIC_ASSERT(offsetof(rt_material, emission_power) == 44, "material_t.emission_power @44");
RT_STATIC_ASSERT(offsetof(rt_material, refExp) == 60, "material_t.refExp @60");
RT_STATIC_ASSERT(sizeof(rt_sphere) == 80, "Sphere is 80 B");
RT_STATIC_ASSERT(offsetof(rt_sphere, center) == 64, "Sphere.center @64");
RT_STATIC_ASSERT(offsetof(rt_sphere, radius) == 76, "Sphere.radius @76");
RT_STATIC_ASSERT(sizeof(rt_seed) == 8, "seed_value_t is 8 B");

#endif /* RT_TYPES_H */
