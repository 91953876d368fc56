/*
 * rt_internal.h — host-side interface between the C-ABI layer (rt_host.cpp),
 * the BVH builder (rt_bvh.cpp) and the HIP kernels (rt_kernels.hip).
 * Not part of the public boundary.
 */
#ifndef RT_INTERNAL_H
#define RT_INTERNAL_H

#include <stdint.h>

#include <string>
#include <vector>

#include "rt_types.h"

/* Traversal stack entries per lane (LDS).  rt_bvh.cpp bounds the tree depth so
   that push-far-child traversal never needs more (checked before launch). */
#define RT_STACK_DEPTH 32
#define RT_BVH_MAX_DEPTH (RT_STACK_DEPTH + 1)
#define RT_BLOCK 256
#define RT_LEAF_MAX 8

/* One BVH node = 4 x float4 = 64 B (both children's boxes in the parent):
     n0 = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
     n1 = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
     n2 = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
     n3 = (child0, child1, 0, 0) as int bits
   child >= 0: inner node index; child < 0: leaf ~((first << 3) | (count - 1)).
   Triangles are stored in leaf order, 3 x float4 = 48 B each:
     t0 = (v0.xyz, original index as int bits), t1 = (e1.xyz, 0), t2 = (e2.xyz, 0)
   with e1 = v1 - v0, e2 = v2 - v0 computed exactly as get_triangle()
   (rtcommon.h:20-37), so the intersection arithmetic is unchanged. */
struct RtBvh {
    std::vector<float> nodes; /* 16 floats per node */
    std::vector<float> tris;  /* 12 floats per triangle */
    uint32_t n_nodes = 0;
    uint32_t n_leaves = 0;
    uint32_t depth = 0;
    double build_seconds = 0.0;
};

/* Builds a binned-SAH BVH over the mesh (rt_bvh.cpp).  Returns false and sets
   err on invalid input. */
bool rt_build_bvh(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris, RtBvh &out,
                  std::string &err);

/* ---- kernel launchers (rt_kernels.hip) ---- */
struct RtTriLaunch {
    float *out;
    uint32_t *seeds;
    const float *nodes;
    const float *tris;
    uint32_t n_tris;
    const rt_sphere *lights; /* emissive spheres only, scene order */
    uint32_t n_lights;
    rt_camera cam;
    uint32_t W, H, Wpad, Hpad, Hl;
    uint32_t sample_rate, max_depth, progressive;
    uint32_t stripe, n_ranks, rank;
    uint32_t *work_counter;
    unsigned long long *counters; /* [4] */
};

struct RtSphLaunch {
    float *out;
    uint32_t *seeds;
    const rt_sphere *spheres;
    uint32_t n_spheres;
    rt_camera cam;
    uint32_t W, H, Wpad, Hpad, Hl;
    uint32_t sample_rate, max_depth, progressive;
    uint32_t stripe, n_ranks, rank;
    unsigned long long *counters;
};

/* All return a hipError_t as int (0 = success). */
int rt_launch_tris(const RtTriLaunch &a, bool linear, bool count, int grid_blocks, void *stream);
int rt_launch_spheres(const RtSphLaunch &a, bool single_sample, void *stream);
int rt_launch_trace_rays(const float *nodes, const float *tris, uint32_t n_tris, const rt_ray *rays, uint32_t n,
                         int any_hit, bool linear, int32_t *out_idx, float *out_t, void *stream);
/* Persistent-grid size for the triangle kernel on this device. */
int rt_tris_grid_blocks(int device, bool linear, bool count, int *blocks);

#endif /* RT_INTERNAL_H */
