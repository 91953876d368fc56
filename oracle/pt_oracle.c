/*
 * pt_oracle.c — CPU restatement of the reference path tracer (TEST
 * INFRASTRUCTURE ONLY).
 *
 * This file is the parity checker for the HIP path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it
 * (liboracle.so); the product library (pathtracer.cl_amd/csrc) never links it
 * and has no CPU fallback.
 *
 * It restates, function by function and in the same floating-point operation
 * order, the OpenCL kernel of krisher/PathTracer.cl:
 *     clrt/ocl/rng.h, geometryFuncs.h, materials.h, rtcommon.h, raytracer.cl
 * under the pinned arithmetic model of include/rt_math.h.  Each function cites
 * the reference lines it follows.
 *
 * Pinning: oracle/Makefile also compiles the reference's own raytracer.cl for
 * x86-64 (oracle/_ref, container only) and tests/golden/make_golden.py records
 * its outputs as fixtures; tests/test_oracle_golden.py checks this restatement
 * against every fixture bit for bit (see DESIGN.md "Oracle").
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math (x86-64 SSE: no excess
 * precision, no FMA).
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rt_math.h"
#include "rt_types.h"

#define OR_API __attribute__((visibility("default")))

typedef struct or_counters {
    uint64_t closest; /* closest-hit scene queries (scene_intersection[_tri]) */
    uint64_t shadow;  /* any-hit queries (visibility_test[_tri]) */
} or_counters;

struct or_bvh;

typedef struct or_mesh {
    const rt_vec3 *verts;
    const int32_t *idx;
    uint32_t n_tris;
    const struct or_bvh *bvh; /* NULL: the reference's linear loops; else the independent BVH mode */
} or_mesh;

/* ------------------------------------------------------------------ rng.h */

/* rng.h:24-42 — Marsaglia multiply-with-carry, 23 mantissa bits -> [0,1). */
OR_API float or_frand(rt_seed *s)
{
    s->x = 36969u * (s->x & 65535u) + (s->x >> 16);
    s->y = 18000u * (s->y & 65535u) + (s->y >> 16);
    uint32_t bits = (s->x << 16) + s->y;
    bits = (bits & 0x007fffffu) | 0x40000000u;
    return (rt_u2f(bits) - 2.0f) / 2.0f;
}

/* rng.h:45-47 */
OR_API float or_strat_rand(rt_seed *s, int cur, int total)
{
    float f = or_frand(s);
    return ((float)cur + f) / (float)total;
}

/* -------------------------------------------------------- geometryFuncs.h */

static inline float dot3(rt_vec3 a, rt_vec3 b) /* geometryFuncs.h:6 DOT() */
{
    return a.x * b.x + a.y * b.y + a.z * b.z;
}

/* geometryFuncs.h:13-27 */
static rt_vec3 perpendicular_vector(rt_vec3 v)
{
    rt_vec3 t;
    if (rt_fabsf(v.y) > 0.9f) {
        float inv = rt_rsqrtf(v.z * v.z + v.y * v.y);
        t.x = 0.0f;
        t.y = -v.z * inv;
        t.z = v.y * inv;
    } else {
        float inv = rt_rsqrtf(v.z * v.z + v.x * v.x);
        t.x = v.z * inv;
        t.y = 0.0f;
        t.z = -v.x * inv;
    }
    return t;
}

/* geometryFuncs.h:29-32 */
static rt_vec3 cross_vec(rt_vec3 a, rt_vec3 b)
{
    rt_vec3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}

/* geometryFuncs.h:41-56 */
OR_API float or_intersect_sphere(const rt_ray *ray, rt_vec3 c, float radius)
{
    float ox = ray->o.x - c.x;
    float oy = ray->o.y - c.y;
    float oz = ray->o.z - c.z;
    float dist2 = ox * ox + oy * oy + oz * oz;
    float b_neg = -(ox * ray->d.x + oy * ray->d.y + oz * ray->d.z);
    float disc = b_neg * b_neg - (dist2 - radius * radius);
    if (disc > 0) {
        float sq = rt_sqrtf(disc);
        if (b_neg - sq > ray->tmin) return b_neg - sq;
        return b_neg + sq;
    }
    return 0.0f;
}

/* geometryFuncs.h:58-69 */
static void sphere_normal(rt_hit_info *hit, rt_vec3 c, float radius)
{
    float inv = 1.0f / radius;
    hit->surface_normal.x = (hit->hit_pt.x - c.x) * inv;
    hit->surface_normal.y = (hit->hit_pt.y - c.y) * inv;
    hit->surface_normal.z = (hit->hit_pt.z - c.z) * inv;
}

/* geometryFuncs.h:71-84 */
OR_API void or_box_normal(rt_hit_info *hit, float xs, float ys, float zs)
{
    rt_vec3 p = hit->hit_pt;
    float dx = rt_fabsf(rt_fabsf(p.x) - xs);
    float dy = rt_fabsf(rt_fabsf(p.y) - ys);
    float dz = rt_fabsf(rt_fabsf(p.z) - zs);
    rt_vec3 n = {0.0f, 0.0f, 0.0f};
    if (dx < dy && dx < dz)
        n.x = -p.x / rt_fabsf(p.x);
    else if (dy < dz)
        n.y = -p.y / rt_fabsf(p.y);
    else
        n.z = -p.z / rt_fabsf(p.z);
    hit->surface_normal = n;
}

/* geometryFuncs.h:86-150, box centred at the origin (raytracer passes
   (float4)0, so center - size == -size exactly). */
OR_API float or_intersects_box(const rt_ray *ray, float xs, float ys, float zs)
{
    float near_t = 0.0f;
    float far_t = rt_inff();
    float t1, t2;
    if (ray->d.x != 0) {
        t1 = (0.0f - xs - ray->o.x) / ray->d.x;
        t2 = (0.0f + xs - ray->o.x) / ray->d.x;
        near_t = rt_minf(t1, t2);
        far_t = rt_maxf(t1, t2);
    } else if (rt_fabsf(ray->o.x - 0.0f) > xs) {
        return 0;
    }
    if (ray->d.y != 0) {
        t1 = (0.0f - ys - ray->o.y) / ray->d.y;
        t2 = (0.0f + ys - ray->o.y) / ray->d.y;
        if (t1 > t2) {
            near_t = rt_maxf(t2, near_t);
            far_t = rt_minf(t1, far_t);
        } else {
            near_t = rt_maxf(t1, near_t);
            far_t = rt_minf(t2, far_t);
        }
    } else if (rt_fabsf(ray->o.y - 0.0f) > ys) {
        return 0;
    }
    if (ray->d.z != 0) {
        t1 = (0.0f - zs - ray->o.z) / ray->d.z;
        t2 = (0.0f + zs - ray->o.z) / ray->d.z;
        if (t1 > t2) {
            near_t = rt_maxf(t2, near_t);
            far_t = rt_minf(t1, far_t);
        } else {
            near_t = rt_maxf(t1, near_t);
            far_t = rt_minf(t2, far_t);
        }
    } else if (rt_fabsf(ray->o.z - 0.0f) > zs) {
        return 0;
    }
    if (near_t > far_t || far_t < ray->tmin) return rt_inff();
    if (near_t < ray->tmin) return far_t;
    return near_t;
}

/* geometryFuncs.h:160-202 — Moller-Trumbore, closest-hit form: accepts
   tmin <= t <= tmax and shrinks tmax. */
OR_API int or_intersects_triangle(rt_ray *ray, float *u, float *v, const rt_triangle *tri)
{
    rt_vec3 p = cross_vec(ray->d, tri->e2);
    float det = dot3(p, tri->e1);
    if (rt_fabsf(det) < RT_SMALL_F) return 0;
    det = 1.0f / det;
    rt_vec3 to = {ray->o.x - tri->v0.x, ray->o.y - tri->v0.y, ray->o.z - tri->v0.z};
    rt_vec3 q = cross_vec(to, tri->e1);
    float e0 = dot3(p, to) * det;
    if (e0 < 0 || e0 > 1) return 0;
    float e1 = dot3(q, ray->d) * det;
    if (e1 < 0 || e1 + e0 > 1) return 0;
    float t = dot3(q, tri->e2) * det;
    if (t > ray->tmax || t < ray->tmin) return 0;
    ray->tmax = t;
    *u = e0;
    *v = e1;
    return 1;
}

/* geometryFuncs.h:212-245 — any-hit form: strict tmin < t < tmax. */
OR_API int or_intersects_triangle_p(const rt_ray *ray, const rt_triangle *tri)
{
    rt_vec3 p = cross_vec(ray->d, tri->e2);
    float det = dot3(p, tri->e1);
    if (rt_fabsf(det) < RT_SMALL_F) return 0;
    det = 1.0f / det;
    rt_vec3 to = {ray->o.x - tri->v0.x, ray->o.y - tri->v0.y, ray->o.z - tri->v0.z};
    rt_vec3 q = cross_vec(to, tri->e1);
    float e0 = dot3(p, to) * det;
    if (e0 < 0 || e0 > 1) return 0;
    float e1 = dot3(q, ray->d) * det;
    if (e1 < 0 || e1 + e0 > 1) return 0;
    float t = dot3(q, tri->e2) * det;
    return (t < ray->tmax && t > ray->tmin);
}

/* ------------------------------------------------------------ materials.h */

/* materials.h:21-35 (returns xyz; the w = pdf lane is unused by callers) */
static rt_vec3 cos_sample_hemisphere(float r1, float r2)
{
    float cos_t = rt_sqrtf(1.0f - r1);
    float sin_t = rt_sqrtf(1.0f - cos_t * cos_t);
    float phi = RT_M_2PI_F * r2;
    rt_vec3 w = {sin_t * rt_cosf(phi), sin_t * rt_sinf(phi), cos_t};
    return w;
}

/* materials.h:44-50 */
static rt_vec3 shading_to_world(rt_vec3 v, rt_vec3 n)
{
    rt_vec3 tx = perpendicular_vector(n);
    rt_vec3 ty = cross_vec(n, tx);
    rt_vec3 r = {tx.x * v.x + ty.x * v.y + n.x * v.z, tx.y * v.x + ty.y * v.y + n.y * v.z,
                 tx.z * v.x + ty.z * v.y + n.z * v.z};
    return r;
}

/* materials.h:59-65 */
static rt_vec3 world_to_shading(rt_vec3 w, rt_vec3 n)
{
    rt_vec3 tx = perpendicular_vector(n);
    rt_vec3 ty = cross_vec(n, tx);
    rt_vec3 r = {dot3(w, tx), dot3(w, ty), dot3(w, n)};
    return r;
}

/* materials.h:76-108 (pdf is always 1) */
static void sample_phong(rt_vec3 *w, float spec_exp, float r1, float r2)
{
    rt_vec3 wi = {-w->x, -w->y, w->z};
    if (spec_exp < 100000.0f) {
        float cos_a = rt_powf(r1, 1.0f / (spec_exp + 1.0f));
        float sin_t = rt_sqrtf(1.0f - cos_a * cos_a);
        float phi = RT_M_2PI_F * r2;
        wi.x = rt_cosf(phi) * sin_t;
        wi.y = rt_sinf(phi) * sin_t;
        wi.z = cos_a;
        float wo_dot_wh = dot3(*w, wi);
        wi.x = -w->x + 2.0f * wo_dot_wh * wi.x;
        wi.y = -w->y + 2.0f * wo_dot_wh * wi.y;
        wi.z = -w->z + 2.0f * wo_dot_wh * wi.z;
    }
    *w = wi;
}

/* materials.h:146-218 */
static int sample_refraction(rt_vec3 *trans, rt_ray *ray, float ior, float blur_exp, float r1, float r2)
{
    float cos_wo = rt_fabsf(ray->d.z);
    int entering = ray->d.z > 0;
    float ei, eo;
    if (entering) {
        ei = 1.0f;
        eo = ior;
    } else {
        ei = ior;
        eo = 1.0f;
    }
    float ratio = ei / eo;
    float cos_sq = 1.0f - (ratio * ratio * (1.0f - ray->d.z * ray->d.z));
    if (cos_sq < 0.0f) {
        ray->d.x *= -1.0f;
        ray->d.y *= -1.0f;
        entering = !entering;
    } else {
        float cos_t = rt_sqrtf(cos_sq);
        if (entering) cos_t = -cos_t;
        rt_vec3 wi = {-ray->d.x * ratio, -ray->d.y * ratio, cos_t};
        if (blur_exp < 100000.0f) {
            float cos_a = rt_powf(r1, 1.0f / (blur_exp + 1.0f));
            float sin_t = rt_sqrtf(1.0f - cos_a * cos_a);
            float phi = RT_M_2PI_F * r2;
            wi.x = rt_cosf(phi) * sin_t;
            wi.y = rt_sinf(phi) * sin_t;
            wi.z = cos_a;
            float wo_dot_wh = dot3(ray->d, wi);
            wi.x = -ray->d.x + 2.0f * wo_dot_wh * wi.x;
            wi.y = -ray->d.y + 2.0f * wo_dot_wh * wi.y;
            wi.z = -ray->d.z + 2.0f * wo_dot_wh * wi.z;
        }
        ray->d = wi;
        cos_t = rt_fabsf(cos_t);
        float parl = (eo * cos_wo - ei * cos_t) / (eo * cos_wo + ei * cos_t);
        float perp = (ei * cos_wo - eo * cos_t) / (ei * cos_wo + eo * cos_t);
        float fres = (parl * parl + perp * perp) * 0.5f;
        fres = (1.0f - fres) / cos_t;
        trans->x *= fres;
        trans->y *= fres;
        trans->z *= fres;
    }
    return entering;
}

/* materials.h:232-271 (the returned pdf is unused by every caller) */
OR_API void or_sphere_emissive_radiance(rt_ray *ray, rt_vec3 c, float radius, float r1, float r2)
{
    rt_vec3 dir = {c.x - ray->o.x, c.y - ray->o.y, c.z - ray->o.z};
    float inv = rt_rsqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
    dir.x *= inv;
    dir.y *= inv;
    dir.z *= inv;
    float sin_max = radius * inv;
    float cos_max = rt_sqrtf(1.0f - sin_max * sin_max);
    float cos_t = 1.0f + r1 * (cos_max - 1.0f);
    float sin_t = rt_sqrtf(1.0f - cos_t * cos_t);
    float phi = RT_M_2PI_F * r2;
    rt_vec3 local = {rt_cosf(phi) * sin_t, rt_sinf(phi) * sin_t, cos_t};
    ray->d = shading_to_world(local, dir);
    ray->tmin = RT_SMALL_F;
    ray->tmax = or_intersect_sphere(ray, c, radius) - RT_SMALL_F;
}

/* ------------------------------------------------------------- rtcommon.h */

/* rtcommon.h:20-37 */
OR_API void or_get_triangle(rt_triangle *t, uint32_t i, const rt_vec3 *verts, const int32_t *idx)
{
    rt_vec3 a = verts[idx[3 * i]];
    rt_vec3 b = verts[idx[3 * i + 1]];
    rt_vec3 c = verts[idx[3 * i + 2]];
    t->v0 = a;
    t->e1.x = b.x - a.x;
    t->e1.y = b.y - a.y;
    t->e1.z = b.z - a.z;
    t->e2.x = c.x - a.x;
    t->e2.y = c.y - a.y;
    t->e2.z = c.z - a.z;
}

/* rtcommon.h:39-52 — linear closest hit: the highest index among equal t. */
OR_API int32_t or_scene_intersection_tri(rt_ray *ray, const rt_vec3 *verts, const int32_t *idx, uint32_t n)
{
    float u, v;
    rt_triangle tri;
    int32_t hit = -1;
    for (uint32_t i = 0; i < n; ++i) {
        or_get_triangle(&tri, i, verts, idx);
        if (or_intersects_triangle(ray, &u, &v, &tri)) hit = (int32_t)i;
    }
    return hit;
}

/* rtcommon.h:59-68 */
OR_API int or_visibility_test_tri(const rt_ray *ray, const rt_vec3 *verts, const int32_t *idx, uint32_t n)
{
    rt_triangle tri;
    for (uint32_t i = 0; i < n; ++i) {
        or_get_triangle(&tri, i, verts, idx);
        if (or_intersects_triangle_p(ray, &tri)) return 0;
    }
    return 1;
}

/* ------------------------------------------- independent BVH mode (oracle) */
/*
 * A second, independent way to answer rtcommon.h:39-52 and :59-68 exactly: a plain binary BVH
 * over the mesh (binned SAH on centroids, leaves of at most 4 triangles), boxes in binary64,
 * no quantisation, no determinant cull, no unhittable-triangle cull, no candidate lists — none
 * of the product's (csrc/rt_bvh.cpp, rt_quant.h) machinery.  It exists so that whole frames at
 * the BASELINE sizes can be checked bit for bit in seconds instead of days (the linear loop is
 * O(N) per ray).  Its answers are the linear loop's by construction:
 *   - every triangle is tested with the reference's own Moller-Trumbore arithmetic
 *     (or_get_triangle + mt_core: the same IEEE operations as or_intersects_triangle);
 *   - closest hit: the linear loop accepts tmin <= t <= (its current tmax), so it ends on the
 *     minimum accepted t with ties to the HIGHEST index; here: accept iff t >= tmin, t <= the
 *     ray's tmax, and (t < best_t or (t == best_t and index > best_index)) — order-free;
 *   - any hit: strict tmin < t < tmax (intersects_triangle_p), any order, first found;
 *   - culling is conservative: a node is skipped only if no triangle below it can be accepted.
 *     The float test accepts a line whose exact barycentrics lie within the MT rounding error
 *     of the triangle, and reports a t within its own rounding error of the exact crossing.
 *     Per node visit both are bounded from the node's largest |e1||e2| and |e1|+|e2|, the ray
 *     origin's distance to the node (|T| = |o - v0|) and the threshold |det| >= 1e-4
 *     (geometryFuncs.h:167): with u = 2^-24,
 *        det_lo = 1e-4 - 8u|d|A,  Db = u(9 L|T||d| + 9 A|d|) / det_lo + 3u   (barycentric error),
 *        pad    = 16 Db L + 4u|T|                                           (spatial error),
 *        Dt     = 4 [u(9|T|A + 8 tb|d|A) / det_lo + 2u tb],  tb = (|T| + pad)/|d|  (t error),
 *     i.e. four times the first-order bounds of the operations (cross and dot products: 2-3
 *     roundings each, the division: one).  The node box is widened by pad and
 *     the ray's interval by Dt before the slab test (binary64).  A node whose det_lo would fall
 *     below 0.5e-4 (|e1||e2| > ~100: no such triangle in any scene here) is always visited.
 * Pinned on the CPU against the linear loop on the golden fixtures and on random and grazing
 * rays (tests/test_oracle_golden.py), and against the reference kernel on strided pixels.
 */
typedef struct or_bnode {
    double lo[3], hi[3]; /* box of the subtree's float triangles (v0, v0 + e1, v0 + e2) */
    double amax, lmax;   /* max |e1||e2| and max |e1| + |e2| over the subtree */
    int32_t a, b;        /* inner: children a, b; leaf: a = -1 - first (into tri), b = count */
} or_bnode;

typedef struct or_bvh {
    or_bnode *nodes;
    uint32_t *tri; /* leaf order -> original triangle index */
    uint32_t n_nodes, n_tris, depth;
} or_bvh;

/* rtcommon.h/geometryFuncs.h:160-202 up to t: 1 if the barycentric tests pass, t written. */
static int mt_core(const rt_ray *ray, const rt_triangle *tri, float *t_out)
{
    rt_vec3 p = cross_vec(ray->d, tri->e2);
    float det = dot3(p, tri->e1);
    if (rt_fabsf(det) < RT_SMALL_F) return 0;
    det = 1.0f / det;
    rt_vec3 to = {ray->o.x - tri->v0.x, ray->o.y - tri->v0.y, ray->o.z - tri->v0.z};
    rt_vec3 q = cross_vec(to, tri->e1);
    float e0 = dot3(p, to) * det;
    if (e0 < 0 || e0 > 1) return 0;
    float e1 = dot3(q, ray->d) * det;
    if (e1 < 0 || e1 + e0 > 1) return 0;
    *t_out = dot3(q, tri->e2) * det;
    return 1;
}

typedef struct bvh_item {
    double lo[3], hi[3], c[3];
    double a, l;
} bvh_item;

typedef struct bvh_build {
    bvh_item *items;
    uint32_t *perm;
    or_bnode *nodes;
    uint32_t n_nodes, cap, depth;
} bvh_build;

static void box_of(const bvh_item *it, const uint32_t *perm, uint32_t n, or_bnode *nd)
{
    for (int k = 0; k < 3; ++k) {
        nd->lo[k] = INFINITY;
        nd->hi[k] = -INFINITY;
    }
    nd->amax = nd->lmax = 0.0;
    for (uint32_t i = 0; i < n; ++i) {
        const bvh_item *t = &it[perm[i]];
        for (int k = 0; k < 3; ++k) {
            if (t->lo[k] < nd->lo[k]) nd->lo[k] = t->lo[k];
            if (t->hi[k] > nd->hi[k]) nd->hi[k] = t->hi[k];
        }
        if (t->a > nd->amax) nd->amax = t->a;
        if (t->l > nd->lmax) nd->lmax = t->l;
    }
}

static double half_area(const double *lo, const double *hi)
{
    const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return (x < 0 || y < 0 || z < 0) ? 0.0 : x * y + y * z + z * x;
}

#define OR_BVH_BINS 16
#define OR_BVH_LEAF 4

/* Builds the subtree over perm[0, n) into node `ni`; binned SAH on the widest centroid axis,
   a median split when SAH finds nothing better than a leaf of > OR_BVH_LEAF triangles. */
static int build_node(bvh_build *B, uint32_t ni, uint32_t first, uint32_t n, uint32_t depth)
{
    if (depth > B->depth) B->depth = depth;
    or_bnode *nd = &B->nodes[ni];
    box_of(B->items, B->perm + first, n, nd);
    if (n <= OR_BVH_LEAF || depth >= 60) {
        nd->a = -1 - (int32_t)first;
        nd->b = (int32_t)n;
        return 0;
    }
    double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < n; ++i) {
        const double *c = B->items[B->perm[first + i]].c;
        for (int k = 0; k < 3; ++k) {
            if (c[k] < clo[k]) clo[k] = c[k];
            if (c[k] > chi[k]) chi[k] = c[k];
        }
    }
    int axis = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
    const double ext = chi[axis] - clo[axis];
    uint32_t mid = n / 2;
    if (ext > 0) {
        uint32_t cnt[OR_BVH_BINS] = {0};
        double blo[OR_BVH_BINS][3], bhi[OR_BVH_BINS][3];
        for (int b = 0; b < OR_BVH_BINS; ++b)
            for (int k = 0; k < 3; ++k) {
                blo[b][k] = INFINITY;
                bhi[b][k] = -INFINITY;
            }
        const double scale = OR_BVH_BINS / ext;
        for (uint32_t i = 0; i < n; ++i) {
            const bvh_item *t = &B->items[B->perm[first + i]];
            int b = (int)((t->c[axis] - clo[axis]) * scale);
            if (b >= OR_BVH_BINS) b = OR_BVH_BINS - 1;
            if (b < 0) b = 0;
            cnt[b]++;
            for (int k = 0; k < 3; ++k) {
                if (t->lo[k] < blo[b][k]) blo[b][k] = t->lo[k];
                if (t->hi[k] > bhi[b][k]) bhi[b][k] = t->hi[k];
            }
        }
        double right_cost[OR_BVH_BINS];
        double rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t rc = 0;
        for (int b = OR_BVH_BINS - 1; b > 0; --b) {
            rc += cnt[b];
            for (int k = 0; k < 3; ++k) {
                if (blo[b][k] < rlo[k]) rlo[k] = blo[b][k];
                if (bhi[b][k] > rhi[k]) rhi[k] = bhi[b][k];
            }
            right_cost[b] = rc ? half_area(rlo, rhi) * rc : 0.0;
        }
        double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t lc = 0;
        double best = INFINITY;
        int best_b = -1;
        for (int b = 0; b < OR_BVH_BINS - 1; ++b) {
            lc += cnt[b];
            for (int k = 0; k < 3; ++k) {
                if (blo[b][k] < llo[k]) llo[k] = blo[b][k];
                if (bhi[b][k] > lhi[k]) lhi[k] = bhi[b][k];
            }
            if (lc == 0 || lc == n) continue;
            const double cost = half_area(llo, lhi) * lc + right_cost[b + 1];
            if (cost < best) {
                best = cost;
                best_b = b;
            }
        }
        if (best_b >= 0) {
            uint32_t i = 0, j = n;
            while (i < j) { /* partition: bin <= best_b first */
                const bvh_item *t = &B->items[B->perm[first + i]];
                int b = (int)((t->c[axis] - clo[axis]) * scale);
                if (b >= OR_BVH_BINS) b = OR_BVH_BINS - 1;
                if (b <= best_b) {
                    ++i;
                } else {
                    --j;
                    const uint32_t tmp = B->perm[first + i];
                    B->perm[first + i] = B->perm[first + j];
                    B->perm[first + j] = tmp;
                }
            }
            mid = i;
        }
    }
    if (mid == 0 || mid == n) mid = n / 2; /* equal centroids: split the range in half */
    if (B->n_nodes + 2 > B->cap) return -1;
    const uint32_t ca = B->n_nodes++, cb = B->n_nodes++;
    nd->a = (int32_t)ca;
    nd->b = (int32_t)cb;
    if (build_node(B, ca, first, mid, depth + 1)) return -1;
    return build_node(B, cb, first + mid, n - mid, depth + 1);
}

OR_API or_bvh *or_bvh_build(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris)
{
    if (!verts || !idx || !n_tris) return NULL;
    for (uint64_t i = 0; i < 3ull * n_tris; ++i)
        if (idx[i] < 0 || (uint32_t)idx[i] >= n_verts) return NULL;
    bvh_build B;
    memset(&B, 0, sizeof(B));
    B.items = (bvh_item *)malloc(sizeof(bvh_item) * n_tris);
    B.perm = (uint32_t *)malloc(sizeof(uint32_t) * n_tris);
    B.cap = 2 * n_tris + 1;
    B.nodes = (or_bnode *)malloc(sizeof(or_bnode) * B.cap);
    or_bvh *out = (or_bvh *)calloc(1, sizeof(or_bvh));
    if (!B.items || !B.perm || !B.nodes || !out) goto fail;
    for (uint32_t i = 0; i < n_tris; ++i) {
        rt_triangle t;
        or_get_triangle(&t, i, (const rt_vec3 *)verts, idx);
        const double p[3][3] = {{t.v0.x, t.v0.y, t.v0.z},
                                {(double)t.v0.x + t.e1.x, (double)t.v0.y + t.e1.y, (double)t.v0.z + t.e1.z},
                                {(double)t.v0.x + t.e2.x, (double)t.v0.y + t.e2.y, (double)t.v0.z + t.e2.z}};
        bvh_item *it = &B.items[i];
        for (int k = 0; k < 3; ++k) {
            double lo = p[0][k], hi = p[0][k];
            for (int v = 1; v < 3; ++v) {
                if (p[v][k] < lo) lo = p[v][k];
                if (p[v][k] > hi) hi = p[v][k];
            }
            it->lo[k] = lo;
            it->hi[k] = hi;
            it->c[k] = 0.5 * (lo + hi);
        }
        const double l1 = sqrt((double)t.e1.x * t.e1.x + (double)t.e1.y * t.e1.y + (double)t.e1.z * t.e1.z);
        const double l2 = sqrt((double)t.e2.x * t.e2.x + (double)t.e2.y * t.e2.y + (double)t.e2.z * t.e2.z);
        it->a = l1 * l2;
        it->l = l1 + l2;
        B.perm[i] = i;
    }
    B.n_nodes = 1;
    if (build_node(&B, 0, 0, n_tris, 0)) goto fail;
    free(B.items);
    out->nodes = B.nodes;
    out->tri = B.perm;
    out->n_nodes = B.n_nodes;
    out->n_tris = n_tris;
    out->depth = B.depth;
    return out;
fail:
    free(B.items);
    free(B.perm);
    free(B.nodes);
    free(out);
    return NULL;
}

OR_API void or_bvh_free(or_bvh *b)
{
    if (!b) return;
    free(b->nodes);
    free(b->tri);
    free(b);
}

OR_API uint32_t or_bvh_nodes(const or_bvh *b) { return b ? b->n_nodes : 0u; }
OR_API uint32_t or_bvh_depth(const or_bvh *b) { return b ? b->depth : 0u; }

/* Per ray, once: the ray in binary64 and its direction's inverse and length. */
typedef struct bvh_ray {
    double o[3], d[3], inv[3], dl;
} bvh_ray;

static void bvh_ray_setup(bvh_ray *r, const rt_ray *ray)
{
    r->o[0] = ray->o.x;
    r->o[1] = ray->o.y;
    r->o[2] = ray->o.z;
    r->d[0] = ray->d.x;
    r->d[1] = ray->d.y;
    r->d[2] = ray->d.z;
    for (int k = 0; k < 3; ++k) r->inv[k] = r->d[k] != 0.0 ? 1.0 / r->d[k] : 0.0;
    r->dl = sqrt(r->d[0] * r->d[0] + r->d[1] * r->d[1] + r->d[2] * r->d[2]);
}

/* Can a triangle below `nd` be accepted with t in [t_lo, t_hi]?  Conservative (see above):
   |T| is bounded by the L1 distance of the origin to the box centre plus the box's L1 half
   diagonal (both at least their Euclidean values); the slab distances are formed with the
   inverse direction (a few binary64 roundings, absorbed by the 1e-12 relative slack). */
static int node_may_hold(const or_bnode *nd, const bvh_ray *r, double t_lo, double t_hi)
{
    const double u = 5.9604644775390625e-8; /* 2^-24 */
    const double dl = r->dl;
    if (!(dl > 0)) return 1;
    double T = 0.0;
    for (int k = 0; k < 3; ++k) T += fabs(r->o[k] - 0.5 * (nd->lo[k] + nd->hi[k])) + 0.5 * (nd->hi[k] - nd->lo[k]);
    const double A = nd->amax, L = nd->lmax;
    const double det_lo = 0.9999e-4 - 8.0 * u * dl * A;
    if (det_lo < 0.5e-4) return 1;
    const double idet = 1.0 / det_lo;
    const double db = u * (9.0 * L * T * dl + 9.0 * A * dl) * idet + 3.0 * u;
    const double pad = 16.0 * db * L + 4.0 * u * T;
    const double tb = (T + pad) / dl;
    const double dt = 4.0 * (u * (9.0 * T * A + 8.0 * tb * dl * A) * idet + 2.0 * u * tb);
    double tn = t_lo - dt, tf = t_hi + dt;
    for (int k = 0; k < 3; ++k) {
        const double lo = nd->lo[k] - pad, hi = nd->hi[k] + pad;
        if (r->d[k] == 0.0) {
            if (r->o[k] < lo || r->o[k] > hi) return 0;
            continue;
        }
        double a = (lo - r->o[k]) * r->inv[k], b = (hi - r->o[k]) * r->inv[k];
        if (a > b) {
            const double s = a;
            a = b;
            b = s;
        }
        a -= 1e-12 * (fabs(a) + 1.0);
        b += 1e-12 * (fabs(b) + 1.0);
        if (a > tn) tn = a;
        if (b < tf) tf = b;
        if (tn > tf) return 0;
    }
    return 1;
}

/* rtcommon.h:39-52 answered through the BVH: the linear loop's hit (see the accept rule above). */
static int32_t bvh_closest(rt_ray *ray, const or_mesh *m)
{
    const or_bvh *bv = m->bvh;
    const float tmin = ray->tmin, tmax0 = ray->tmax;
    float best_t = tmax0;
    int32_t best = -1;
    bvh_ray br;
    bvh_ray_setup(&br, ray);
    uint32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const or_bnode *nd = &bv->nodes[stack[--sp]];
        if (!node_may_hold(nd, &br, tmin, best_t)) continue;
        if (nd->a < 0) {
            const uint32_t first = (uint32_t)(-1 - nd->a);
            for (int32_t j = 0; j < nd->b; ++j) {
                const uint32_t i = bv->tri[first + (uint32_t)j];
                rt_triangle tri;
                float t;
                or_get_triangle(&tri, i, m->verts, m->idx);
                if (!mt_core(ray, &tri, &t)) continue;
                if (!(t >= tmin && t <= tmax0)) continue;
                if (t < best_t || (t == best_t && (int32_t)i > best)) {
                    best_t = t;
                    best = (int32_t)i;
                }
            }
            continue;
        }
        if (sp + 2 > 128) abort(); /* depth is capped at 60 */
        /* nearer child last (popped first): by the distance of the box centres along d */
        const or_bnode *ca = &bv->nodes[nd->a], *cb = &bv->nodes[nd->b];
        double pa = 0.0, pb = 0.0;
        for (int k = 0; k < 3; ++k) {
            pa += br.d[k] * (ca->lo[k] + ca->hi[k]);
            pb += br.d[k] * (cb->lo[k] + cb->hi[k]);
        }
        if (pa <= pb) {
            stack[sp++] = (uint32_t)nd->b;
            stack[sp++] = (uint32_t)nd->a;
        } else {
            stack[sp++] = (uint32_t)nd->a;
            stack[sp++] = (uint32_t)nd->b;
        }
    }
    if (best >= 0) ray->tmax = best_t;
    return best;
}

/* rtcommon.h:59-68 answered through the BVH: 1 if no triangle occludes (tmin < t < tmax). */
static int bvh_visible(const rt_ray *ray, const or_mesh *m)
{
    const or_bvh *bv = m->bvh;
    bvh_ray br;
    bvh_ray_setup(&br, ray);
    uint32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const or_bnode *nd = &bv->nodes[stack[--sp]];
        if (!node_may_hold(nd, &br, ray->tmin, ray->tmax)) continue;
        if (nd->a < 0) {
            const uint32_t first = (uint32_t)(-1 - nd->a);
            for (int32_t j = 0; j < nd->b; ++j) {
                rt_triangle tri;
                or_get_triangle(&tri, bv->tri[first + (uint32_t)j], m->verts, m->idx);
                if (or_intersects_triangle_p(ray, &tri)) return 0;
            }
            continue;
        }
        if (sp + 2 > 128) abort();
        stack[sp++] = (uint32_t)nd->b;
        stack[sp++] = (uint32_t)nd->a;
    }
    return 1;
}

static int32_t mesh_closest(rt_ray *ray, const or_mesh *m)
{
    return m->bvh ? bvh_closest(ray, m) : or_scene_intersection_tri(ray, m->verts, m->idx, m->n_tris);
}

static int mesh_visible(const rt_ray *ray, const or_mesh *m)
{
    return m->bvh ? bvh_visible(ray, m) : or_visibility_test_tri(ray, m->verts, m->idx, m->n_tris);
}

/* rtcommon.h:78-105 — one sample per emissive sphere, triangles occlude. */
static rt_vec3 sample_direct_illumination_tri(const rt_hit_info *hit, const or_mesh *m, const rt_sphere *lights,
                                              uint32_t n_lights, rt_seed *seed, or_counters *cnt)
{
    rt_ray ray;
    memset(&ray, 0, sizeof(ray));
    ray.o.x = hit->hit_pt.x + hit->surface_normal.x * RT_SMALL_F;
    ray.o.y = hit->hit_pt.y + hit->surface_normal.y * RT_SMALL_F;
    ray.o.z = hit->hit_pt.z + hit->surface_normal.z * RT_SMALL_F;
    rt_vec3 irr = {0.0f, 0.0f, 0.0f};
    for (uint32_t l = 0; l < n_lights; ++l) {
        const rt_sphere *light = &lights[l];
        if (light->mat.emission_power != 0) {
            float r1 = or_frand(seed);
            float r2 = or_frand(seed);
            or_sphere_emissive_radiance(&ray, light->center, light->radius, r1, r2);
            cnt->shadow++;
            if (mesh_visible(&ray, m)) {
                float cw = ray.d.x * hit->surface_normal.x + ray.d.y * hit->surface_normal.y +
                           ray.d.z * hit->surface_normal.z;
                if (cw > 0) {
                    irr.x += light->mat.emission.x * cw;
                    irr.y += light->mat.emission.y * cw;
                    irr.z += light->mat.emission.z * cw;
                }
            }
        }
    }
    return irr;
}

/* rtcommon.h:107-121 — strict interval: the lowest index wins ties. */
OR_API int32_t or_scene_intersection(rt_ray *ray, const rt_sphere *s, uint32_t n)
{
    int32_t hit = -1;
    for (uint32_t i = 0; i < n; ++i) {
        float d = or_intersect_sphere(ray, s[i].center, s[i].radius);
        if (d > ray->tmin && d < ray->tmax) {
            hit = (int32_t)i;
            ray->tmax = d;
        }
    }
    return hit;
}

/* rtcommon.h:128-138 */
OR_API int or_visibility_test(const rt_ray *ray, const rt_sphere *s, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i) {
        float d = or_intersect_sphere(ray, s[i].center, s[i].radius);
        if (d > ray->tmin && d < ray->tmax) return 0;
    }
    return 1;
}

/* rtcommon.h:148-174 — LIGHT_SAMPLES stratified samples per emissive sphere. */
static rt_vec3 sample_direct_illumination(const rt_hit_info *hit, const rt_sphere *s, uint32_t n, uint32_t spl,
                                          rt_seed *seed, or_counters *cnt)
{
    rt_ray ray;
    memset(&ray, 0, sizeof(ray));
    ray.o.x = hit->hit_pt.x + hit->surface_normal.x * RT_SMALL_F;
    ray.o.y = hit->hit_pt.y + hit->surface_normal.y * RT_SMALL_F;
    ray.o.z = hit->hit_pt.z + hit->surface_normal.z * RT_SMALL_F;
    rt_vec3 irr = {0.0f, 0.0f, 0.0f};
    const float inv_samples = 1.0f / (float)spl;
    for (uint32_t k = 0; k < n; ++k) {
        const rt_sphere *light = &s[k];
        if (light->mat.emission_power != 0) {
            for (int i = 0; i < (int)spl; ++i) {
                float r1 = or_frand(seed);
                float r2 = or_strat_rand(seed, i, (int)spl);
                or_sphere_emissive_radiance(&ray, light->center, light->radius, r1, r2);
                cnt->shadow++;
                if (or_visibility_test(&ray, s, n)) {
                    float cw = ray.d.x * hit->surface_normal.x + ray.d.y * hit->surface_normal.y +
                               ray.d.z * hit->surface_normal.z;
                    if (cw > 0) {
                        irr.x += light->mat.emission.x * cw * inv_samples;
                        irr.y += light->mat.emission.y * cw * inv_samples;
                        irr.z += light->mat.emission.z * cw * inv_samples;
                    }
                }
            }
        }
    }
    return irr;
}

/* rtcommon.h:184-251 */
OR_API int or_sample_material(rt_ray *ray, const rt_hit_info *hit, const rt_material *mat, rt_seed *seed)
{
    ray->o = hit->hit_pt;
    ray->d.x *= -1.0f;
    ray->d.y *= -1.0f;
    ray->d.z *= -1.0f;
    ray->d = world_to_shading(ray->d, hit->surface_normal);
    ray->tmin = RT_SMALL_F;
    ray->tmax = rt_inff();
    float p = or_frand(seed);
    float r1 = or_frand(seed);
    float r2 = or_frand(seed);
    if (p < mat->ks) {
        /* `1.0 / samplePhong(...)` is a binary64 division of 1.0 by 1.0f */
        sample_phong(&ray->d, mat->specExp, r1, r2);
        const float inv_pdf = (float)(1.0 / 1.0);
        ray->diffuse_bounce = 0;
        ray->propagation.x *= ray->d.z * inv_pdf;
        ray->propagation.y *= ray->d.z * inv_pdf;
        ray->propagation.z *= ray->d.z * inv_pdf;
    } else if (p < (mat->ks + mat->kd)) {
        ray->d = cos_sample_hemisphere(r1, r2);
        ray->diffuse_bounce = 1;
        ray->propagation.x *= mat->diffuse.x;
        ray->propagation.y *= mat->diffuse.y;
        ray->propagation.z *= mat->diffuse.z;
    } else if (p < (mat->ks + mat->kd + mat->kt)) {
        if (sample_refraction(&ray->propagation, ray, mat->ior, mat->refExp, r1, r2)) {
            ray->extinction = mat->extinction;
        } else {
            ray->extinction.x = 0;
            ray->extinction.y = 0;
            ray->extinction.z = 0;
        }
        const float cwi = rt_fabsf(ray->d.z);
        ray->propagation.x *= cwi;
        ray->propagation.y *= cwi;
        ray->propagation.z *= cwi;
        ray->diffuse_bounce = 0;
    } else {
        return 0;
    }
    ray->d = shading_to_world(ray->d, hit->surface_normal);
    return 1;
}

/* rtcommon.h:267-365 (box branch :320-361: direct light, albedo 0.7, Lambert
   bounce — the bounce draws its two numbers even at the last depth) */
OR_API rt_vec3 or_trace_path(rt_ray *ray, const rt_sphere *s, uint32_t n, uint32_t max_depth, rt_seed *seed,
                             or_counters *cnt)
{
    const float bw = (float)RT_BOX_WIDTH, bh = (float)RT_BOX_HEIGHT;
    rt_vec3 color = {0.0f, 0.0f, 0.0f};
    for (uint32_t depth = 0; depth <= max_depth; ++depth) {
        cnt->closest++;
        int32_t hi = or_scene_intersection(ray, s, n);
        if (hi >= 0) {
            const rt_sphere *hs = &s[hi];
            rt_hit_info hit;
            hit.hit_pt.x = ray->o.x + ray->d.x * ray->tmax;
            hit.hit_pt.y = ray->o.y + ray->d.y * ray->tmax;
            hit.hit_pt.z = ray->o.z + ray->d.z * ray->tmax;
            sphere_normal(&hit, hs->center, hs->radius);
            if (ray->extinction.x > 0.0f) ray->propagation.x *= rt_expf(rt_logf(ray->extinction.x) * ray->tmax);
            if (ray->extinction.y > 0.0f) ray->propagation.y *= rt_expf(rt_logf(ray->extinction.y) * ray->tmax);
            if (ray->extinction.z > 0.0f) ray->propagation.z *= rt_expf(rt_logf(ray->extinction.z) * ray->tmax);
            if (!ray->diffuse_bounce && hs->mat.emission_power != 0) {
                color.x += ray->propagation.x * hs->mat.emission.x;
                color.y += ray->propagation.y * hs->mat.emission.y;
                color.z += ray->propagation.z * hs->mat.emission.z;
            }
            if (hs->mat.kd > 0.0f) {
                rt_vec3 direct = sample_direct_illumination(&hit, s, n, RT_LIGHT_SAMPLES, seed, cnt);
                const float scale = hs->mat.kd * RT_M_1_PI_F;
                color.x += ray->propagation.x * direct.x * hs->mat.diffuse.x * scale;
                color.y += ray->propagation.y * direct.y * hs->mat.diffuse.y * scale;
                color.z += ray->propagation.z * direct.z * hs->mat.diffuse.z * scale;
            }
            if (depth == max_depth) break;
            if (!or_sample_material(ray, &hit, &hs->mat, seed)) break;
        } else {
            float hd = or_intersects_box(ray, bw, bh, bw);
            if (hd > ray->tmin && hd < ray->tmax) {
                ray->tmax = hd;
                rt_hit_info hit;
                hit.hit_pt.x = ray->o.x + ray->d.x * ray->tmax;
                hit.hit_pt.y = ray->o.y + ray->d.y * ray->tmax;
                hit.hit_pt.z = ray->o.z + ray->d.z * ray->tmax;
                or_box_normal(&hit, bw, bh, bw);
                rt_vec3 direct = sample_direct_illumination(&hit, s, n, RT_LIGHT_SAMPLES, seed, cnt);
                const float scale = RT_M_1_PI_F;
                ray->propagation.x *= 0.7f;
                ray->propagation.y *= 0.7f;
                ray->propagation.z *= 0.7f;
                color.x += ray->propagation.x * direct.x * scale;
                color.y += ray->propagation.y * direct.y * scale;
                color.z += ray->propagation.z * direct.z * scale;
                ray->o = hit.hit_pt;
                ray->tmin = RT_SMALL_F;
                ray->tmax = rt_inff();
                float r1 = or_frand(seed);
                float r2 = or_frand(seed);
                ray->d = cos_sample_hemisphere(r1, r2);
                ray->d = shading_to_world(ray->d, hit.surface_normal);
                ray->diffuse_bounce = 1;
            } else {
                break;
            }
        }
    }
    return color;
}

/* rtcommon.h:371-470 — triangles are lit by the emissive spheres and never
   bounce; the box bounces. */
OR_API rt_vec3 or_trace_path_tri(rt_ray ray, const or_mesh *m, const rt_sphere *s, uint32_t n, uint32_t max_depth,
                                 rt_seed *seed, or_counters *cnt)
{
    const float bw = (float)RT_BOX_WIDTH, bh = (float)RT_BOX_HEIGHT;
    rt_vec3 color = {0.0f, 0.0f, 0.0f};
    rt_triangle ht;
    for (uint32_t depth = 0; depth <= max_depth; ++depth) {
        cnt->closest++;
        int32_t ti = mesh_closest(&ray, m);
        if (ti >= 0) {
            or_get_triangle(&ht, (uint32_t)ti, m->verts, m->idx);
            rt_hit_info hit;
            hit.hit_pt.x = ray.o.x + ray.d.x * ray.tmax;
            hit.hit_pt.y = ray.o.y + ray.d.y * ray.tmax;
            hit.hit_pt.z = ray.o.z + ray.d.z * ray.tmax;
            hit.surface_normal = cross_vec(ht.e2, ht.e1); /* unnormalised (rtcommon.h:389) */
            if (ray.extinction.x > 0.0f) ray.propagation.x *= rt_expf(rt_logf(ray.extinction.x) * ray.tmax);
            if (ray.extinction.y > 0.0f) ray.propagation.y *= rt_expf(rt_logf(ray.extinction.y) * ray.tmax);
            if (ray.extinction.z > 0.0f) ray.propagation.z *= rt_expf(rt_logf(ray.extinction.z) * ray.tmax);
            rt_vec3 direct = sample_direct_illumination_tri(&hit, m, s, n, seed, cnt);
            const float scale = 1.0f * RT_M_1_PI_F;
            color.x += ray.propagation.x * direct.x * scale * 0.7f;
            color.y += ray.propagation.y * direct.y * scale * 0.7f;
            color.z += ray.propagation.z * direct.z * scale * 0.7f;
            break; /* rtcommon.h:418-421: both exits break */
        } else {
            float hd = or_intersects_box(&ray, bw, bh, bw);
            if (hd > ray.tmin && hd < ray.tmax) {
                ray.tmax = hd;
                rt_hit_info hit;
                hit.hit_pt.x = ray.o.x + ray.d.x * ray.tmax;
                hit.hit_pt.y = ray.o.y + ray.d.y * ray.tmax;
                hit.hit_pt.z = ray.o.z + ray.d.z * ray.tmax;
                or_box_normal(&hit, bw, bh, bw);
                rt_vec3 direct = sample_direct_illumination_tri(&hit, m, s, n, seed, cnt);
                const float scale = RT_M_1_PI_F;
                ray.propagation.x *= 0.7f;
                ray.propagation.y *= 0.7f;
                ray.propagation.z *= 0.7f;
                color.x += ray.propagation.x * direct.x * scale;
                color.y += ray.propagation.y * direct.y * scale;
                color.z += ray.propagation.z * direct.z * scale;
                ray.o = hit.hit_pt;
                ray.tmin = RT_SMALL_F;
                ray.tmax = rt_inff();
                float r1 = or_frand(seed);
                float r2 = or_frand(seed);
                ray.d = cos_sample_hemisphere(r1, r2);
                ray.d = shading_to_world(ray.d, hit.surface_normal);
                ray.diffuse_bounce = 1;
            } else {
                break;
            }
        }
    }
    return color;
}

/* ----------------------------------------------------------- raytracer.cl */

enum { OR_KERNEL_SPHERES = 0, OR_KERNEL_SPHERES_SS = 1, OR_KERNEL_TRIS = 2 };

typedef struct or_frame {
    float *out;
    const rt_camera *cam;
    const rt_sphere *spheres;
    uint32_t n_spheres;
    uint32_t W, H, Wpad, Hpad;
    uint32_t sample_rate, max_depth, progressive;
    uint32_t *seeds;
    const or_mesh *mesh;
    int kernel;
    /* optional pixel subset (cpu baseline): pixels[i] = y*W+x, and a cap on the
       samples traced per pixel (a prefix of the pixel's own sample sequence) */
    const uint32_t *pixels;
    uint32_t n_pixels;
    uint32_t max_samples;
} or_frame;

/* raytracer.cl:81-85 / :149-153 / :221-224 — normalize(view + right*a + up*b)
   with the float4 w lanes (always 0) carried through the dot product. */
static rt_ray camera_ray(const rt_camera *cam, float a, float b)
{
    rt_float4 v;
    v.x = (cam->view.x + cam->right.x * a) + cam->up.x * b;
    v.y = (cam->view.y + cam->right.y * a) + cam->up.y * b;
    v.z = (cam->view.z + cam->right.z * a) + cam->up.z * b;
    v.w = (cam->view.w + cam->right.w * a) + cam->up.w * b;
    float len = rt_sqrtf(((v.x * v.x + v.y * v.y) + v.z * v.z) + v.w * v.w);
    rt_ray r;
    r.o.x = cam->position.x;
    r.o.y = cam->position.y;
    r.o.z = cam->position.z;
    r.d.x = v.x / len;
    r.d.y = v.y / len;
    r.d.z = v.z / len;
    r.tmin = RT_SMALL_F;
    r.tmax = rt_inff();
    r.propagation.x = r.propagation.y = r.propagation.z = 1.0f;
    r.extinction.x = r.extinction.y = r.extinction.z = 0.0f;
    r.diffuse_bounce = 0;
    return r;
}

/* One work-item: raytracer.cl:46-104 (spheres), :120-166 (single sample),
   :184-243 (triangles). */
static void render_pixel(const or_frame *f, uint32_t x, uint32_t y, or_counters *cnt)
{
    if (x >= f->W || y >= f->H) return;
    const uint32_t plane = f->Wpad * f->Hpad;
    uint32_t slot;
    if (f->kernel == OR_KERNEL_SPHERES)
        slot = ((y + f->progressive) % f->Hpad) * f->Wpad + x; /* raytracer.cl:20-24 */
    else
        slot = y * f->Wpad + x; /* raytracer.cl:142-144, :207-209 */
    rt_seed seed = {f->seeds[slot], f->seeds[plane + slot]};
    const float hw = ((float)f->W) / 2.0f, hh = ((float)f->H) / 2.0f;
    float px = 0.0f, py = 0.0f, pz = 0.0f, pw = 0.0f;
    uint32_t traced = 0;
    if (f->kernel == OR_KERNEL_SPHERES_SS) {
        float a = (float)x + or_frand(&seed);
        float b = (float)y + or_frand(&seed);
        rt_ray ray = camera_ray(f->cam, a - hw, b - hh);
        rt_vec3 c = or_trace_path(&ray, f->spheres, f->n_spheres, f->max_depth, &seed, cnt);
        px = c.x;
        py = c.y;
        pz = c.z;
    } else {
        const uint32_t sr = f->sample_rate;
        for (uint32_t sx = 0; sx < sr; ++sx) {
            for (uint32_t sy = 0; sy < sr; ++sy) {
                if (f->max_samples && traced >= f->max_samples) goto done;
                float a = (float)x + or_strat_rand(&seed, (int)sx, (int)sr);
                float b = (float)y + or_strat_rand(&seed, (int)sy, (int)sr);
                rt_ray ray = camera_ray(f->cam, a - hw, b - hh);
                rt_vec3 c;
                if (f->kernel == OR_KERNEL_TRIS)
                    c = or_trace_path_tri(ray, f->mesh, f->spheres, f->n_spheres, f->max_depth, &seed, cnt);
                else
                    c = or_trace_path(&ray, f->spheres, f->n_spheres, f->max_depth, &seed, cnt);
                px += c.x;
                py += c.y;
                pz += c.z;
                traced++;
            }
        }
        const float n = (float)(sr * sr);
        px /= n;
        py /= n;
        pz /= n;
        pw /= n;
    }
    if (f->progressive > 0) { /* OpenCL mix(a,b,t) = a + (b-a)*t */
        const float t = 1.0f / (float)f->progressive;
        const float *o = &f->out[4 * ((size_t)y * f->W + x)];
        px = o[0] + (px - o[0]) * t;
        py = o[1] + (py - o[1]) * t;
        pz = o[2] + (pz - o[2]) * t;
        pw = o[3] + (pw - o[3]) * t;
    }
    float *o = &f->out[4 * ((size_t)y * f->W + x)];
    o[0] = px;
    o[1] = py;
    o[2] = pz;
    o[3] = pw;
    f->seeds[slot] = seed.x;
    f->seeds[plane + slot] = seed.y;
done:
    return;
}

typedef struct or_job {
    const or_frame *f;
    int tid, nthreads;
    or_counters cnt;
} or_job;

static void *worker(void *arg)
{
    or_job *j = (or_job *)arg;
    const or_frame *f = j->f;
    or_counters cnt = {0, 0}; /* thread-local: the jobs' counters share cache lines */
    if (f->pixels) {
        for (uint32_t i = (uint32_t)j->tid; i < f->n_pixels; i += (uint32_t)j->nthreads)
            render_pixel(f, f->pixels[i] % f->W, f->pixels[i] / f->W, &cnt);
    } else {
        for (uint32_t y = (uint32_t)j->tid; y < f->H; y += (uint32_t)j->nthreads)
            for (uint32_t x = 0; x < f->W; ++x) render_pixel(f, x, y, &cnt);
    }
    j->cnt = cnt;
    return NULL;
}

static int run_frame(const or_frame *f, int nthreads, or_counters *cnt)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    or_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].f = f;
        jobs[t].tid = t;
        jobs[t].nthreads = nthreads;
        jobs[t].cnt.closest = jobs[t].cnt.shadow = 0;
    }
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) return -1;
    worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    if (cnt) {
        cnt->closest = cnt->shadow = 0;
        for (int t = 0; t < nthreads; ++t) {
            cnt->closest += jobs[t].cnt.closest;
            cnt->shadow += jobs[t].cnt.shadow;
        }
    }
    return 0;
}

/* raytrace (kernel 0) / raytrace_ss (kernel 1) over the whole frame. */
OR_API int or_render_spheres(float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n, uint32_t W, uint32_t H,
                             uint32_t Wpad, uint32_t Hpad, uint32_t sample_rate, uint32_t max_depth,
                             uint32_t progressive, uint32_t *seeds, int single_sample, int nthreads,
                             or_counters *cnt)
{
    or_frame f;
    memset(&f, 0, sizeof(f));
    f.out = out;
    f.cam = cam;
    f.spheres = s;
    f.n_spheres = n;
    f.W = W;
    f.H = H;
    f.Wpad = Wpad;
    f.Hpad = Hpad;
    f.sample_rate = sample_rate;
    f.max_depth = max_depth;
    f.progressive = progressive;
    f.seeds = seeds;
    f.kernel = single_sample ? OR_KERNEL_SPHERES_SS : OR_KERNEL_SPHERES;
    return run_frame(&f, nthreads, cnt);
}

/* raytrace_tris over the whole frame, or over a pixel subset with at most
   max_samples samples per pixel (0 = all); bvh: NULL for the reference's linear loops, or a
   tree from or_bvh_build over the same verts / idx (the same results, O(log N) per ray). */
OR_API int or_render_tris_bvh(float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n, uint32_t W,
                              uint32_t H, uint32_t Wpad, uint32_t Hpad, uint32_t sample_rate, uint32_t max_depth,
                              uint32_t progressive, uint32_t *seeds, const float *verts, const int32_t *idx,
                              uint32_t n_tris, const uint32_t *pixels, uint32_t n_pixels, uint32_t max_samples,
                              int nthreads, or_counters *cnt, const or_bvh *bvh)
{
    if (bvh && bvh->n_tris != n_tris) return -1;
    or_mesh m = {(const rt_vec3 *)verts, idx, n_tris, bvh};
    or_frame f;
    memset(&f, 0, sizeof(f));
    f.out = out;
    f.cam = cam;
    f.spheres = s;
    f.n_spheres = n;
    f.W = W;
    f.H = H;
    f.Wpad = Wpad;
    f.Hpad = Hpad;
    f.sample_rate = sample_rate;
    f.max_depth = max_depth;
    f.progressive = progressive;
    f.seeds = seeds;
    f.mesh = &m;
    f.kernel = OR_KERNEL_TRIS;
    f.pixels = pixels;
    f.n_pixels = n_pixels;
    f.max_samples = max_samples;
    return run_frame(&f, nthreads, cnt);
}

OR_API int or_render_tris(float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n, uint32_t W, uint32_t H,
                          uint32_t Wpad, uint32_t Hpad, uint32_t sample_rate, uint32_t max_depth,
                          uint32_t progressive, uint32_t *seeds, const float *verts, const int32_t *idx,
                          uint32_t n_tris, const uint32_t *pixels, uint32_t n_pixels, uint32_t max_samples,
                          int nthreads, or_counters *cnt)
{
    return or_render_tris_bvh(out, cam, s, n, W, H, Wpad, Hpad, sample_rate, max_depth, progressive, seeds, verts, idx,
                              n_tris, pixels, n_pixels, max_samples, nthreads, cnt, NULL);
}

/* Primary-ray closest hits for a batch of rays (hit index + t), linear
   traversal exactly as rtcommon.h:39-52.  Used for the hit-index parity
   tests against the GPU BVH. */
OR_API void or_closest_hits(const rt_ray *rays, uint32_t n_rays, const float *verts, const int32_t *idx,
                            uint32_t n_tris, int32_t *out_idx, float *out_t)
{
    for (uint32_t i = 0; i < n_rays; ++i) {
        rt_ray r = rays[i];
        out_idx[i] = or_scene_intersection_tri(&r, (const rt_vec3 *)verts, idx, n_tris);
        out_t[i] = r.tmax;
    }
}

OR_API void or_any_hits(const rt_ray *rays, uint32_t n_rays, const float *verts, const int32_t *idx,
                        uint32_t n_tris, int32_t *out_occluded)
{
    for (uint32_t i = 0; i < n_rays; ++i)
        out_occluded[i] = !or_visibility_test_tri(&rays[i], (const rt_vec3 *)verts, idx, n_tris);
}

/* The same two queries through the independent BVH mode (or_bvh_build over verts / idx). */
OR_API void or_closest_hits_bvh(const rt_ray *rays, uint32_t n_rays, const float *verts, const int32_t *idx,
                                const or_bvh *bvh, int32_t *out_idx, float *out_t)
{
    or_mesh m = {(const rt_vec3 *)verts, idx, bvh->n_tris, bvh};
    for (uint32_t i = 0; i < n_rays; ++i) {
        rt_ray r = rays[i];
        out_idx[i] = bvh_closest(&r, &m);
        out_t[i] = r.tmax;
    }
}

OR_API void or_any_hits_bvh(const rt_ray *rays, uint32_t n_rays, const float *verts, const int32_t *idx,
                            const or_bvh *bvh, int32_t *out_occluded)
{
    or_mesh m = {(const rt_vec3 *)verts, idx, bvh->n_tris, bvh};
    for (uint32_t i = 0; i < n_rays; ++i) out_occluded[i] = !bvh_visible(&rays[i], &m);
}

/* Host camera helper restated for the KAT (RayTracer.cpp:33-47 and
   RayTracerCL.cpp:178-215 are restated in the product library, not here). */
OR_API float or_math_sin(float x) { return rt_sinf(x); }
OR_API float or_math_cos(float x) { return rt_cosf(x); }
OR_API float or_math_exp(float x) { return rt_expf(x); }
OR_API float or_math_log(float x) { return rt_logf(x); }
OR_API float or_math_pow(float x, float y) { return rt_powf(x, y); }

/* Vectorised: the pinned builtins over whole argument ranges (tests/test_oracle_golden.py
   test_math_model_sanity).  fn: 0 sin, 1 cos, 2 exp, 3 log, 4 pow(x, y[0]), 5 / 6 the sine /
   cosine half of rt_sincosf (the triangle kernel's shared light / bounce direction). */
OR_API void or_math_vec(int fn, const float *x, const float *y, float *out, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        float s, c;
        switch (fn) {
        case 0: out[i] = rt_sinf(x[i]); break;
        case 1: out[i] = rt_cosf(x[i]); break;
        case 2: out[i] = rt_expf(x[i]); break;
        case 3: out[i] = rt_logf(x[i]); break;
        case 4: out[i] = rt_powf(x[i], y[0]); break;
        case 5: rt_sincosf(x[i], &s, &c); out[i] = s; break;
        default: rt_sincosf(x[i], &s, &c); out[i] = c; break;
        }
    }
}

/* Pointer-only wrappers for the per-function known-answer tests. */
OR_API float or_kat_intersect_sphere(const rt_ray *r, const rt_vec3 *c, float radius)
{
    return or_intersect_sphere(r, *c, radius);
}

OR_API void or_kat_emissive(rt_ray *r, const rt_vec3 *c, float radius, float r1, float r2)
{
    or_sphere_emissive_radiance(r, *c, radius, r1, r2);
}
