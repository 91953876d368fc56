/*
 * ref_driver.c — NDRange driver for the reference kernel compiled for x86-64
 * (TEST INFRASTRUCTURE ONLY; container-side, part of oracle/_ref/libptref.so).
 *
 * Reproduces what RayTracerCL does around clEnqueueNDRangeKernel
 * (clrt/RayTracerCL.cpp:229-232, :289-292): a padded global range
 * (Wpad x Hpad, the overdraw region returning early inside the kernel), one
 * call per work-item with get_global_id/get_global_size answered by clshim.c.
 * Work-items are independent (each owns its pixel and seed slot), so rows are
 * split across threads; the output is bit-identical for any thread count.
 *
 * Also exports thin pointer-based wrappers around the reference's own helper
 * functions (every helper is an external symbol of the compiled object) for
 * the per-function known-answer fixtures.
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "rt_types.h"

typedef float float4 __attribute__((ext_vector_type(4)));

extern __thread size_t clshim_gid[3];
extern __thread size_t clshim_gsz[3];

/* Kernel bodies as emitted by clang for the three __kernel functions of
   clrt/ocl/raytracer.cl (:46, :120, :184). */
void __clang_ocl_kern_imp_raytrace(float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n, uint32_t W,
                                   uint32_t H, uint32_t sr, uint32_t depth, uint32_t prog, uint32_t *seeds);
void __clang_ocl_kern_imp_raytrace_ss(float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n, uint32_t W,
                                      uint32_t H, uint32_t depth, uint32_t prog, uint32_t *seeds);
void __clang_ocl_kern_imp_raytrace_tris(float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n, uint32_t W,
                                        uint32_t H, uint32_t sr, uint32_t depth, uint32_t prog, uint32_t *seeds,
                                        const rt_vec3 *verts, const int32_t *idx, uint32_t n_tris);

/* Reference helpers (rng.h, geometryFuncs.h, materials.h, rtcommon.h). */
float frand(rt_seed *seed);
float strat_rand(rt_seed *seed, int cur, int total);
float intersectSphere(const rt_ray *ray, rt_vec3 c, float r);
float intersectsBox(const rt_ray *ray, float4 center, float xs, float ys, float zs);
void boxNormal(const rt_ray *ray, rt_hit_info *hit, float xs, float ys, float zs);
_Bool intersects_triangle(rt_ray *ray, float *u, float *v, const rt_triangle *tri);
_Bool intersects_triangle_p(const rt_ray *ray, const rt_triangle *tri);
float sphereEmissiveRadiance(rt_ray *ray, rt_vec3 c, float r, float r1, float r2);
_Bool sample_material(rt_ray *ray, const rt_hit_info *hit, const rt_material *mat, rt_seed *seed);
void get_triangle(rt_triangle *t, uint32_t i, const rt_vec3 *verts, const int32_t *idx);
int scene_intersection_tri(rt_ray *ray, const rt_vec3 *verts, const int32_t *idx, uint32_t n);
_Bool visibility_test_tri(const rt_ray *ray, const rt_vec3 *verts, const int32_t *idx, uint32_t n);

#define REF_API __attribute__((visibility("default")))

enum { REF_SPHERES = 0, REF_SPHERES_SS = 1, REF_TRIS = 2 };

typedef struct ref_launch {
    int kernel;
    float *out;
    const rt_camera *cam;
    const rt_sphere *s;
    uint32_t n, W, H, Wpad, Hpad, sr, depth, prog;
    uint32_t *seeds;
    const rt_vec3 *verts;
    const int32_t *idx;
    uint32_t n_tris;
    int tid, nthreads;
} ref_launch;

static void *ref_worker(void *arg)
{
    ref_launch *L = (ref_launch *)arg;
    clshim_gsz[0] = L->Wpad;
    clshim_gsz[1] = L->Hpad;
    clshim_gsz[2] = 1;
    clshim_gid[2] = 0;
    for (uint32_t y = (uint32_t)L->tid; y < L->Hpad; y += (uint32_t)L->nthreads) {
        for (uint32_t x = 0; x < L->Wpad; ++x) {
            clshim_gid[0] = x;
            clshim_gid[1] = y;
            switch (L->kernel) {
            case REF_SPHERES:
                __clang_ocl_kern_imp_raytrace(L->out, L->cam, L->s, L->n, L->W, L->H, L->sr, L->depth, L->prog,
                                              L->seeds);
                break;
            case REF_SPHERES_SS:
                __clang_ocl_kern_imp_raytrace_ss(L->out, L->cam, L->s, L->n, L->W, L->H, L->depth, L->prog,
                                                 L->seeds);
                break;
            default:
                __clang_ocl_kern_imp_raytrace_tris(L->out, L->cam, L->s, L->n, L->W, L->H, L->sr, L->depth,
                                                   L->prog, L->seeds, L->verts, L->idx, L->n_tris);
            }
        }
    }
    return NULL;
}

/* One clEnqueueNDRangeKernel + finish() of the chosen reference kernel. */
REF_API int ref_launch_kernel(int kernel, float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n,
                              uint32_t W, uint32_t H, uint32_t Wpad, uint32_t Hpad, uint32_t sr, uint32_t depth,
                              uint32_t prog, uint32_t *seeds, const float *verts, const int32_t *idx,
                              uint32_t n_tris, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 128) nthreads = 128;
    if (Wpad < W || Hpad < H) return -1;
    ref_launch L[128];
    pthread_t th[128];
    for (int t = 0; t < nthreads; ++t) {
        ref_launch l = {kernel, out, cam, s, n, W, H, Wpad, Hpad, sr, depth, prog, seeds,
                        (const rt_vec3 *)verts, idx, n_tris, t, nthreads};
        L[t] = l;
    }
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[t], NULL, ref_worker, &L[t]) != 0) return -2;
    ref_worker(&L[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* The same launch restricted to a pixel subset (pixels[i] = y*W + x): bench.py's
   bounded CPU baseline runs the reference kernel on strided whole pixels.  Each
   work-item is the kernel's own (same gid, same padded global size), so every listed
   pixel and seed slot ends exactly as in a full launch. */
typedef struct ref_pixels_job {
    ref_launch L;
    const uint32_t *pixels;
    uint32_t n_pixels;
} ref_pixels_job;

static void *ref_pixels_worker(void *arg)
{
    ref_pixels_job *J = (ref_pixels_job *)arg;
    ref_launch *L = &J->L;
    clshim_gsz[0] = L->Wpad;
    clshim_gsz[1] = L->Hpad;
    clshim_gsz[2] = 1;
    clshim_gid[2] = 0;
    for (uint32_t i = (uint32_t)L->tid; i < J->n_pixels; i += (uint32_t)L->nthreads) {
        clshim_gid[0] = J->pixels[i] % L->W;
        clshim_gid[1] = J->pixels[i] / L->W;
        if (L->kernel == REF_TRIS)
            __clang_ocl_kern_imp_raytrace_tris(L->out, L->cam, L->s, L->n, L->W, L->H, L->sr, L->depth, L->prog,
                                               L->seeds, L->verts, L->idx, L->n_tris);
        else
            __clang_ocl_kern_imp_raytrace(L->out, L->cam, L->s, L->n, L->W, L->H, L->sr, L->depth, L->prog,
                                          L->seeds);
    }
    return NULL;
}

REF_API int ref_launch_pixels(int kernel, float *out, const rt_camera *cam, const rt_sphere *s, uint32_t n,
                              uint32_t W, uint32_t H, uint32_t Wpad, uint32_t Hpad, uint32_t sr, uint32_t depth,
                              uint32_t prog, uint32_t *seeds, const float *verts, const int32_t *idx,
                              uint32_t n_tris, const uint32_t *pixels, uint32_t n_pixels, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 128) nthreads = 128;
    if (Wpad < W || Hpad < H || (kernel != REF_TRIS && kernel != REF_SPHERES)) return -1;
    for (uint32_t i = 0; i < n_pixels; ++i)
        if (pixels[i] >= W * H) return -1;
    ref_pixels_job J[128];
    pthread_t th[128];
    for (int t = 0; t < nthreads; ++t) {
        ref_launch l = {kernel, out, cam, s, n, W, H, Wpad, Hpad, sr, depth, prog, seeds,
                        (const rt_vec3 *)verts, idx, n_tris, t, nthreads};
        J[t].L = l;
        J[t].pixels = pixels;
        J[t].n_pixels = n_pixels;
    }
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[t], NULL, ref_pixels_worker, &J[t]) != 0) return -2;
    ref_pixels_worker(&J[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* ---- per-function known-answer wrappers --------------------------------- */

REF_API void ref_frand_seq(rt_seed *seed, float *out, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i) out[i] = frand(seed);
}

REF_API void ref_strat_seq(rt_seed *seed, float *out, uint32_t n, int total)
{
    for (uint32_t i = 0; i < n; ++i) out[i] = strat_rand(seed, (int)(i % (uint32_t)total), total);
}

REF_API float ref_intersect_sphere(const rt_ray *ray, const rt_vec3 *c, float r) { return intersectSphere(ray, *c, r); }

REF_API float ref_intersects_box(const rt_ray *ray, float xs, float ys, float zs)
{
    float4 c = {0.0f, 0.0f, 0.0f, 0.0f};
    return intersectsBox(ray, c, xs, ys, zs);
}

REF_API void ref_box_normal(const rt_ray *ray, rt_hit_info *hit, float xs, float ys, float zs)
{
    boxNormal(ray, hit, xs, ys, zs);
}

REF_API int ref_intersects_triangle(rt_ray *ray, float *u, float *v, const rt_triangle *tri)
{
    return intersects_triangle(ray, u, v, tri) ? 1 : 0;
}

REF_API int ref_intersects_triangle_p(const rt_ray *ray, const rt_triangle *tri)
{
    return intersects_triangle_p(ray, tri) ? 1 : 0;
}

REF_API void ref_sphere_emissive(rt_ray *ray, const rt_vec3 *c, float r, float r1, float r2)
{
    (void)sphereEmissiveRadiance(ray, *c, r, r1, r2);
}

REF_API int ref_sample_material(rt_ray *ray, const rt_hit_info *hit, const rt_material *mat, rt_seed *seed)
{
    return sample_material(ray, hit, mat, seed) ? 1 : 0;
}

REF_API void ref_closest_hits(const rt_ray *rays, uint32_t n_rays, const float *verts, const int32_t *idx,
                              uint32_t n_tris, int32_t *out_idx, float *out_t)
{
    for (uint32_t i = 0; i < n_rays; ++i) {
        rt_ray r = rays[i];
        out_idx[i] = scene_intersection_tri(&r, (const rt_vec3 *)verts, idx, n_tris);
        out_t[i] = r.tmax;
    }
}

REF_API void ref_any_hits(const rt_ray *rays, uint32_t n_rays, const float *verts, const int32_t *idx,
                          uint32_t n_tris, int32_t *out_occluded)
{
    for (uint32_t i = 0; i < n_rays; ++i)
        out_occluded[i] = visibility_test_tri(&rays[i], (const rt_vec3 *)verts, idx, n_tris) ? 0 : 1;
}
