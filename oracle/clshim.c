/*
 * clshim.c — OpenCL C builtins for running the reference kernel on the host
 * (TEST INFRASTRUCTURE ONLY; container-side, builds oracle/_ref).
 *
 * The reference's clrt/ocl/raytracer.cl is compiled UNCHANGED, from where it
 * lies under /root/reference, by ROCm clang for x86-64 (oracle/Makefile).
 * Clang leaves 16 OpenCL builtins as external calls; this file defines them:
 *   - the NDRange query functions, backed by per-thread ids that the driver
 *     (ref_driver.c) sets before each work-item, and
 *   - the math builtins, mapped to the pinned arithmetic model in
 *     include/rt_math.h — the same implementations the HIP kernels use.
 * The OpenCL spec leaves builtin accuracy to the implementation, so defining
 * these is exactly the "pinned model" of SURVEY.md §8c; nothing of the
 * reference's algorithm lives here.
 *
 * Symbols use the Itanium-mangled names clang emits for OpenCL overloads.
 *
 * Built with -DCLSHIM_LIBM (oracle/Makefile `ref_libm` -> oracle/_ref_libm/) the
 * transcendentals come from glibc's libm instead (sinf, cosf, expf, logf, powf: another
 * conforming OpenCL builtin library).  That second build of the unchanged reference
 * measures how much the result depends on the builtin library the pinned model fixes
 * (oracle/libm_sensitivity.py).
 */
#include <stddef.h>
#include <stdint.h>

#include "rt_math.h"
#ifdef CLSHIM_LIBM
#include <math.h>
#define SHIM_SIN(x) sinf(x)
#define SHIM_COS(x) cosf(x)
#define SHIM_EXP(x) expf(x)
#define SHIM_LOG(x) logf(x)
#define SHIM_POW(x, y) powf(x, y)
#else
#define SHIM_SIN(x) rt_sinf(x)
#define SHIM_COS(x) rt_cosf(x)
#define SHIM_EXP(x) rt_expf(x)
#define SHIM_LOG(x) rt_logf(x)
#define SHIM_POW(x, y) rt_powf(x, y)
#endif

typedef float float4 __attribute__((ext_vector_type(4)));

__thread size_t clshim_gid[3];
__thread size_t clshim_gsz[3] = {1, 1, 1};

#define CLSYM(name) __asm__(name)

size_t cl_get_global_id(unsigned d) CLSYM("_Z13get_global_idj");
size_t cl_get_global_id(unsigned d) { return d < 3 ? clshim_gid[d] : 0; }

size_t cl_get_global_size(unsigned d) CLSYM("_Z15get_global_sizej");
size_t cl_get_global_size(unsigned d) { return d < 3 ? clshim_gsz[d] : 1; }

float cl_cos(float x) CLSYM("_Z3cosf");
float cl_cos(float x) { return SHIM_COS(x); }
float cl_sin(float x) CLSYM("_Z3sinf");
float cl_sin(float x) { return SHIM_SIN(x); }
float cl_exp(float x) CLSYM("_Z3expf");
float cl_exp(float x) { return SHIM_EXP(x); }
float cl_log(float x) CLSYM("_Z3logf");
float cl_log(float x) { return SHIM_LOG(x); }
float cl_pow(float x, float y) CLSYM("_Z3powff");
float cl_pow(float x, float y) { return SHIM_POW(x, y); }
float cl_sqrt(float x) CLSYM("_Z4sqrtf");
float cl_sqrt(float x) { return rt_sqrtf(x); }
float cl_rsqrt(float x) CLSYM("_Z5rsqrtf");
float cl_rsqrt(float x) { return rt_rsqrtf(x); }
float cl_fabs(float x) CLSYM("_Z4fabsf");
float cl_fabs(float x) { return rt_fabsf(x); }
float cl_min(float x, float y) CLSYM("_Z3minff");
float cl_min(float x, float y) { return rt_minf(x, y); }
float cl_max(float x, float y) CLSYM("_Z3maxff");
float cl_max(float x, float y) { return rt_maxf(x, y); }

/* mix(a, b, t) = a + (b - a) * t (OpenCL 1.2 §6.12.4) */
float4 cl_mix(float4 a, float4 b, float t) CLSYM("_Z3mixDv4_fS_f");
float4 cl_mix(float4 a, float4 b, float t)
{
    float4 r;
    r.x = a.x + (b.x - a.x) * t;
    r.y = a.y + (b.y - a.y) * t;
    r.z = a.z + (b.z - a.z) * t;
    r.w = a.w + (b.w - a.w) * t;
    return r;
}

/* normalize(v) pinned as v / sqrt(((x*x + y*y) + z*z) + w*w) */
float4 cl_normalize(float4 v) CLSYM("_Z9normalizeDv4_f");
float4 cl_normalize(float4 v)
{
    float l = rt_sqrtf(((v.x * v.x + v.y * v.y) + v.z * v.z) + v.w * v.w);
    float4 r;
    r.x = v.x / l;
    r.y = v.y / l;
    r.z = v.z / l;
    r.w = v.w / l;
    return r;
}

float4 cl_vload4(size_t off, const float *p) CLSYM("_Z6vload4mPU8CLglobalKf");
float4 cl_vload4(size_t off, const float *p)
{
    float4 r;
    r.x = p[4 * off];
    r.y = p[4 * off + 1];
    r.z = p[4 * off + 2];
    r.w = p[4 * off + 3];
    return r;
}

void cl_vstore4(float4 v, size_t off, float *p) CLSYM("_Z7vstore4Dv4_fmPU8CLglobalf");
void cl_vstore4(float4 v, size_t off, float *p)
{
    p[4 * off] = v.x;
    p[4 * off + 1] = v.y;
    p[4 * off + 2] = v.z;
    p[4 * off + 3] = v.w;
}
