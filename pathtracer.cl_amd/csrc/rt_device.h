/*
 * rt_device.h — device-side path-tracing primitives for gfx950.
 *
 * The sampling / shading arithmetic is the reference (clrt/ocl headers), kept in
 * the same IEEE operation order so results are bit-identical to the OpenCL
 * kernel under the pinned model of include/rt_math.h (compiled with
 * -ffp-contract=off; HIP's f32 division and sqrt are correctly rounded).
 * Data layout and control flow are the MI355X design:
 * vectors live in registers as V3, scene records are read through scalar
 * loads, and the path state machine lives in rt_kernels.hip.
 */
#ifndef RT_DEVICE_H
#define RT_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_math.h"
#include "rt_types.h"

#pragma clang fp contract(off)

#define RTD static __device__ __forceinline__

struct V3 {
    float x, y, z;
};

RTD V3 v3(float x, float y, float z)
{
    V3 r;
    r.x = x;
    r.y = y;
    r.z = z;
    return r;
}
RTD V3 v3f(rt_vec3 a) { return v3(a.x, a.y, a.z); }
/* DOT() of geometryFuncs.h:6: (a.x*b.x + a.y*b.y) + a.z*b.z */
RTD float dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* cross_vec, geometryFuncs.h:29-32 */
RTD V3 cross3(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

struct Seed {
    uint32_t x, y;
};

/* MWC generator, rng.h:24-42 */
RTD float frand(Seed &s)
{
    s.x = 36969u * (s.x & 65535u) + (s.x >> 16);
    s.y = 18000u * (s.y & 65535u) + (s.y >> 16);
    uint32_t bits = (s.x << 16) + s.y;
    bits = (bits & 0x007fffffu) | 0x40000000u;
    return (__uint_as_float(bits) - 2.0f) / 2.0f;
}

/* rng.h:45-47 */
RTD float strat_rand(Seed &s, int cur, int total)
{
    float f = frand(s);
    return ((float)cur + f) / (float)total;
}

/* geometryFuncs.h:13-27 */
RTD V3 perpendicular(V3 v)
{
    if (rt_fabsf(v.y) > 0.9f) {
        float inv = rt_rsqrtf(v.z * v.z + v.y * v.y);
        return v3(0.0f, -v.z * inv, v.y * inv);
    }
    float inv = rt_rsqrtf(v.z * v.z + v.x * v.x);
    return v3(v.z * inv, 0.0f, -v.x * inv);
}

/* materials.h:44-50 */
RTD V3 shading_to_world(V3 v, V3 n)
{
    V3 tx = perpendicular(n);
    V3 ty = cross3(n, tx);
    return v3(tx.x * v.x + ty.x * v.y + n.x * v.z, tx.y * v.x + ty.y * v.y + n.y * v.z,
              tx.z * v.x + ty.z * v.y + n.z * v.z);
}

/* materials.h:59-65 */
RTD V3 world_to_shading(V3 w, V3 n)
{
    V3 tx = perpendicular(n);
    V3 ty = cross3(n, tx);
    return v3(dot3(w, tx), dot3(w, ty), dot3(w, n));
}

/* materials.h:21-35 */
RTD V3 cos_sample_hemisphere(float r1, float r2)
{
    float ct = rt_sqrtf(1.0f - r1);
    float st = rt_sqrtf(1.0f - ct * ct);
    float phi = RT_M_2PI_F * r2;
    return v3(st * rt_cosf(phi), st * rt_sinf(phi), ct);
}

/* geometryFuncs.h:41-56 */
RTD float intersect_sphere(V3 o, V3 d, float tmin, V3 c, float radius)
{
    float ox = o.x - c.x;
    float oy = o.y - c.y;
    float oz = o.z - c.z;
    float dist2 = ox * ox + oy * oy + oz * oz;
    float b_neg = -(ox * d.x + oy * d.y + oz * d.z);
    float disc = b_neg * b_neg - (dist2 - radius * radius);
    if (disc > 0) {
        float sq = rt_sqrtf(disc);
        if (b_neg - sq > tmin) return b_neg - sq;
        return b_neg + sq;
    }
    return 0.0f;
}

/* geometryFuncs.h:86-150 for the origin-centred box of raytracer.cl:16-17 */
RTD float intersect_box(V3 o, V3 d, float tmin, float xs, float ys, float zs)
{
    float nt = 0.0f, ft = rt_inff();
    float t1, t2;
    if (d.x != 0) {
        t1 = (0.0f - xs - o.x) / d.x;
        t2 = (0.0f + xs - o.x) / d.x;
        nt = rt_minf(t1, t2);
        ft = rt_maxf(t1, t2);
    } else if (rt_fabsf(o.x - 0.0f) > xs) {
        return 0;
    }
    if (d.y != 0) {
        t1 = (0.0f - ys - o.y) / d.y;
        t2 = (0.0f + ys - o.y) / d.y;
        if (t1 > t2) {
            nt = rt_maxf(t2, nt);
            ft = rt_minf(t1, ft);
        } else {
            nt = rt_maxf(t1, nt);
            ft = rt_minf(t2, ft);
        }
    } else if (rt_fabsf(o.y - 0.0f) > ys) {
        return 0;
    }
    if (d.z != 0) {
        t1 = (0.0f - zs - o.z) / d.z;
        t2 = (0.0f + zs - o.z) / d.z;
        if (t1 > t2) {
            nt = rt_maxf(t2, nt);
            ft = rt_minf(t1, ft);
        } else {
            nt = rt_maxf(t1, nt);
            ft = rt_minf(t2, ft);
        }
    } else if (rt_fabsf(o.z - 0.0f) > zs) {
        return 0;
    }
    if (nt > ft || ft < tmin) return rt_inff();
    if (nt < tmin) return ft;
    return nt;
}

/* geometryFuncs.h:71-84 */
RTD V3 box_normal(V3 p, float xs, float ys, float zs)
{
    float dx = rt_fabsf(rt_fabsf(p.x) - xs);
    float dy = rt_fabsf(rt_fabsf(p.y) - ys);
    float dz = rt_fabsf(rt_fabsf(p.z) - zs);
    if (dx < dy && dx < dz) return v3(-p.x / rt_fabsf(p.x), 0.0f, 0.0f);
    if (dy < dz) return v3(0.0f, -p.y / rt_fabsf(p.y), 0.0f);
    return v3(0.0f, 0.0f, -p.z / rt_fabsf(p.z));
}

/* materials.h:232-271: direction toward a uniformly sampled point of the
   light's subtended cone; tmin = SMALL_F, tmax = hit distance - SMALL_F.  */
RTD V3 sphere_light_dir(V3 o, V3 c, float radius, float r1, float r2, float &tmax)
{
    V3 dir = v3(c.x - o.x, c.y - o.y, c.z - o.z);
    float inv = rt_rsqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
    dir.x *= inv;
    dir.y *= inv;
    dir.z *= inv;
    float sin_max = radius * inv;
    float cos_max = rt_sqrtf(1.0f - sin_max * sin_max);
    float ct = 1.0f + r1 * (cos_max - 1.0f);
    float st = rt_sqrtf(1.0f - ct * ct);
    float phi = RT_M_2PI_F * r2;
    V3 d = shading_to_world(v3(rt_cosf(phi) * st, rt_sinf(phi) * st, ct), dir);
    tmax = intersect_sphere(o, d, RT_SMALL_F, c, radius) - RT_SMALL_F;
    return d;
}

/* ---- sphere-scene materials (rtcommon.h:184-251, materials.h:76-218) ---- */

struct PathRay {
    V3 o, d;
    float tmin, tmax;
    V3 prop, ext;
    uint32_t diffuse;
};

/* materials.h:76-108 */
RTD V3 sample_phong(V3 w, float spec_exp, float r1, float r2)
{
    V3 wi = v3(-w.x, -w.y, w.z);
    if (spec_exp < 100000.0f) {
        float cos_a = rt_powf(r1, 1.0f / (spec_exp + 1.0f));
        float st = rt_sqrtf(1.0f - cos_a * cos_a);
        float phi = RT_M_2PI_F * r2;
        wi = v3(rt_cosf(phi) * st, rt_sinf(phi) * st, cos_a);
        float wo_dot_wh = dot3(w, wi);
        wi.x = -w.x + 2.0f * wo_dot_wh * wi.x;
        wi.y = -w.y + 2.0f * wo_dot_wh * wi.y;
        wi.z = -w.z + 2.0f * wo_dot_wh * wi.z;
    }
    return wi;
}

/* materials.h:146-218 */
RTD bool sample_refraction(PathRay &r, float ior, float blur_exp, float r1, float r2)
{
    float cos_wo = rt_fabsf(r.d.z);
    bool entering = r.d.z > 0;
    float ei = entering ? 1.0f : ior;
    float eo = entering ? ior : 1.0f;
    float ratio = ei / eo;
    float cos_sq = 1.0f - (ratio * ratio * (1.0f - r.d.z * r.d.z));
    if (cos_sq < 0.0f) {
        r.d.x *= -1.0f;
        r.d.y *= -1.0f;
        return !entering;
    }
    float ct = rt_sqrtf(cos_sq);
    if (entering) ct = -ct;
    V3 wi = v3(-r.d.x * ratio, -r.d.y * ratio, ct);
    if (blur_exp < 100000.0f) {
        float cos_a = rt_powf(r1, 1.0f / (blur_exp + 1.0f));
        float st = rt_sqrtf(1.0f - cos_a * cos_a);
        float phi = RT_M_2PI_F * r2;
        wi = v3(rt_cosf(phi) * st, rt_sinf(phi) * st, cos_a);
        float wo_dot_wh = dot3(r.d, wi);
        wi.x = -r.d.x + 2.0f * wo_dot_wh * wi.x;
        wi.y = -r.d.y + 2.0f * wo_dot_wh * wi.y;
        wi.z = -r.d.z + 2.0f * wo_dot_wh * wi.z;
    }
    r.d = wi;
    ct = rt_fabsf(ct);
    float parl = (eo * cos_wo - ei * ct) / (eo * cos_wo + ei * ct);
    float perp = (ei * cos_wo - eo * ct) / (ei * cos_wo + eo * ct);
    float fres = (parl * parl + perp * perp) * 0.5f;
    fres = (1.0f - fres) / ct;
    r.prop.x *= fres;
    r.prop.y *= fres;
    r.prop.z *= fres;
    return entering;
}

/* rtcommon.h:184-251 */
RTD bool sample_material(PathRay &r, V3 hit_pt, V3 n, const rt_material &m, Seed &seed)
{
    r.o = hit_pt;
    r.d = world_to_shading(v3(r.d.x * -1.0f, r.d.y * -1.0f, r.d.z * -1.0f), n);
    r.tmin = RT_SMALL_F;
    r.tmax = rt_inff();
    float p = frand(seed);
    float r1 = frand(seed);
    float r2 = frand(seed);
    if (p < m.ks) {
        r.d = sample_phong(r.d, m.specExp, r1, r2); /* pdf == 1: 1.0/pdf == 1 */
        r.diffuse = 0;
        r.prop.x *= r.d.z * 1.0f;
        r.prop.y *= r.d.z * 1.0f;
        r.prop.z *= r.d.z * 1.0f;
    } else if (p < (m.ks + m.kd)) {
        r.d = cos_sample_hemisphere(r1, r2);
        r.diffuse = 1;
        r.prop.x *= m.diffuse.x;
        r.prop.y *= m.diffuse.y;
        r.prop.z *= m.diffuse.z;
    } else if (p < (m.ks + m.kd + m.kt)) {
        if (sample_refraction(r, m.ior, m.refExp, r1, r2))
            r.ext = v3f(m.extinction);
        else
            r.ext = v3(0.0f, 0.0f, 0.0f);
        const float cwi = rt_fabsf(r.d.z);
        r.prop.x *= cwi;
        r.prop.y *= cwi;
        r.prop.z *= cwi;
        r.diffuse = 0;
    } else {
        return false;
    }
    r.d = shading_to_world(r.d, n);
    return true;
}

#endif /* RT_DEVICE_H */
