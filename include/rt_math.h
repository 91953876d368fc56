/*
 * rt_math.h — the pinned arithmetic model.
 *
 * OpenCL leaves the accuracy of sin/cos/exp/log/pow/rsqrt/normalize to the
 * implementation, so "the reference's result" is only defined once those
 * builtins are fixed.  This header fixes them, and it is compiled into all
 * three parties that must agree bit for bit:
 *   - the HIP kernels (device, gfx950),
 *   - the CPU oracle restatement (oracle/pt_oracle.c),
 *   - the builtin shim that the reference's own raytracer.cl is linked
 *     against when it is compiled for x86 (oracle/clshim.c).
 *
 * Rules that make the results identical on x86 and gfx950:
 *   - only IEEE-754 +, -, *, / and sqrt, each correctly rounded, in binary32
 *     or binary64; no FMA contraction (every TU is built with
 *     -ffp-contract=off; HIP division/sqrt are correctly rounded by default);
 *   - integer/bit manipulation for range reduction and scaling;
 *   - no calls into libm or the device math library.
 *
 * sin/cos/exp/log follow Cephes' single-precision algorithms (S. Moshier,
 * public algorithms: Cody-Waite reduction + minimax polynomials); pow is
 * evaluated as exp(y*log(x)) in binary64 and rounded once to binary32.
 * Accuracy: sin/cos ≤ 2 ulp for |x| < 8192 (the kernels only ever pass
 * 2π·U[0,1)), exp/log ≤ 2 ulp, pow ≈ correctly rounded for x ≥ 0.
 */
#ifndef RT_MATH_H
#define RT_MATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define RT_HD static __host__ __device__ __forceinline__
#else
#define RT_HD static inline
#endif

#define RT_INF_BITS 0x7f800000u
#define RT_M_PI_F 3.14159265358979323846f   /* materials.h:11 */
#define RT_M_1_PI_F 0.318309886f            /* materials.h:12 */
#define RT_M_2PI_F 6.283185307f             /* materials.h:15 */

RT_HD uint32_t rt_f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
RT_HD float rt_u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
RT_HD uint64_t rt_d2u(double f) { uint64_t u; __builtin_memcpy(&u, &f, 8); return u; }
RT_HD double rt_u2d(uint64_t u) { double f; __builtin_memcpy(&f, &u, 8); return f; }

RT_HD float rt_inff(void) { return rt_u2f(RT_INF_BITS); }
RT_HD float rt_nanf(void) { return rt_u2f(0x7fc00000u); }
RT_HD int rt_isnanf(float x) { return (rt_f2u(x) & 0x7fffffffu) > RT_INF_BITS; }

/* OpenCL fabs / min / max (min: y<x?y:x, max: x<y?y:x — OpenCL 1.2 §6.12.4). */
RT_HD float rt_fabsf(float x) { return rt_u2f(rt_f2u(x) & 0x7fffffffu); }
RT_HD float rt_minf(float x, float y) { return (y < x) ? y : x; }
RT_HD float rt_maxf(float x, float y) { return (x < y) ? y : x; }

/* Correctly rounded square root on both sides (sqrtss / the gfx950 CR sequence). */
RT_HD float rt_sqrtf(float x) { return __builtin_sqrtf(x); }
/* rsqrt pinned as 1/sqrt. */
RT_HD float rt_rsqrtf(float x) { return 1.0f / __builtin_sqrtf(x); }

/* 2^n as a float, n in [-126, 127]. */
RT_HD float rt_pow2i(int n) { return rt_u2f((uint32_t)(n + 127) << 23); }

/* z * 2^n with a single rounding (z in about [0.5, 2]). */
RT_HD float rt_ldexpf(float z, int n)
{
    if (n > 127) {
        if (n > 254) return z * rt_inff();
        return (z * rt_pow2i(127)) * rt_pow2i(n - 127);
    }
    if (n < -126) {
        if (n < -151 - 24) return z * 0.0f;
        /* first an exact scaling into the normal range, then one rounding */
        return (z * rt_pow2i(n + 126)) * rt_pow2i(-126);
    }
    return z * rt_pow2i(n);
}

/* ---- sin / cos (Cephes sinf.c / cosf.c structure) ---------------------- */
#define RT_FOPI 1.27323954473516f
#define RT_DP1 0.78515625f
#define RT_DP2 2.4187564849853515625e-4f
#define RT_DP3 3.77489497744594108e-8f

RT_HD float rt_sin_poly(float x, float z)
{
    float y = -1.9515295891e-4f * z;
    y = y + 8.3321608736e-3f;
    y = y * z;
    y = y - 1.6666654611e-1f;
    y = y * z;
    y = y * x;
    return y + x;
}

RT_HD float rt_cos_poly(float z)
{
    float y = 2.443315711809948e-5f * z;
    y = y - 1.388731625493765e-3f;
    y = y * z;
    y = y + 4.166664568298827e-2f;
    y = y * z;
    y = y * z;
    y = y - 0.5f * z;
    return y + 1.0f;
}

/* Shared octant reduction: returns r in [-pi/4, pi/4] and octant j in 0..7. */
RT_HD float rt_trig_reduce(float ax, int *jout)
{
    int j = (int)(ax * RT_FOPI);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    *jout = j & 7;
    float r = ax - y * RT_DP1;
    r = r - y * RT_DP2;
    r = r - y * RT_DP3;
    return r;
}

RT_HD float rt_sinf(float x)
{
    float ax = rt_fabsf(x);
    if (!(ax < 1.0e7f)) return x - x; /* inf / nan / out of the reduced range */
    int sign = (x < 0.0f) ? -1 : 1;
    int j;
    float r = rt_trig_reduce(ax, &j);
    if (j > 3) { sign = -sign; j -= 4; }
    float z = r * r;
    float y = (j == 1 || j == 2) ? rt_cos_poly(z) : rt_sin_poly(r, z);
    return (sign < 0) ? -y : y;
}

RT_HD float rt_cosf(float x)
{
    float ax = rt_fabsf(x);
    if (!(ax < 1.0e7f)) return x - x;
    int sign = 1;
    int j;
    float r = rt_trig_reduce(ax, &j);
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    float z = r * r;
    float y = (j == 1 || j == 2) ? rt_sin_poly(r, z) : rt_cos_poly(z);
    return (sign < 0) ? -y : y;
}

/* sin and cos of one argument with one shared reduction: bit-identical to rt_sinf(x)
   and rt_cosf(x) (the same operations, evaluated once). */
RT_HD void rt_sincosf(float x, float *s, float *c)
{
    float ax = rt_fabsf(x);
    if (!(ax < 1.0e7f)) {
        *s = x - x;
        *c = x - x;
        return;
    }
    int j;
    float r = rt_trig_reduce(ax, &j);
    int ssign = (x < 0.0f) ? -1 : 1, csign = 1;
    if (j > 3) {
        ssign = -ssign;
        csign = -csign;
        j -= 4;
    }
    if (j > 1) csign = -csign;
    float z = r * r;
    const float sp = rt_sin_poly(r, z), cp = rt_cos_poly(z);
    const int swap = (j == 1 || j == 2);
    const float sy = swap ? cp : sp, cy = swap ? sp : cp;
    *s = (ssign < 0) ? -sy : sy;
    *c = (csign < 0) ? -cy : cy;
}

/* ---- exp (Cephes expf.c structure) -------------------------------------- */
RT_HD float rt_expf(float x)
{
    if (rt_isnanf(x)) return x;
    if (x > 88.72283905206835f) return rt_inff();
    if (x < -103.278929903431851103f) return 0.0f;
    float z = __builtin_floorf(1.44269504088896341f * x + 0.5f);
    float r = x - z * 0.693359375f;
    r = r - z * -2.12194440e-4f;
    int n = (int)z;
    float zz = r * r;
    float p = 1.9875691500e-4f * r;
    p = p + 1.3981999507e-3f;
    p = p * r;
    p = p + 8.3334519073e-3f;
    p = p * r;
    p = p + 4.1665795894e-2f;
    p = p * r;
    p = p + 1.6666665459e-1f;
    p = p * r;
    p = p + 5.0000001201e-1f;
    p = p * zz;
    p = p + r;
    p = p + 1.0f;
    return rt_ldexpf(p, n);
}

/* ---- log (Cephes logf.c structure) -------------------------------------- */
RT_HD float rt_logf(float x)
{
    if (rt_isnanf(x)) return x;
    if (x < 0.0f) return rt_nanf();
    if (x == 0.0f) return -rt_inff();
    if (x == rt_inff()) return x;
    int e = 0;
    uint32_t u = rt_f2u(x);
    if (u < 0x00800000u) { /* subnormal: scale into the normal range, exactly */
        x = x * 33554432.0f; /* 2^25 */
        u = rt_f2u(x);
        e = -25;
    }
    e += (int)((u >> 23) & 0xff) - 126;              /* x = m * 2^e, m in [0.5, 1) */
    float m = rt_u2f((u & 0x007fffffu) | 0x3f000000u);
    if (m < 0.707106781186547524f) {
        e -= 1;
        m = m + m;
        m = m - 1.0f;
    } else {
        m = m - 1.0f;
    }
    float z = m * m;
    float y = 7.0376836292e-2f * m;
    y = y - 1.1514610310e-1f;
    y = y * m;
    y = y + 1.1676998740e-1f;
    y = y * m;
    y = y - 1.2420140846e-1f;
    y = y * m;
    y = y + 1.4249322787e-1f;
    y = y * m;
    y = y - 1.6668057665e-1f;
    y = y * m;
    y = y + 2.0000714765e-1f;
    y = y * m;
    y = y - 2.4999993993e-1f;
    y = y * m;
    y = y + 3.3333331174e-1f;
    y = y * m;
    y = y * z;
    float fe = (float)e;
    if (e) y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    if (e) r = r + 0.693359375f * fe;
    return r;
}

/* ---- pow: exp(y*log(x)) in binary64, one final rounding ----------------- */
RT_HD double rt_log_d(double x) /* x > 0, finite, normal */
{
    uint64_t u = rt_d2u(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    double m = rt_u2d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1,2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
    double p = 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    p = p * s2;
    double lm = (s + s) + (s + s) * p;
    double de = (double)e;
    return de * 6.93147180369123816490e-01 + (de * 1.90821492927058770002e-10 + lm);
}

RT_HD double rt_exp_d(double x) /* -110 <= x <= 89 */
{
    double k = __builtin_floor(x * 1.44269504088896338700 + 0.5);
    double r = x - k * 6.93147180369123816490e-01;
    r = r - k * 1.90821492927058770002e-10;
    double p = 1.0 / 479001600.0; /* 1/12! */
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    int n = (int)k;
    return p * rt_u2d((uint64_t)(n + 1023) << 52);
}

RT_HD float rt_powf(float x, float y)
{
    if (y == 0.0f) return 1.0f;
    if (x == 1.0f) return 1.0f;
    if (rt_isnanf(x) || rt_isnanf(y)) return rt_nanf();
    float sign = 1.0f;
    if (x < 0.0f) {
        /* negative base: defined only for integral y */
        if (__builtin_floorf(y) != y) return rt_nanf();
        float half = y * 0.5f;
        if (rt_fabsf(y) < 16777216.0f && __builtin_floorf(half) != half) sign = -1.0f;
        x = -x;
    }
    if (x == 0.0f) return (y > 0.0f) ? 0.0f * sign : rt_inff() * sign;
    if (x == rt_inff()) return (y > 0.0f) ? rt_inff() * sign : 0.0f * sign;
    if (y == rt_inff()) return (x > 1.0f) ? rt_inff() : 0.0f;
    if (y == -rt_inff()) return (x > 1.0f) ? 0.0f : rt_inff();
    double lx = rt_log_d((double)x); /* binary64 covers binary32 subnormals as normals */
    double t = (double)y * lx;
    /* e^89 > FLT_MAX; e^-110 < half the smallest subnormal: both ends round
       to inf / 0 in binary32, and keep rt_exp_d's 2^n scale a normal double. */
    if (t > 89.0) return rt_inff() * sign;
    if (t < -110.0) return 0.0f * sign;
    return (float)rt_exp_d(t) * sign;
}

#endif /* RT_MATH_H */
