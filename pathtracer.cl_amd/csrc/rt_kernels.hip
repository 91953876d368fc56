/*
 * rt_kernels.hip — gfx950 kernels of the MI355X path tracer.
 *
 *   k_spheres<SS>      raytrace / raytrace_ss   (clrt/ocl/raytracer.cl:46-104, :120-166)
 *   k_tris<LIN, CNT>   raytrace_tris            (clrt/ocl/raytracer.cl:184-243)
 *   k_trace_rays       closest / any-hit queries (rtcommon.h:39-68), parity tests
 *
 * k_tris is a persistent wavefront state machine: every loop iteration each
 * live lane performs exactly ONE ray query (a path segment's closest hit or one
 * shadow ray) through a shared traversal loop, then advances its path.  Lanes
 * whose pixel finished are refilled from a global pixel queue with one
 * ballot + popcount + atomicAdd per wave (prefix-rank assignment), so SIMD
 * lanes stay busy until the queue drains.  The traversal stack lives in LDS
 * ([depth][lane] stride 256: conflict-free), BVH nodes and triangles are
 * 16-B-aligned float4 records read with dwordx4 loads.  See DESIGN.md.
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "rt_device.h"
#include "rt_internal.h"
#include "rt_quant.h"

#pragma clang fp contract(off)

#ifndef RT_DIAG_RAYSPLIT
#define RT_DIAG_RAYSPLIT 0 /* diagnostics build: counting launches sum the stepping loop's steps of shadow rays
                              from mesh hits / shadow rays from the box / camera rays into counters 10 / 11 / 12 */
#endif
#ifndef RT_DIAG_MIX
#define RT_DIAG_MIX 0 /* diagnostics build (profiles/step_mix.py): counting launches report the stepping
                         rounds' wave-step mix in the per-pixel-maximum counters */
#endif

namespace {

constexpr float kInf = __builtin_huge_valf();

/* ------------------------------------------------------------------------ */
/* Ray/triangle test (geometryFuncs.h:160-245): barycentric part shared by the
   closest-hit and any-hit forms.  Returns false on rejection, else t.        */
__device__ __forceinline__ bool mt_test(V3 o, V3 d, const float4 &a, const float4 &b, const float4 &c, float &t)
{
    const V3 v0 = v3(a.x, a.y, a.z);
    const V3 e1 = v3(b.x, b.y, b.z);
    const V3 e2 = v3(c.x, c.y, c.z);
    const V3 p = cross3(d, e2);
    const float det = dot3(p, e1);
    /* Evaluated without early exits so that the vertex fetch is not sunk below the
       determinant test; the accepted path computes exactly the reference's values. */
    const float inv = 1.0f / det;
    const V3 to = v3(o.x - v0.x, o.y - v0.y, o.z - v0.z);
    const V3 q = cross3(to, e1);
    const float u = dot3(p, to) * inv;
    const float v = dot3(q, d) * inv;
    t = dot3(q, e2) * inv;
    return !(rt_fabsf(det) < RT_SMALL_F) && !(u < 0 || u > 1) && !(v < 0 || v + u > 1);
}

/* Conservative slab test against one child box (culling only: no parity
   constraint, explicit FMAs allowed). */
__device__ __forceinline__ float slab(float lo_x, float hi_x, float lo_y, float hi_y, float lo_z, float hi_z, V3 inv,
                                      V3 oi, float tmin_c, float tmax_c, bool &hit)
{
    const float x0 = __builtin_fmaf(lo_x, inv.x, -oi.x);
    const float x1 = __builtin_fmaf(hi_x, inv.x, -oi.x);
    const float y0 = __builtin_fmaf(lo_y, inv.y, -oi.y);
    const float y1 = __builtin_fmaf(hi_y, inv.y, -oi.y);
    const float z0 = __builtin_fmaf(lo_z, inv.z, -oi.z);
    const float z1 = __builtin_fmaf(hi_z, inv.z, -oi.z);
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x0, x1), __builtin_fminf(y0, y1)),
                                     __builtin_fmaxf(__builtin_fminf(z0, z1), tmin_c));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x0, x1), __builtin_fmaxf(y0, y1)),
                                     __builtin_fminf(__builtin_fmaxf(z0, z1), tmax_c));
    hit = tn <= tf;
    return tn;
}

__device__ __forceinline__ float safe_rcp(float d)
{
    const float e = 1e-18f;
    const float dd = (rt_fabsf(d) > e) ? d : (d < 0.0f ? -e : e);
    return __builtin_amdgcn_rcpf(dd);
}

/* Culling margin on the t interval: covers the rounding of the reference's
   intersection t relative to the box slabs (boxes are padded as well). */
__device__ __forceinline__ float t_slack(float t) { return t * 1.0009765625f + 1e-4f; }

struct TravCounts {
    uint32_t nodes;
    uint32_t tests;
    uint32_t leaves;
};

/* Leaf of the full-precision traversals (trav_step, traverse): the reference's triangle tests on
   slots [first, first+count), in order, ending at an any-hit query's first occluder. */
template <bool COUNT>
__device__ __forceinline__ bool leaf_accept(int s, float4 a, V3 d, bool ok, float t, float tmin, float tmax,
                                            bool any_hit, int &best, int &best_orig, float &best_t, bool &done)
{
    if (!ok) return false;
    if (any_hit) {
        if (t < tmax && t > tmin) {
            best = s;
            done = true;
        }
    } else {
        const int orig = __float_as_int(a.w);
        if (!(t < tmin) && (t < best_t || (t == best_t && orig > best_orig))) {
            best = s;
            best_orig = orig;
            best_t = t;
            return true;
        }
    }
    return false;
}

template <bool COUNT>
__device__ __forceinline__ bool leaf_tests(const float4 *__restrict__ tris, int first, int count, V3 o, V3 d,
                                           float tmin, float tmax, bool any_hit, int &best, int &best_orig,
                                           float &best_t, TravCounts &cnt)
{
    bool done = false;
    for (int k = 0; k < count; ++k) {
        const int s0 = first + k;
        const float4 a0 = tris[3 * s0], b0 = tris[3 * s0 + 1], c0 = tris[3 * s0 + 2];
        if (COUNT) cnt.tests++;
        float t0 = 0.0f;
        const bool h0 = mt_test(o, d, a0, b0, c0, t0);
        leaf_accept<COUNT>(s0, a0, d, h0, t0, tmin, tmax, any_hit, best, best_orig, best_t, done);
        if (done) return true;
    }
    return false;
}

/* Per-lane traversal stack: [depth][lane] in LDS (stride RT_BLOCK dwords, bank
   conflict free) with an overflow tail in global memory for the rare rays of a
   4-wide tree whose worst-case stack exceeds RT_STACK_DEPTH.  The two parts are
   typed by address space, so that a pop that may come from either stays a
   ds_read plus a global load under lane masks — never a generic (flat) load, which
   would occupy the vector-memory address path for every LDS pop. */
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) int lds_int;
typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(1))) int32_t glob_int;
#else
typedef int lds_int;
typedef float lds_float;
typedef int32_t glob_int;
#endif

struct Stack {
    lds_int *lds;
    glob_int *spill_block; /* the block's spill area (uniform): lane l owns [l * cap, (l + 1) * cap) */
    uint32_t cap;
    int sp;
    __device__ __forceinline__ glob_int *spill_slot(int i) const
    {
        return spill_block + threadIdx.x * cap + (uint32_t)(i - RT_STACK_DEPTH);
    }
    __device__ __forceinline__ void push(int v)
    {
        if (sp < RT_STACK_DEPTH) lds[sp * RT_BLOCK] = v;
        else *spill_slot(sp) = v;
        ++sp;
    }
    __device__ __forceinline__ int pop()
    {
        --sp;
        int v;
        if (sp < RT_STACK_DEPTH) v = lds[sp * RT_BLOCK];
        else v = *spill_slot(sp);
        return v;
    }
    __device__ __forceinline__ void init(int *lds_base, int32_t *spill_base, uint32_t spill_cap)
    {
        lds = (lds_int *)(lds_base + threadIdx.x);
        spill_block = (glob_int *)(spill_base + (size_t)blockIdx.x * RT_BLOCK * spill_cap);
        cap = spill_cap;
        sp = 0;
    }
};

__device__ __forceinline__ void cas(float &ta, int &ca, float &tb, int &cb)
{
    const bool sw = tb < ta;
    const float t = sw ? tb : ta;
    const int c = sw ? cb : ca;
    tb = sw ? ta : tb;
    cb = sw ? ca : cb;
    ta = t;
    ca = c;
}

/* Resumable per-lane traversal of the binary or 4-wide tree: the whole query
   state is this struct plus the lane's stack, so a query can be advanced one
   node (or one leaf) at a time and suspended between steps. */
struct TravState {
    int node;      /* next node to visit (>= 0 inner, < 0 leaf) */
    int best;      /* leaf-order slot of the current closest / occluding hit, -1 none */
    int best_orig; /* its original triangle index (tie rule) */
    float best_t;  /* closest hit so far (= tmax of an any-hit query) */
    V3 inv, oi;    /* 1/d and o/d for the slab tests */
};

__device__ __forceinline__ void trav_begin(TravState &s, Stack &stk, V3 o, V3 d, float tmax)
{
    s.inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    s.oi = v3(o.x * s.inv.x, o.y * s.inv.y, o.z * s.inv.z);
    s.node = 0;
    s.best = -1;
    s.best_orig = -1;
    s.best_t = tmax;
    stk.sp = 0;
}

/* Half `hi` of a word of two f16 values, widened to f32 (exact; folds into the
   op_sel of v_fma_mix_f32). */
__device__ __forceinline__ float half_of(uint32_t w, int hi)
{
    const uint16_t b = (uint16_t)(hi ? (w >> 16) : (w & 0xffffu));
    return (float)__builtin_bit_cast(_Float16, b);
}

/* The 4 child boxes of a compressed node (rt_quant.h; the record as its four dwordx4 words)
   against the ray: c[] the children by their sort key t[] ascending (misses last, kInf); returns
   how many were hit (0 also when the determinant cull skips the subtree).  Culling only. */
__device__ __forceinline__ int node_children(uint4 q0, uint4 q1, uint4 q2, uint4 q3, V3 inv, V3 oi, V3 d,
                                         float best_t, bool any_hit, bool longest, float (&t)[4], int (&c)[4])
{
    const float tmin_c = -1e-3f;
    const float tmax_c = t_slack(best_t);
    const uint32_t w = q0.w;
    constexpr int kExpBias = RT_QEXP_MIN + 24; /* scales carry the 2^24 of the f16-subnormal planes */
    const float sx = __builtin_amdgcn_ldexpf(inv.x, (int)(w & 31u) + kExpBias);
    const float sy = __builtin_amdgcn_ldexpf(inv.y, (int)((w >> 5) & 31u) + kExpBias);
    const float sz = __builtin_amdgcn_ldexpf(inv.z, (int)((w >> 10) & 31u) + kExpBias);
    const float bx = __builtin_fmaf(__uint_as_float(q0.x), inv.x, -oi.x);
    const float by = __builtin_fmaf(__uint_as_float(q0.y), inv.y, -oi.y);
    const float bzo = __builtin_fmaf(__uint_as_float(q0.z), inv.z, -oi.z);
    const bool px = inv.x >= 0.0f, py = inv.y >= 0.0f, pz = inv.z >= 0.0f;
    const uint32_t nxw = px ? q1.x : q1.y, fxw = px ? q1.y : q1.x;
    const uint32_t nyw = py ? q1.z : q1.w, fyw = py ? q1.w : q1.z;
    const uint32_t nzw = pz ? q2.x : q2.y, fzw = pz ? q2.y : q2.x;
    int nhit = 0;
    /* the any-hit order's per-query terms (below): -1 selects the longest-segment key, and the
       penalty that sends boxes holding the ray origin last */
    const float lsel = longest ? -1.0f : 0.0f, pen = any_hit ? 1e4f : 0.0f;
    /* Plane bytes as f16 subnormals: v_perm_b32 spreads two bytes of a plane word into
       the low bytes of two 16-bit halves (0x00bb = b * 2^-24 as f16, exact), and
       v_fma_mix_f32 converts a half and does the FMA in one instruction, with the
       2^24 folded into the scale's exponent: (b * 2^-24) * (s * 2^24) + base is exactly
       fma(b, s, base) — the same bits as a byte convert + FMA, in 3/4 of the VALU. */
    const float sx24 = sx, sy24 = sy, sz24 = sz;
    const uint32_t nx01 = __builtin_amdgcn_perm(0u, nxw, 0x0c010c00u), nx23 = __builtin_amdgcn_perm(0u, nxw, 0x0c030c02u);
    const uint32_t ny01 = __builtin_amdgcn_perm(0u, nyw, 0x0c010c00u), ny23 = __builtin_amdgcn_perm(0u, nyw, 0x0c030c02u);
    const uint32_t nz01 = __builtin_amdgcn_perm(0u, nzw, 0x0c010c00u), nz23 = __builtin_amdgcn_perm(0u, nzw, 0x0c030c02u);
    const uint32_t fx01 = __builtin_amdgcn_perm(0u, fxw, 0x0c010c00u), fx23 = __builtin_amdgcn_perm(0u, fxw, 0x0c030c02u);
    const uint32_t fy01 = __builtin_amdgcn_perm(0u, fyw, 0x0c010c00u), fy23 = __builtin_amdgcn_perm(0u, fyw, 0x0c030c02u);
    const uint32_t fz01 = __builtin_amdgcn_perm(0u, fzw, 0x0c010c00u), fz23 = __builtin_amdgcn_perm(0u, fzw, 0x0c030c02u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float tn = __builtin_fmaxf(
            __builtin_fmaxf(__builtin_fmaf(half_of(i < 2 ? nx01 : nx23, i & 1), sx24, bx),
                            __builtin_fmaf(half_of(i < 2 ? ny01 : ny23, i & 1), sy24, by)),
            __builtin_fmaxf(__builtin_fmaf(half_of(i < 2 ? nz01 : nz23, i & 1), sz24, bzo), tmin_c));
        const float tf = __builtin_fminf(
            __builtin_fminf(__builtin_fmaf(half_of(i < 2 ? fx01 : fx23, i & 1), sx24, bx),
                            __builtin_fmaf(half_of(i < 2 ? fy01 : fy23, i & 1), sy24, by)),
            __builtin_fminf(__builtin_fmaf(half_of(i < 2 ? fz01 : fz23, i & 1), sz24, bzo), tmax_c));
        const bool h = tn <= tf; /* an unused slot's inverted box never passes */
        c[i] = (int)(i == 0 ? q3.x : i == 1 ? q3.y : i == 2 ? q3.z : q3.w);
        /* Any hit (the answer is order-free): children whose box holds the ray origin (the
           surface a shadow ray leaves, whose own triangles it cannot hit) are visited
           last, and a ray leaving the mesh (`longest`) takes the others by the length of
           its box segment, longest first — measured on the CPU model to find an occluder
           in the fewest steps; rays from the box walls keep nearest first. */
        const float key = __builtin_fmaf(lsel, tf, tn); /* tn - tf (longest) or tn, exactly */
        t[i] = h ? (tn <= 0.0f ? key + pen : key) : kInf;
        nhit += h ? 1 : 0;
    }
    /* Determinant cull (rt_quant.h): the node's normal box bounds d . N = det over its
       subtree; below 1e-4 (with the float error bound) no triangle can be accepted, so
       the subtree is skipped.  Culling only: the same results, fewer steps. */
    {
        /* v_perm_b32 picks, per axis, the hi byte (d >= 0) or the lo byte into `nb` (the box
           corner maximising d . N) and the other into `fb`; v_cvt_f32_ubyteN converts in
           place; the +128 byte bias folds into one per-ray term */
        const uint32_t nlo = q2.z, nhi = q2.w;
        const float nsc = __builtin_amdgcn_ldexpf(1.0f, (int)(nlo >> 24) - 128);
        const uint32_t sel_n = (px ? 4u : 0u) | (py ? 5u : 1u) << 8 | (pz ? 6u : 2u) << 16;
        const uint32_t sel_f = (px ? 0u : 4u) | (py ? 1u : 5u) << 8 | (pz ? 2u : 6u) << 16;
        const uint32_t nb = __builtin_amdgcn_perm(nhi, nlo, sel_n), fb = __builtin_amdgcn_perm(nhi, nlo, sel_f);
        const float bias = 128.0f * (d.x + d.y + d.z);
        const float fhi = __builtin_fmaf(d.x, (float)(nb & 0xffu),
                                         __builtin_fmaf(d.y, (float)((nb >> 8) & 0xffu),
                                                        __builtin_fmaf(d.z, (float)((nb >> 16) & 0xffu), -bias)));
        const float flo = __builtin_fmaf(d.x, (float)(fb & 0xffu),
                                         __builtin_fmaf(d.y, (float)((fb >> 8) & 0xffu),
                                                        __builtin_fmaf(d.z, (float)((fb >> 16) & 0xffu), -bias)));
        const float l1 = __builtin_fabsf(d.x) + __builtin_fabsf(d.y) + __builtin_fabsf(d.z);
        /* bias rounding: |fl(128 sum d) - 128 sum d| <= 3u * 128 |d|_1, inside the margin */
        const float bound = __builtin_fmaf(__builtin_fmaxf(fhi, -flo) * nsc, 1.02f, 5e-7f * l1);
        if (bound < 1e-4f) nhit = 0;
    }
    if (nhit > 0) {
        cas(t[0], c[0], t[1], c[1]);
        cas(t[2], c[2], t[3], c[3]);
        cas(t[0], c[0], t[2], c[2]);
        cas(t[1], c[1], t[3], c[3]);
        cas(t[1], c[1], t[2], c[2]);
    }
    return nhit;
}

/* One step of the compressed 4-wide traversal (rt_quant.h).  Every lane fetches
   exactly one 64-B record per step — a node, or ONE triangle of its current leaf —
   with the same three dwordx4 loads, so a wave-step costs one memory round trip
   whatever mix of node and leaf lanes it holds (a leaf of k triangles takes k
   steps; the leaf cursor is the leaf code itself: first slot and remaining count). */
template <bool COUNT>
__device__ __forceinline__ bool trav_step_q(const float4 *__restrict__ nodes, const float4 *__restrict__ tris,
                                            TravState &s, Stack &stk, V3 o, V3 d, float tmin, bool any_hit,
                                            TravCounts &cnt, bool longest = false, lds_float *hn_out = nullptr)
{
    const V3 inv = s.inv, oi = s.oi;
    const int node = s.node;
    const bool leaf = node < 0;
    /* wave-uniform: every lane's pushes and pops of this step stay in the LDS part
       of the stack (almost always), so they need no per-lane LDS/spill selection */
    const bool lds_only = !__any(stk.sp + 3 > RT_STACK_DEPTH);
    const uint32_t enc = (uint32_t)(~node);
    const uint4 *rec = leaf ? reinterpret_cast<const uint4 *>(tris) + 3 * (enc >> 3)
                            : reinterpret_cast<const uint4 *>(nodes) + 4 * node;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u *vrec = reinterpret_cast<const v4u *>(rec);
    v4u w0 = vrec[0], w1 = vrec[1], w2 = vrec[2];
    /* the child links (d[12..15]) only for node lanes: the load runs under their exec mask,
       so leaf lanes add no addresses to it (-1 %) */
    v4u w3 = {0u, 0u, 0u, 0u};
    if (!leaf) w3 = vrec[3];
    /* Every lane's record arrives as whole dwordx4 loads issued together: without this
       the compiler narrows loads to the components each branch uses (x4 + x3 + x2 +
       dword) and sinks the child links below the box test, i.e. 5-6 vector-memory
       instructions per step instead of 4 (each costs the address path ~16 cycles per
       wave whatever its width) and a second dependent round trip for node lanes. */
    asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
    const uint4 q0 = make_uint4(w0.x, w0.y, w0.z, w0.w), q1 = make_uint4(w1.x, w1.y, w1.z, w1.w);
    const uint4 q2 = make_uint4(w2.x, w2.y, w2.z, w2.w);
    const uint4 q3 = make_uint4(w3.x, w3.y, w3.z, w3.w);
    if (leaf) {
        if (COUNT) {
            cnt.tests++;
            cnt.leaves++;
        }
        const float4 a = make_float4(__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z),
                                     __uint_as_float(q0.w));
        const float4 b = make_float4(__uint_as_float(q1.x), __uint_as_float(q1.y), __uint_as_float(q1.z), 0.0f);
        const float4 c = make_float4(__uint_as_float(q2.x), __uint_as_float(q2.y), __uint_as_float(q2.z), 0.0f);
        float t = 0.0f;
        const bool h = mt_test(o, d, a, b, c, t);
        const int slot = (int)(enc >> 3);
        if (h) {
            if (any_hit) {
                if (t < s.best_t && t > tmin) {
                    s.best = slot;
                    return true;
                }
            } else if (!(t < tmin)) {
                /* the accept rule t < best_t || (t == best_t && orig > best_orig): the best hit's
                   original index is read back from its record on the rare exact tie instead of
                   being carried in a register (which the compiler spilled on every step) */
                bool acc = t < s.best_t;
                if (!acc && t == s.best_t)
                    acc = s.best < 0 || __float_as_int(a.w) > __float_as_int(tris[3 * s.best].w);
                if (acc) {
                    s.best = slot;
                    s.best_t = t;
                    if (hn_out) { /* the hit's unnormalised normal for the shading (rtcommon.h:389) */
                        const V3 n = cross3(v3(c.x, c.y, c.z), v3(b.x, b.y, b.z));
                        hn_out[0] = n.x;
                        hn_out[RT_BLOCK] = n.y;
                        hn_out[2 * RT_BLOCK] = n.z;
                    }
                }
            }
        }
        /* a camera candidate list (k_pixel_lists) is sorted, r1.w = the next candidate's
           earliest accept t: past the best hit, nothing later can be accepted (tree leaves: 0) */
        if (!any_hit && s.best_t < __uint_as_float(q1.w)) return true;
        if (enc & 7u) { /* next triangle of this leaf */
            s.node = ~(int)((((enc >> 3) + 1u) << 3) | ((enc & 7u) - 1u));
            return false;
        }
    } else {
        if (COUNT) cnt.nodes++;
        float t[4];
        int c[4];
        const int nhit = node_children(q0, q1, q2, q3, inv, oi, d, s.best_t, any_hit, longest, t, c);
        if (nhit > 0) {
            if (lds_only) {
                /* the nhit - 1 farther hits, farthest first, written unconditionally at
                   sp, sp+1, sp+2 (slots above the new top hold junk) */
                const int v0 = nhit >= 4 ? c[3] : (nhit == 3 ? c[2] : c[1]);
                const int v1 = nhit >= 4 ? c[2] : c[1];
                lds_int *top = stk.lds + stk.sp * RT_BLOCK;
                top[0] = v0;
                top[RT_BLOCK] = v1;
                top[2 * RT_BLOCK] = c[1];
                stk.sp += nhit - 1;
            } else {
                if (nhit >= 4) stk.push(c[3]);
                if (nhit >= 3) stk.push(c[2]);
                if (nhit >= 2) stk.push(c[1]);
            }
            s.node = c[0];
            return false;
        }
    }
    if (stk.sp == 0) return true;
    if (lds_only) s.node = stk.lds[--stk.sp * RT_BLOCK];
    else s.node = stk.pop();
    return false;
}


/* One traversal step; returns true when the query is complete.  Closest hit:
   the result equals the reference's linear loop (minimum t, ties to the highest
   original index — rtcommon.h:39-52 with intersects_triangle's `t > tmax`
   rejection).  Any hit: best >= 0 iff some triangle has tmin < t < tmax
   (rtcommon.h:59-68). */
template <int TRAV, bool COUNT>
__device__ __forceinline__ bool trav_step(const float4 *__restrict__ nodes, const float4 *__restrict__ tris,
                                          TravState &s, Stack &stk, V3 o, V3 d, float tmin, bool any_hit,
                                          TravCounts &cnt, bool longest = false, lds_float *hn_out = nullptr)
{
    if (TRAV == RT_TRAV_BVH4Q)
        return trav_step_q<COUNT>(nodes, tris, s, stk, o, d, tmin, any_hit, cnt, longest, hn_out);
    const float tmin_c = -1e-3f;
    const V3 inv = s.inv, oi = s.oi;
    int node = s.node;
    if (node >= 0) {
        if (COUNT) cnt.nodes++;
        const float tmax_c = t_slack(s.best_t);
        {
            /* 4-wide: near/far slab planes picked by the direction signs, so each
               child costs 6 FMAs + max3/min3 and no min/max pairs. */
            const int nxo = inv.x >= 0.0f ? 0 : 1, nyo = inv.y >= 0.0f ? 2 : 3, nzo = inv.z >= 0.0f ? 4 : 5;
            const int fxo = 1 - nxo, fyo = 5 - nyo, fzo = 9 - nzo;
            const float4 *nd = nodes + 8 * node;
            const float4 nx = nd[nxo], fx = nd[fxo], ny = nd[nyo], fy = nd[fyo], nz = nd[nzo], fz = nd[fzo];
            const float4 cc = nd[6];
            float t[4];
            int c[4];
            const float nxs[4] = {nx.x, nx.y, nx.z, nx.w}, fxs[4] = {fx.x, fx.y, fx.z, fx.w};
            const float nys[4] = {ny.x, ny.y, ny.z, ny.w}, fys[4] = {fy.x, fy.y, fy.z, fy.w};
            const float nzs[4] = {nz.x, nz.y, nz.z, nz.w}, fzs[4] = {fz.x, fz.y, fz.z, fz.w};
            const int cs[4] = {__float_as_int(cc.x), __float_as_int(cc.y), __float_as_int(cc.z),
                               __float_as_int(cc.w)};
            int nhit = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float tn = __builtin_fmaxf(
                    __builtin_fmaxf(__builtin_fmaf(nxs[i], inv.x, -oi.x), __builtin_fmaf(nys[i], inv.y, -oi.y)),
                    __builtin_fmaxf(__builtin_fmaf(nzs[i], inv.z, -oi.z), tmin_c));
                const float tf = __builtin_fminf(
                    __builtin_fminf(__builtin_fmaf(fxs[i], inv.x, -oi.x), __builtin_fmaf(fys[i], inv.y, -oi.y)),
                    __builtin_fminf(__builtin_fmaf(fzs[i], inv.z, -oi.z), tmax_c));
                const bool h = (tn <= tf) && (cs[i] != RT_EMPTY_CHILD);
                t[i] = h ? tn : kInf;
                c[i] = cs[i];
                nhit += h ? 1 : 0;
            }
            if (nhit > 0) {
                /* sort the (entry distance, child) pairs: misses (inf) sink to the end */
                cas(t[0], c[0], t[1], c[1]);
                cas(t[2], c[2], t[3], c[3]);
                cas(t[0], c[0], t[2], c[2]);
                cas(t[1], c[1], t[3], c[3]);
                cas(t[1], c[1], t[2], c[2]);
                if (nhit >= 4) stk.push(c[3]);
                if (nhit >= 3) stk.push(c[2]);
                if (nhit >= 2) stk.push(c[1]);
                s.node = c[0];
                return false;
            }
        }
    } else {
        const int enc = ~node;
        if (COUNT) cnt.leaves++;
        if (leaf_tests<COUNT>(tris, enc >> 3, (enc & 7) + 1, o, d, tmin, s.best_t, any_hit, s.best, s.best_orig,
                              s.best_t, cnt))
            return true;
    }
    if (stk.sp == 0) return true;
    s.node = stk.pop();
    return false;
}

/* One ray query.  Closest hit (any_hit = false): returns the leaf-order slot of
   the hit (or -1) with t in tmax; the result equals the reference's linear
   loop: minimum t, ties to the highest original index (rtcommon.h:39-52 with
   intersects_triangle's `t > tmax` rejection).  Any hit: returns >= 0 iff some
   triangle has tmin < t < tmax (rtcommon.h:59-68). */
template <int TRAV, bool COUNT>
__device__ __forceinline__ int traverse(const float4 *__restrict__ nodes, const float4 *__restrict__ tris,
                                        uint32_t n_tris, V3 o, V3 d, float tmin, float &tmax, bool any_hit,
                                        Stack &stk, TravCounts &cnt)
{
    int best = -1;
    int best_orig = -1;
    float best_t = tmax;
    if (TRAV == RT_TRAV_LINEAR) {
        /* The reference algorithm: every triangle, in a wave-uniform loop (the
           slot index is uniform, so the records come in through scalar loads). */
        bool live = true;
        for (uint32_t s = 0; s < n_tris; ++s) {
            if (live) {
                const float4 a = tris[3 * s], b = tris[3 * s + 1], c = tris[3 * s + 2];
                float t;
                if (COUNT) cnt.tests++;
                if (mt_test(o, d, a, b, c, t)) {
                    if (any_hit) {
                        if (t < tmax && t > tmin) {
                            best = (int)s;
                            live = false;
                        }
                    } else {
                        const int orig = __float_as_int(a.w);
                        if (!(t < tmin) && (t < best_t || (t == best_t && orig > best_orig))) {
                            best = (int)s;
                            best_orig = orig;
                            best_t = t;
                        }
                    }
                }
            }
            if (!__any(live)) break;
        }
        if (!any_hit) tmax = best_t;
        return best;
    }

    TravState st;
    trav_begin(st, stk, o, d, tmax);
    while (!trav_step<TRAV, COUNT>(nodes, tris, st, stk, o, d, tmin, any_hit, cnt)) {
    }
    if (!any_hit) tmax = st.best_t;
    return st.best;
}

/* a launch-uniform float held in an SGPR */
__device__ __forceinline__ float uniform_f(float v)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

/* Queue items for a wave's idle lanes (ranked by a prefix popcount of the idle ballot) from a
   wave-private batch of kBatch consecutive items: one atomicAdd per batch instead of one per
   refill.  A single head word saturates at about 88 dequeues per microsecond
   (MI355X_MICROARCH.md, dequeue), which the many short tasks of a sample-split launch exceed.
   Wave-uniform: call with every lane active; bnext / bend start equal; batch >= the takers
   per wave (k <= batch).  batch 0: exactly the items the idle lanes need, none held back — for
   queues of long tasks (many-sample whole pixels), where a batch held by a wave whose lanes are
   busy starts its last items late: the dragon frame's last tile started ~9 ms after the queue
   ran dry (profiles/r05r), and at ~20 dequeues per microsecond one atomic per refill is cheap. */
constexpr uint32_t kBatch = 64;

__device__ __forceinline__ uint32_t batch_take(uint32_t *counter, unsigned long long idle, uint32_t &bnext,
                                               uint32_t &bend, uint32_t batch = kBatch)
{
    const uint32_t k = (uint32_t)__popcll(idle);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
    const uint32_t avail = bend - bnext;
    const uint32_t from_b = k < avail ? k : avail;
    uint32_t nb = 0;
    const uint32_t take = batch ? batch : k - from_b;
    if (k > from_b) {
        const int leader = __ffsll((long long)idle) - 1;
        if ((int)(threadIdx.x & 63) == leader) nb = atomicAdd(counter, take);
        nb = __builtin_amdgcn_readfirstlane(__shfl(nb, leader));
    }
    const uint32_t item = rank < from_b ? bnext + rank : nb + (rank - from_b);
    if (k > from_b) {
        bnext = nb + (k - from_b);
        bend = nb + take;
    } else {
        bnext += k;
    }
    return item;
}

/* Multi-head queue (RT_QHEADS heads, RT_QSTRIDE words apart): a launch's items are 64-item groups
   (an 8 x 8 tile, or one chunk layer of a tile); head h owns the groups g = h, h + RT_QHEADS, ...
   (in queue order), and a wave takes `batch` items of a head at a time, starting at the head of
   its block (blockIdx.x mod RT_QHEADS) and moving on to the next head when one is drained.  More
   heads take more dequeues per microsecond than one (a single head word saturates near 88), so
   the batches can be small enough that no wave holds back many of the queue's last items while
   its lanes are busy.  The wave's state is one word `qs`: the head of its batch [bnext, bend)
   (local indices, bits 0-3), the head it takes from next (bits 4-7), and how many heads in a row
   it found drained (bits 8-11: RT_QHEADS of them, the queue is empty).  At most one atomic per
   take; a lane whose take found a drained head stays idle and takes again in the next iteration.
   Returns the lane's item or ~0u.  Wave-uniform, like batch_take. */
__device__ __forceinline__ uint32_t mq_take(uint32_t *heads, uint32_t n_tasks, unsigned long long idle, uint32_t &bnext,
                                            uint32_t &bend, uint32_t &qs, uint32_t batch, uint32_t span = 64u)
{
    constexpr uint32_t Q = RT_QHEADS;
    const uint32_t k = (uint32_t)__popcll(idle);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
    const uint32_t avail = bend - bnext;
    const uint32_t from_b = k < avail ? k : avail;
    const uint32_t bq = qs & 15u, hq = (qs >> 4) & 15u;
    /* local index l of head q -> queue item: span-item group (l / span) x Q + q, offset l mod span (span
       64: a tile; a split launch's 64 x chunks: a tile's chunk layers together) */
    auto global = [&](uint32_t l, uint32_t q) { return ((l / span) * Q + q) * span + l % span; };
    uint32_t item = rank < from_b ? global(bnext + rank, bq) : ~0u;
    bnext += from_b;
    if (k > from_b && (qs >> 8) < Q) {
        const int leader = __ffsll((long long)idle) - 1;
        uint32_t nb = 0;
        const uint32_t take = batch ? batch : k - from_b; /* batch 0: exactly the items needed */
        if ((int)(threadIdx.x & 63) == leader) nb = atomicAdd(heads + RT_QSTRIDE * hq, take);
        nb = __builtin_amdgcn_readfirstlane(__shfl(nb, leader));
        const uint32_t n_groups = n_tasks / span;
        const uint32_t n_local = (n_groups > hq ? (n_groups - hq + Q - 1u) / Q : 0u) * span;
        if (nb < n_local) {
            const uint32_t r = rank - from_b;
            bend = nb + take < n_local ? nb + take : n_local;
            if (rank >= from_b && nb + r < bend) item = global(nb + r, hq);
            const uint32_t need = k - from_b;
            bnext = nb + (need < bend - nb ? need : bend - nb);
            qs = hq | hq << 4; /* the batch's head, the same head next, no drained heads */
        } else { /* drained: the next head, one more drained in a row */
            qs = (qs & 15u) | ((hq + 1u) % Q) << 4 | ((qs >> 8) + 1u) << 8;
        }
    }
    return item;
}

/* RT_SPLIT_BOX launches: the number of items of split_box[split_item_base ...] this launch takes
   (the list's length from the device when split_n_dev is set), at most split_item_cap */
__device__ __forceinline__ uint32_t box_items(const RtTriLaunch &a)
{
    const uint32_t n = a.split_n_dev ? *a.split_n_dev : a.split_n_box;
    const uint32_t m = n > a.split_item_base ? n - a.split_item_base : 0u;
    return a.split_item_cap && m > a.split_item_cap ? a.split_item_cap : m;
}

/* shader-clock timestamp (s_memtime), counting launches only */
__device__ __forceinline__ unsigned long long wave_clock()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ void flush_counters(unsigned long long *dst, const unsigned long long (&v)[RT_N_COUNTERS],
                                               bool with_trav)
{
    for (int i = 0; i < RT_N_SUM_COUNTERS; ++i) {
        if (!with_trav && i >= 2 && i != RT_CNT_SKIPPED) continue;
        const unsigned long long w = wave_sum(v[i]);
        if ((threadIdx.x & 63) == 0) atomicAdd(&dst[i], w);
    }
    if (with_trav) /* per-pixel maxima (RT_DIAG_MIX builds: the wave-step mix, summed) */
        for (int i = RT_N_SUM_COUNTERS; i < RT_N_COUNTERS; ++i) {
            if (RT_DIAG_MIX || RT_DIAG_RAYSPLIT) atomicAdd(&dst[i], v[i]);
            else atomicMax(&dst[i], v[i]);
        }
}

/* raytracer.cl:81-85: normalize(view + right*a + up*b), float4 lanes incl. w,
   normalize pinned as v / sqrt(dot(v, v)). */
__device__ __forceinline__ V3 camera_dir(const rt_camera &cam, float a, float b)
{
    const float x = (cam.view.x + cam.right.x * a) + cam.up.x * b;
    const float y = (cam.view.y + cam.right.y * a) + cam.up.y * b;
    const float z = (cam.view.z + cam.right.z * a) + cam.up.z * b;
    const float w = (cam.view.w + cam.right.w * a) + cam.up.w * b;
    const float len = rt_sqrtf(((x * x + y * y) + z * z) + w * w);
    return v3(x / len, y / len, z / len);
}

/* The frame row of a tile's row yl: the interleaved partition's formula, or the owner map's stripe
   list (rt_tile.stripe_owner; only a frame's last stripe can be short, and it is its owner's last) */
template <class L>
__device__ __forceinline__ uint32_t global_row(const L &a, uint32_t yl)
{
    if (a.stripe_map) return a.stripe_map[yl / a.stripe] * a.stripe + yl % a.stripe;
    if (a.n_ranks <= 1) return yl;
    return ((yl / a.stripe) * a.n_ranks + a.rank) * a.stripe + (yl % a.stripe);
}

/* A pixel's camera-ray candidate list (k_pixel_lists) packed in one word, read when the lane takes
   the pixel instead of before every sample's camera query (one dependent load less per sample):
   (first slot / 8) << RT_LIST_BITS | (count - 1) — lists start on 8-record multiples and slots stay
   below 2^28 (rt_host.cpp list_cap), so the word stays below RT_LPACK_EMPTY. */
constexpr uint32_t RT_LPACK_NONE = 0xffffffffu, RT_LPACK_EMPTY = 0xfffffffeu;
__device__ __forceinline__ uint32_t list_pack(const RtTriLaunch &a, uint32_t x, uint32_t yl, uint32_t tiles_x)
{
    if (!a.list_code) return RT_LPACK_NONE;
    const uint32_t code = a.list_code[yl * a.W + x];
    const uint32_t block = a.list_tile[(yl >> 3) * tiles_x + (x >> 3)];
    if (code == RT_LIST_NONE) return RT_LPACK_NONE;
    if (code == RT_LIST_EMPTY) return RT_LPACK_EMPTY;
    const uint32_t first = block + ((code >> RT_LIST_BITS) << 3);
    return ((first >> 3) << RT_LIST_BITS) | (code & (RT_LIST_MAX - 1u));
}

#ifndef RT_DIAG_SKIP
#define RT_DIAG_SKIP 0 /* diagnostics builds: k_tris skips the box pixels (1) or the mesh pixels (2) */
#endif

#ifndef RT_SEED_UNROLL
#define RT_SEED_UNROLL 4 /* seed-pass traversal steps per loop iteration */
#endif

/* Cooperative queries of the long chains' seed pass (coop_round below): the 4 lanes of a group
   (lanes 4g..4g+3 of a wave) advance ONE query together, its stack in LDS (RT_COOP_STACK entries
   per group).  Quad (4-lane group) exchanges through DPP quad_perm: a VALU modifier, not an LDS round trip
   like ds_bpermute (__shfl), whose latency a lone chain's wave cannot hide */
template <int CTRL>
__device__ __forceinline__ int quad_dpp(int v)
{
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int M> /* the value of lane sub ^ M */
__device__ __forceinline__ int quad_xor(int v)
{
    return M == 1 ? quad_dpp<0xB1>(v) : M == 2 ? quad_dpp<0x4E>(v) : quad_dpp<0x1B>(v);
}
__device__ __forceinline__ float quad_xorf1(float v) { return __int_as_float(quad_xor<1>(__float_as_int(v))); }
__device__ __forceinline__ float quad_xorf2(float v) { return __int_as_float(quad_xor<2>(__float_as_int(v))); }
/* the value of quad lane k (k uniform within the quad) */
__device__ __forceinline__ int quad_bcast(int v, int k)
{
    const int b0 = quad_dpp<0x00>(v), b1 = quad_dpp<0x55>(v), b2 = quad_dpp<0xAA>(v), b3 = quad_dpp<0xFF>(v);
    return k == 0 ? b0 : k == 1 ? b1 : k == 2 ? b2 : b3;
}

/* The 4-lane group's stack in the block's LDS stack area, inside the words its wave's lanes own
   in the per-lane layout ([depth][lane], RT_BLOCK words per depth): entry e of group g of wave w
   is word RT_BLOCK * (e / 4) + 64 w + 4 g + e % 4 (2-way bank conflicts between the groups). */
template <int G>
struct CoopStackG {
    static constexpr int kCap = RT_STACK_DEPTH * G; /* entries: the group's words of its wave's columns */
    lds_int *base; /* word 64 w + G g */
    __device__ __forceinline__ lds_int &operator[](int e) const
    {
        e = e < 0 ? 0 : e >= kCap ? kCap - 1 : e; /* never outside the group's words */
        return base[RT_BLOCK * (e / G) + (e % G)];
    }
};
typedef CoopStackG<4> CoopStack;

struct CoopQuery {
    int best, best_orig, sp;
    float best_t;
    V3 inv, oi;
};

__device__ __forceinline__ void coop_begin(CoopQuery &q, V3 o, V3 d, float tmax)
{
    q.inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    q.oi = v3(o.x * q.inv.x, o.y * q.inv.y, o.z * q.inv.z);
    q.best = -1;
    q.best_orig = -1;
    q.best_t = tmax;
    q.sp = 0;
}


/* Cooperative closest-hit query, one stack ITEM per lane: each round the 4 lanes of a group take
   the top entries of the group's stack — a node (one lane: its 4 child boxes) or the triangles of
   a leaf or candidate-list block (one lane each) — so a round tests up to 4 records of different
   subtrees instead of one node's boxes (scripts/sim_group_trav.cpp on box-path queries: 3.2
   rounds per closest-hit query, against 4.9 one-record steps).  The closest hit is order-free
   (minimum t, ties to the highest original index), so taking entries out of depth-first order
   changes only the work; a sorted candidate list's early end takes the bound of the last record
   tested, the latest in list order.  The group's whole query is on its stack (q.sp entries: the
   root, or the list blocks, pushed at the start); the item assignment is computed alike in the
   4 lanes.  Above `multi_sp` entries a round takes ONE item: 4 nodes add at most 12 entries, and
   a one-item depth-first walk from there at most the tree's worst stack (rt_host.cpp), so the
   stack stays inside the group's RT_COOP_STACK words. */
__device__ __forceinline__ bool coop_round(const float4 *__restrict__ nodes, const float4 *__restrict__ tris,
                                           CoopQuery &q, const CoopStack &gst, V3 o, V3 d, float tmin,
                                           uint32_t n_nodes, uint32_t n_recs, int multi_sp, unsigned long long *guard)
{
    const int lane = (int)(threadIdx.x & 63), sub = lane & 3, gbase = lane & ~3;
    if (q.sp <= 0) return true;
    const int L = q.sp <= multi_sp ? 4 : 1; /* lanes taking items this round */
    int e[4], cu[5];
    cu[0] = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        e[j] = gst[q.sp - 1 - j]; /* read past the bottom: slot 0, unused */
        /* entry j (from the top) takes one lane if a node, one per triangle if a leaf */
        const int dm = j >= q.sp ? 0 : e[j] >= 0 ? 1 : (int)(~(uint32_t)e[j] & 7u) + 1;
        cu[j + 1] = cu[j] + dm;
    }
    /* branch-free, alike in the 4 lanes: lane `sub` takes entry j with cu[j] <= sub < cu[j+1]; the
       entries with cu[j+1] <= L are taken whole, and a leaf only partly taken stays on the stack
       with its first triangles removed */
    const int n_act = cu[4] < L ? cu[4] : L; /* lanes 0 .. n_act - 1 hold an item */
    const bool act = sub < n_act;
    const int j = (sub >= cu[1] ? 1 : 0) + (sub >= cu[2] ? 1 : 0) + (sub >= cu[3] ? 1 : 0);
    const int item = j == 0 ? e[0] : j == 1 ? e[1] : j == 2 ? e[2] : e[3];
    const int off = sub - (j == 0 ? 0 : j == 1 ? cu[1] : j == 2 ? cu[2] : cu[3]);
    const int top = q.sp < 4 ? q.sp : 4;
    int nfull = (cu[1] <= L ? 1 : 0) + (cu[2] <= L ? 1 : 0) + (cu[3] <= L ? 1 : 0) + (cu[4] <= L ? 1 : 0);
    nfull = nfull < top ? nfull : top;
    const int cp = nfull == 0 ? 0 : nfull == 1 ? cu[1] : nfull == 2 ? cu[2] : cu[3];
    const bool partial = nfull < top && cp < L;
    const int ep = nfull == 0 ? e[0] : nfull == 1 ? e[1] : nfull == 2 ? e[2] : e[3];
    const uint32_t used = (uint32_t)(L - cp), enp = ~(uint32_t)ep;
    const int part = ~(int)((((enp >> 3) + used) << 3) | ((enp & 7u) - used));
    /* the partly taken leaf's rest goes back now, in place (below every push of this round), so
       that nothing of the assignment stays live across the round but nfull */
    if (partial && sub == 0) gst[q.sp - 1 - nfull] = part;
    const bool leaf = item < 0;
    const uint32_t slot = (~(uint32_t)item >> 3) + (uint32_t)off;
    /* every record index is checked: a defect ends the query instead of reading outside the tree,
       and is reported (the render then fails: rt_synchronize) */
    const bool bad = act && (leaf ? slot >= n_recs : (uint32_t)item >= n_nodes);
    if ((__ballot(bad) >> gbase) & 15ull) {
        if (sub == 0) atomicOr(guard, (unsigned long long)RT_GUARD_INDEX); /* rare path: no register carried */
        return true;
    }
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u w0 = {0u, 0u, 0u, 0u}, w1 = w0, w2 = w0, w3 = w0;
    if (act) {
        const v4u *vrec = reinterpret_cast<const v4u *>(leaf ? reinterpret_cast<const uint4 *>(tris) + 3 * slot
                                                             : reinterpret_cast<const uint4 *>(nodes) + 4 * item);
        w0 = vrec[0];
        w1 = vrec[1];
        w2 = vrec[2];
        if (!leaf) w3 = vrec[3];
    }
    asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
    float ct = kInf, lbound = 0.0f;
    int co = -1, cs = -1, nh = 0;
    float t[4];
    int c[4];
    if (act && leaf) {
        const float4 ta = make_float4(__uint_as_float(w0.x), __uint_as_float(w0.y), __uint_as_float(w0.z),
                                      __uint_as_float(w0.w));
        const float4 tb = make_float4(__uint_as_float(w1.x), __uint_as_float(w1.y), __uint_as_float(w1.z), 0.0f);
        const float4 tc = make_float4(__uint_as_float(w2.x), __uint_as_float(w2.y), __uint_as_float(w2.z), 0.0f);
        float tt = 0.0f;
        const bool h = mt_test(o, d, ta, tb, tc, tt);
        const int orig = __float_as_int(ta.w);
        if (h && !(tt < tmin) && (tt < q.best_t || (tt == q.best_t && orig > q.best_orig))) {
            ct = tt;
            co = orig;
            cs = (int)slot;
        }
        lbound = __uint_as_float(w1.w); /* a list record: the next candidate's bound (tree leaves: 0) */
    } else if (act) {
        const uint4 q0 = make_uint4(w0.x, w0.y, w0.z, w0.w), q1 = make_uint4(w1.x, w1.y, w1.z, w1.w);
        const uint4 q2 = make_uint4(w2.x, w2.y, w2.z, w2.w), q3 = make_uint4(w3.x, w3.y, w3.z, w3.w);
        nh = node_children(q0, q1, q2, q3, q.inv, q.oi, d, q.best_t, false, false, t, c);
    }
    /* the group's best candidate: minimum t, ties to the highest original index */
    {
        const float ot = quad_xorf1(ct);
        const int oo = quad_xor<1>(co), os = quad_xor<1>(cs);
        const bool take = os >= 0 && (cs < 0 || ot < ct || (ot == ct && oo > co));
        ct = take ? ot : ct;
        co = take ? oo : co;
        cs = take ? os : cs;
    }
    {
        const float ot = quad_xorf2(ct);
        const int oo = quad_xor<2>(co), os = quad_xor<2>(cs);
        const bool take = os >= 0 && (cs < 0 || ot < ct || (ot == ct && oo > co));
        ct = take ? ot : ct;
        co = take ? oo : co;
        cs = take ? os : cs;
    }
    if (cs >= 0) {
        q.best = cs;
        q.best_t = ct;
        q.best_orig = co;
    }
    if (q.best_t < __int_as_float(quad_bcast(__float_as_int(lbound), n_act - 1))) return true;
    /* the stack: the taken entries off, a partly taken leaf back on top, then each node lane's hit
       children (lane 0's on top, each lane's nearest child last) */
    const int h1 = quad_dpp<0x55>(nh), h2 = quad_dpp<0xAA>(nh), h3 = quad_dpp<0xFF>(nh);
    const int total = quad_dpp<0x00>(nh) + h1 + h2 + h3;
    const int above = (sub < 1 ? h1 : 0) + (sub < 2 ? h2 : 0) + (sub < 3 ? h3 : 0);
    const int sp = q.sp - nfull;
    if (sp + total > CoopStack::kCap) { /* cannot happen (multi_sp bound, rt_host.cpp): reported, not clamped */
        if (sub == 0) atomicOr(guard, (unsigned long long)RT_GUARD_STACK);
        return true;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < nh) gst[sp + above + nh - 1 - i] = c[i];
    q.sp = sp + total;
    return q.sp == 0;
}

#ifndef RT_SEED_STATS
#define RT_SEED_STATS 0 /* diagnostics builds: per-pixel query / immediate-answer / iteration counts (RT_PIXEL_STATS) */
#endif
#ifndef RT_SEED_IMM
#define RT_SEED_IMM 2 /* path-advance passes per seed-pass iteration (queries answered at once chain) */
#endif

/* A cooperative query of the tree starts at the root's children: the root node (uniform, loaded
   once per wave into registers) is tested in the path advance instead of in a stepping round of
   its own, and the hit children go on the group's stack, nearest on top.  Returns false when no
   child box is hit (or the determinant cull rules the tree out): no mesh hit, without a round.
   Culling only: the same children coop_round would push from the root. */
__device__ __forceinline__ bool coop_root(uint4 r0, uint4 r1, uint4 r2, uint4 r3, CoopQuery &q, const CoopStack &gst, V3 d,
                                          bool writer)
{
    float t[4];
    int c[4];
    const int nh = node_children(r0, r1, r2, r3, q.inv, q.oi, d, q.best_t, false, false, t, c);
    if (writer) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < nh) gst[nh - 1 - i] = c[i];
    }
    q.sp = nh;
    return nh > 0;
}

/* The same for a one-lane query (trav_step_q's state): the root's hit children go on the lane's
   stack, the nearest becomes the next node.  Returns false when none is hit. */
__device__ __forceinline__ bool lane_root(uint4 r0, uint4 r1, uint4 r2, uint4 r3, TravState &s, Stack &stk, V3 d)
{
    float t[4];
    int c[4];
    const int nh = node_children(r0, r1, r2, r3, s.inv, s.oi, d, s.best_t, false, false, t, c);
    if (nh >= 4) stk.push(c[3]);
    if (nh >= 3) stk.push(c[2]);
    if (nh >= 2) stk.push(c[1]);
    s.node = c[0];
    return nh > 0;
}

template <int G> /* lanes per query: 1 (trav_step_q) or 4 (coop_round) */
__device__ __forceinline__ void seed_pass(const RtTriLaunch &a, int *s_stack)
{
    constexpr bool COOP = G > 1;
    Stack stk;
    stk.init(s_stack, a.spill, a.spill_cap);
    const int lane = (int)(threadIdx.x & 63), gbase = lane & ~(G - 1);
    CoopStack gst;
    gst.base = (lds_int *)(s_stack + (threadIdx.x & ~63u) + (uint32_t)gbase);
    if (COOP) /* the wave's stack words start as the root: an entry read before it is written is a node */
        for (int k = 0; k < RT_STACK_DEPTH; ++k) s_stack[k * RT_BLOCK + threadIdx.x] = 0;
    const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(a.nodes);
    const float4 *__restrict__ tris = reinterpret_cast<const float4 *>(a.tris);
    /* the root node (coop_root): a uniform address, so scalar loads */
    const uint4 *__restrict__ rootp = reinterpret_cast<const uint4 *>(a.nodes);
    const uint4 rq0 = rootp[0], rq1 = rootp[1], rq2 = rootp[2], rq3 = rootp[3];
    const uint32_t spp = a.sample_rate * a.sample_rate, fine = a.split_fine, nseed = a.split_nseed;
    const uint32_t plane = a.Wpad * a.Hpad;
    const uint32_t tiles_x = (a.W + 7u) >> 3, tiles_y = (a.Hl + 7u) >> 3;
    const uint32_t n_items = a.split_which == RT_SPLIT_BOX ? box_items(a)
                                                           : tiles_x * tiles_y * 64u;
    const uint32_t nl = a.n_lights;
    const float hw = uniform_f(((float)a.W) / 2.0f);
    const float hh = uniform_f(((float)a.H) / 2.0f);
    const float bw = (float)RT_BOX_WIDTH, bh = (float)RT_BOX_HEIGHT;
    bool have = false, next = false, running = false, fin = false, drained = false;
    uint32_t x = 0, yl = 0, sample = 0, depth = 0;
    uint32_t pslot = 0; /* the chain's seeds: its pixel, or its slot (split_seed_slot) */
    uint32_t lpack = RT_LPACK_NONE; /* the pixel's candidate list (list_pack) */
    uint32_t bnext = 0, bend = 0; /* the wave's batch of queue items (batch_take) */
    Seed seed = {0u, 0u};
    V3 qo = v3(0.0f, 0.0f, 0.0f), qd = v3(0.0f, 0.0f, 1.0f);
    TravState ts;
    ts.node = 0;
    ts.best = -1;
    ts.best_orig = -1;
    ts.best_t = kInf;
    ts.inv = qo;
    ts.oi = qo;
    CoopQuery cq;
    coop_begin(cq, qo, qd, kInf);
    uint32_t st_steps = 0, st_box = 0, st_t0 = 0; /* diagnostics (RT_PIXEL_STATS): per pixel */
    uint32_t q_steps = 0;                          /* rounds of the current query */
    /* diagnostics builds (RT_SEED_STATS): per pixel the queries that took rounds, the queries
       answered in the path advance, and the loop iterations */
    uint32_t st_q = 0, st_imm = 0, st_it = 0;
    unsigned long long st_adv = 0, st_rnd = 0; /* clocks in the path advance / in stepping rounds */
    unsigned long long *const guard = a.counters + RT_CNT_GUARD; /* RT_GUARD_* flags (rt_synchronize) */
    for (;;) {
        /* lanes (COOP: groups) without a pixel take the next ones of the queue */
        /* takers: the first split_gpw lanes (COOP: 4-lane groups) of the wave */
        const uint32_t gpw = a.split_gpw ? a.split_gpw : 64u / G;
        const unsigned long long idle = __ballot(!have && lane == gbase && (uint32_t)(lane / G) < gpw);
        if (idle && !drained) {
            /* a batch per wave of as many items as it has takers */
            uint32_t item = batch_take(a.split_counter, idle, bnext, bend, gpw);
            if (COOP) item = __shfl(item, gbase);
            drained = bnext >= n_items;
            if (!have) {
                if (item < n_items) {
                    bool take;
                    if (a.split_which == RT_SPLIT_BOX) { /* the box pixels (long chains), by slot */
                        const uint32_t p = a.split_box[a.split_item_base + item];
                        x = p % a.W;
                        yl = p / a.W;
                        pslot = a.split_seed_slot ? item : p;
                        take = true;
                    } else {
                        uint32_t tile = item >> 6;
                        const uint32_t in = item & 63u;
                        if (a.tile_order) tile = a.tile_order[tile];
                        x = (tile % tiles_x) * 8u + (in & 7u);
                        yl = (tile / tiles_x) * 8u + (in >> 3);
                        take = x < a.W && yl < a.Hl;
                        if (take && a.split_which == RT_SPLIT_MESH) take = a.pixel_class[(size_t)yl * a.W + x] == -1;
                        pslot = yl * a.W + x;
                    }
                    if (take) {
                        const uint32_t slot = global_row(a, yl) * a.Wpad + x;
                        seed.x = a.seeds[slot];
                        seed.y = a.seeds[plane + slot];
                        lpack = list_pack(a, x, yl, tiles_x);
                        sample = 0;
                        have = true;
                        next = true;
                        if (a.pixel_stats) {
                            st_steps = st_box = 0;
                            if (RT_SEED_STATS) {
                                st_q = st_imm = st_it = 0;
                                st_adv = st_rnd = 0;
                            }
                            st_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        }
                    }
                }
            }
        }
        if (!__any(have)) {
            if (drained) break;
            continue;
        }
        /* The path advance, over as many segments and samples as it takes before the next stepping
           round: a new sample's camera ray, and every query answered without a round — an empty
           candidate list, a box bounce whose ray misses the root's child boxes (tested from
           registers) — advances at once, up to RT_SEED_IMM passes.  Box paths mostly
           leave the mesh's box alone, so a long chain's samples are mostly resolved here, without a
           memory round trip. */
        const unsigned long long t_adv0 = RT_SEED_STATS ? wave_clock() : 0ull;
        for (int pass = 0;; ++pass) {
            /* a new sample: the chunk's first seed, then the camera ray and its query */
            if (next) {
                next = false;
                if ((sample == spp || sample % fine == 0u) && lane == gbase) {
                    const uint32_t c = sample == spp ? nseed - 1u : sample / fine;
                    reinterpret_cast<uint2 *>(a.split_seed)[(size_t)pslot * nseed + c] = make_uint2(seed.x, seed.y);
                }
                if (sample == spp) {
                    have = false;
                    if (a.pixel_stats && lane == gbase) {
                        uint32_t *ps = a.pixel_stats + 8 * ((size_t)yl * a.W + x);
                        ps[0] = st_t0;
                        ps[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        ps[2] = st_steps;
                        ps[3] = st_box;
                        ps[4] = 1u + (uint32_t)a.split_which | (RT_SEED_STATS ? st_it << 4 : 0u);
                        if (RT_SEED_STATS) {
                            ps[7] = st_q << 16 | (st_imm & 0xffffu);
                            ps[5] = (uint32_t)(st_adv >> 6);
                            ps[6] = (uint32_t)(st_rnd >> 6);
                        }
                    }
                } else {
                    const uint32_t sx = sample / a.sample_rate, sy = sample % a.sample_rate;
                    const float fa = (float)x + strat_rand(seed, (int)sx, (int)a.sample_rate);
                    const uint32_t y = global_row(a, yl);
                    const float fb = (float)y + strat_rand(seed, (int)sy, (int)a.sample_rate);
                    qo = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
                    qd = camera_dir(a.cam, fa - hw, fb - hh);
                    depth = 0;
                    if (COOP) coop_begin(cq, qo, qd, kInf);
                    else trav_begin(ts, stk, qo, qd, kInf);
                    q_steps = 0;
                    running = true;
                    { /* the pixel's candidate list, as k_tris takes it */
                        const uint32_t pc = (lpack & (RT_LIST_MAX - 1u)) + 1u, first = (lpack >> RT_LIST_BITS) << 3;
                        if (lpack == RT_LPACK_EMPTY) {
                            running = false;
                            ts.best = -1;
                            cq.best = -1;
                            fin = true;
                        } else if (lpack != RT_LPACK_NONE) {
                            for (uint32_t b = (pc - 1u) >> 3; b > 0u; --b) {
                                const uint32_t k = pc - 8u * b < 8u ? pc - 8u * b : 8u;
                                const int v = ~(int)(((first + 8u * b) << 3) | (k - 1u));
                                if (COOP) {
                                    if (lane == gbase) gst[cq.sp] = v;
                                    ++cq.sp;
                                } else {
                                    stk.push(v);
                                }
                            }
                            const int n0 = ~(int)((first << 3) | ((pc < 8u ? pc : 8u) - 1u));
                            if (COOP) { /* coop_round: the list's first block on top */
                                if (lane == gbase) gst[cq.sp] = n0;
                                ++cq.sp;
                            } else {
                                ts.node = n0;
                            }
                        } else if (COOP) { /* no list: the tree, from the root's children */
                            if (!coop_root(rq0, rq1, rq2, rq3, cq, gst, qd, lane == gbase)) {
                                running = false;
                                fin = true;
                            }
                        } else if (!lane_root(rq0, rq1, rq2, rq3, ts, stk, qd)) {
                            running = false;
                            fin = true;
                        }
                    }
                }
            }
            /* lanes whose query completed: the segment's draws, then the bounce or the next sample */
            if (fin) {
                fin = false;
                if (RT_SEED_STATS && q_steps == 0) ++st_imm; /* answered without a round */
                bool sample_done = true;
                const bool mesh_hit = (COOP ? cq.best : ts.best) >= 0;
                if (mesh_hit) { /* mesh hit: the light samples' draws, no bounce (rtcommon.h:411-421) */
                    for (uint32_t l = 0; l < nl; ++l) {
                        (void)frand(seed);
                        (void)frand(seed);
                    }
                } else { /* the enclosing box (rtcommon.h:425-466) */
                    const float hd = intersect_box(qo, qd, RT_SMALL_F, bw, bh, bw);
                    if (depth == 0) ++st_box;
                    if (hd > RT_SMALL_F && hd < kInf) {
                        const V3 hp = v3(qo.x + qd.x * hd, qo.y + qd.y * hd, qo.z + qd.z * hd);
                        const V3 hn = box_normal(hp, bw, bh, bw);
                        for (uint32_t l = 0; l < nl; ++l) {
                            (void)frand(seed);
                            (void)frand(seed);
                        }
                        const float r1 = frand(seed);
                        const float r2 = frand(seed);
                        const float ct = rt_sqrtf(1.0f - r1);
                        const float st = rt_sqrtf(1.0f - ct * ct);
                        const float phi = RT_M_2PI_F * r2;
                        float sphi, cphi;
                        rt_sincosf(phi, &sphi, &cphi);
                        qd = shading_to_world(v3(cphi * st, sphi * st, ct), hn);
                        qo = hp;
                        ++depth;
                        if (depth <= a.max_depth) {
                            sample_done = false;
                            q_steps = 0;
                            running = true;
                            if (COOP) {
                                coop_begin(cq, qo, qd, kInf);
                                if (!coop_root(rq0, rq1, rq2, rq3, cq, gst, qd, lane == gbase)) {
                                    running = false; /* misses the mesh's box: no mesh hit, at once */
                                    fin = true;
                                }
                            } else {
                                trav_begin(ts, stk, qo, qd, kInf);
                                if (!lane_root(rq0, rq1, rq2, rq3, ts, stk, qd)) {
                                    running = false;
                                    fin = true;
                                }
                            }
                        }
                    }
                }
                if (sample_done) {
                    /* the sample's mesh-hit depth (0xff: only the box), as k_chain_seeds stores it */
                    if (a.split_hit_depth && lane == gbase)
                        a.split_hit_depth[(size_t)pslot * spp + sample] = mesh_hit ? (uint8_t)depth : (uint8_t)0xffu;
                    ++sample;
                    next = true;
                }
            }
            /* at most RT_SEED_IMM passes before the next stepping round: the lanes whose queries
               need a traversal must not wait long for those whose answers come at once */
            if (pass + 1 >= RT_SEED_IMM || !__any(next || fin)) break;
        }
        unsigned long long t_rnd0 = 0;
        if (RT_SEED_STATS) {
            ++st_it;
            t_rnd0 = wave_clock();
            st_adv += t_rnd0 - t_adv0;
        }
        /* step the running queries (the box pixels' chains at top priority: they run beside the
           chunk tasks and set when the box pixels' chunks can start) */
        if (a.split_which == RT_SPLIT_BOX) __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (int u = 0; u < RT_SEED_UNROLL; ++u) {
            if (running) {
                ++st_steps;
                ++q_steps;
                bool done;
                if constexpr (G == 4) {
                    done = coop_round(nodes, tris, cq, gst, qo, qd, RT_SMALL_F, a.n_nodes4, a.n_recs, a.coop_multi_sp,
                                      guard);
                } else {
                    TravCounts tc = {0u, 0u, 0u};
                    done = trav_step_q<false>(nodes, tris, ts, stk, qo, qd, RT_SMALL_F, false, tc);
                }
                /* The seed needs only WHETHER a segment hits the mesh (a hit ends the sample
                   after the light samples' draws, wherever it is): the query ends at its first
                   accepted triangle (the closest-hit rule's acceptance, t >= tmin) */
                const bool exists = (COOP ? cq.best : ts.best) >= 0; /* the query ends at its first accepted triangle */
                /* a query never takes 2^14 rounds (a ray meets far fewer nodes than that):
                   a bound every wave reaches, whatever a defect would do to a stack (reported) */
                if (q_steps > (1u << 14)) atomicOr(guard, (unsigned long long)RT_GUARD_ROUNDS);
                if (done || exists || q_steps > (1u << 14)) {
                    running = false;
                    fin = true;
                    if (RT_SEED_STATS) ++st_q;
                }
            }
        }
        if (RT_SEED_STATS) st_rnd += wave_clock() - t_rnd0;
    }
}

/* One MWC generator of frand (rng.h:9-47: x = A (x & 0xffff) + (x >> 16)) advanced by k draws.
   With M = A 2^16 - 1 the step is x -> A x mod M on the states below M (the step keeps them
   there; a fresh seed at or above M gets there within 2 steps, M itself is a fixed point), so
   k draws are one multiplication by A^k mod M (`mul`, from the host); a^-1 = 2^16 mod M undoes
   the canonicalising steps.  Small k: the steps themselves. */
/* Does the segment o + t d, tmin <= t <= tmax, miss the box [lo, hi]?  Slab test with the hardware
   reciprocal; the box is the mesh's bounds padded far beyond the test's rounding (mesh_bounds), so
   a segment reported missing meets no triangle.  A zero direction component on a slab plane gives
   0 x inf = NaN, which min/max drop (a ray in that plane lies outside the triangles' padded box
   anyway). */
__device__ __forceinline__ bool segment_misses_box(V3 o, V3 d, float tmin, float tmax, const float *lo, const float *hi)
{
    const float ix = __builtin_amdgcn_rcpf(d.x), iy = __builtin_amdgcn_rcpf(d.y), iz = __builtin_amdgcn_rcpf(d.z);
    const float x1 = (lo[0] - o.x) * ix, x2 = (hi[0] - o.x) * ix;
    const float y1 = (lo[1] - o.y) * iy, y2 = (hi[1] - o.y) * iy;
    const float z1 = (lo[2] - o.z) * iz, z2 = (hi[2] - o.z) * iz;
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x1, x2), __builtin_fminf(y1, y2)),
                                     __builtin_fmaxf(__builtin_fminf(z1, z2), tmin));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x1, x2), __builtin_fmaxf(y1, y2)),
                                     __builtin_fminf(__builtin_fmaxf(z1, z2), tmax));
    return tn > tf;
}

template <uint32_t A>
__device__ __forceinline__ uint32_t mwc_jump(uint32_t x, uint32_t k, uint32_t mul)
{
    constexpr uint32_t M = A * 65536u - 1u;
    if (k <= 16u) {
        for (uint32_t i = 0; i < k; ++i) x = A * (x & 65535u) + (x >> 16);
        return x;
    }
    uint32_t k0 = 0;
    while (x > M) { /* at most 2 steps (every 32-bit state checked) */
        x = A * (x & 65535u) + (x >> 16);
        ++k0;
    }
    if (x == M) return M;
    for (uint32_t i = 0; i < k0; ++i) mul = (uint32_t)(((unsigned long long)mul * 65536u) % M);
    return (uint32_t)(((unsigned long long)x * mul) % M);
}

/* ------------------------------------------------------------------------ */
/* Subtree-parallel seed pass of the long chains (k_chain_seeds): G lanes per chain.  The seed
   needs only WHETHER a segment meets the mesh (an accepted triangle anywhere), and that answer
   is an OR over any cut of the tree: lane `sub` of a group owns edge `sub` of a fixed cut of the
   tree's top levels (a child slot of a node — chain_cut, breadth first, at most G edges), tests
   that child's box from an LDS copy of its parent's record when a query starts, and walks the
   subtree below alone, depth first, with k_tris's one-record step (trav_step_q) and its own
   stack; the query ends at the first step after which some lane of the group has accepted a
   triangle, or when every lane's subtree is exhausted.  A camera ray with a candidate list
   spreads the list's triangles over the lanes in runs of ceil(count / G).  The group's lanes
   carry the chain's path state alike (the same values computed in every lane), so a path
   advance costs one lane's instructions; the work of a query is split over G lanes without a
   shared stack or an item assignment (coop_round's cost: DESIGN.md §4.5). */
#ifndef RT_CHAIN_IMM
#define RT_CHAIN_IMM 2 /* path-advance passes per iteration */
#endif
#ifndef RT_CHAIN_UNROLL
#define RT_CHAIN_UNROLL 3 /* traversal steps per iteration (1 / 2 / 3 / 4: 8-way tile 16.8 / 16.4 / 16.3 / 16.4 ms, r04h2) */
#endif

/* child slot k of a compressed node against the ray, unsorted: node_children's box test for one
   child (the same plane values: byte * 2^e * inv + (origin * inv - o * inv)) and the node's
   determinant cull.  Culling only. */
__device__ __forceinline__ bool edge_hit(uint4 q0, uint4 q1, uint4 q2, int k, V3 inv, V3 oi, V3 d)
{
    const uint32_t w = q0.w;
    const float sx = __builtin_amdgcn_ldexpf(inv.x, (int)(w & 31u) + RT_QEXP_MIN);
    const float sy = __builtin_amdgcn_ldexpf(inv.y, (int)((w >> 5) & 31u) + RT_QEXP_MIN);
    const float sz = __builtin_amdgcn_ldexpf(inv.z, (int)((w >> 10) & 31u) + RT_QEXP_MIN);
    const float bx = __builtin_fmaf(__uint_as_float(q0.x), inv.x, -oi.x);
    const float by = __builtin_fmaf(__uint_as_float(q0.y), inv.y, -oi.y);
    const float bz = __builtin_fmaf(__uint_as_float(q0.z), inv.z, -oi.z);
    const bool px = inv.x >= 0.0f, py = inv.y >= 0.0f, pz = inv.z >= 0.0f;
    const uint32_t sh = 8u * (uint32_t)k;
    const float nbx = (float)(((px ? q1.x : q1.y) >> sh) & 255u), fbx = (float)(((px ? q1.y : q1.x) >> sh) & 255u);
    const float nby = (float)(((py ? q1.z : q1.w) >> sh) & 255u), fby = (float)(((py ? q1.w : q1.z) >> sh) & 255u);
    const float nbz = (float)(((pz ? q2.x : q2.y) >> sh) & 255u), fbz = (float)(((pz ? q2.y : q2.x) >> sh) & 255u);
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(nbx, sx, bx), __builtin_fmaf(nby, sy, by)),
                                     __builtin_fmaxf(__builtin_fmaf(nbz, sz, bz), -1e-3f));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaf(fbx, sx, bx), __builtin_fmaf(fby, sy, by)),
                                     __builtin_fmaf(fbz, sz, bz));
    if (!(tn <= tf)) return false;
    /* the determinant cull of node_children */
    const uint32_t nlo = q2.z, nhi = q2.w;
    const float nsc = __builtin_amdgcn_ldexpf(1.0f, (int)(nlo >> 24) - 128);
    const uint32_t sel_n = (px ? 4u : 0u) | (py ? 5u : 1u) << 8 | (pz ? 6u : 2u) << 16;
    const uint32_t sel_f = (px ? 0u : 4u) | (py ? 1u : 5u) << 8 | (pz ? 2u : 6u) << 16;
    const uint32_t nb = __builtin_amdgcn_perm(nhi, nlo, sel_n), fb = __builtin_amdgcn_perm(nhi, nlo, sel_f);
    const float bias = 128.0f * (d.x + d.y + d.z);
    const float fhi = __builtin_fmaf(d.x, (float)(nb & 0xffu),
                                     __builtin_fmaf(d.y, (float)((nb >> 8) & 0xffu),
                                                    __builtin_fmaf(d.z, (float)((nb >> 16) & 0xffu), -bias)));
    const float flo = __builtin_fmaf(d.x, (float)(fb & 0xffu),
                                     __builtin_fmaf(d.y, (float)((fb >> 8) & 0xffu),
                                                    __builtin_fmaf(d.z, (float)((fb >> 16) & 0xffu), -bias)));
    const float l1 = __builtin_fabsf(d.x) + __builtin_fabsf(d.y) + __builtin_fabsf(d.z);
    const float bound = __builtin_fmaf(__builtin_fmaxf(fhi, -flo) * nsc, 1.02f, 5e-7f * l1);
    return !(bound < 1e-4f);
}

__device__ __forceinline__ int link_of(uint4 l, int k) { return (int)(k == 0 ? l.x : k == 1 ? l.y : k == 2 ? l.z : l.w); }

/* The cut: the root's used child slots, then, level by level (a pass over the list in order), an
   edge to an inner node replaced by that node's used slots while the list stays within G edges.
   Thread 0 of the block, into s_par / s_slot; returns the edge count. */
template <int G>
__device__ int chain_cut(const uint4 *__restrict__ qn, uint32_t n_nodes, int *s_par, int *s_slot)
{
    if (n_nodes == 0) return 0;
    int n = 0;
    {
        const uint4 l = qn[3];
        for (int k = 0; k < 4; ++k)
            if (link_of(l, k) != RT_EMPTY_CHILD && n < G) {
                s_par[n] = 0;
                s_slot[n] = k;
                ++n;
            }
    }
    for (bool grew = true; grew;) {
        grew = false;
        for (int i = 0; i < n;) {
            const int c = link_of(qn[4 * s_par[i] + 3], s_slot[i]);
            if (c < 0 || c == RT_EMPTY_CHILD || (uint32_t)c >= n_nodes) {
                ++i;
                continue;
            }
            const uint4 l = qn[4 * c + 3];
            int m = 0;
            for (int k = 0; k < 4; ++k) m += link_of(l, k) != RT_EMPTY_CHILD ? 1 : 0;
            if (m == 0 || n - 1 + m > G) {
                ++i;
                continue;
            }
            for (int j = n - 1; j > i; --j) {
                s_par[j + m - 1] = s_par[j];
                s_slot[j + m - 1] = s_slot[j];
            }
            int t = i;
            for (int k = 0; k < 4; ++k)
                if (link_of(l, k) != RT_EMPTY_CHILD) {
                    s_par[t] = c;
                    s_slot[t] = k;
                    ++t;
                }
            n += m - 1;
            i += m; /* the new edges are the next level's: not expanded in this pass */
            grew = true;
        }
    }
    return n;
}

/* intersect_box (geometryFuncs.h:86-150) for a group of G >= 8 lanes carrying the same ray: the
   six slab divisions one per lane (lanes 0-5 of the group), gathered; the same operations on
   the same values as intersect_box, so the same bits. */
__device__ __forceinline__ float group_box(V3 o, V3 d, float tmin, float xs, float ys, float zs, int sub, int gbase)
{
    const int kk = sub < 6 ? sub : 0, ax = kk >> 1;
    const float oa = ax == 0 ? o.x : ax == 1 ? o.y : o.z, da = ax == 0 ? d.x : ax == 1 ? d.y : d.z;
    const float sa = ax == 0 ? xs : ax == 1 ? ys : zs;
    const float q = ((kk & 1) ? (0.0f + sa) - oa : (0.0f - sa) - oa) / da;
    const float tx1 = __shfl(q, gbase), tx2 = __shfl(q, gbase + 1), ty1 = __shfl(q, gbase + 2);
    const float ty2 = __shfl(q, gbase + 3), tz1 = __shfl(q, gbase + 4), tz2 = __shfl(q, gbase + 5);
    float nt = 0.0f, ft = rt_inff();
    if (d.x != 0) {
        nt = rt_minf(tx1, tx2);
        ft = rt_maxf(tx1, tx2);
    } else if (rt_fabsf(o.x - 0.0f) > xs) {
        return 0;
    }
    if (d.y != 0) {
        if (ty1 > ty2) {
            nt = rt_maxf(ty2, nt);
            ft = rt_minf(ty1, ft);
        } else {
            nt = rt_maxf(ty1, nt);
            ft = rt_minf(ty2, ft);
        }
    } else if (rt_fabsf(o.y - 0.0f) > ys) {
        return 0;
    }
    if (d.z != 0) {
        if (tz1 > tz2) {
            nt = rt_maxf(tz2, nt);
            ft = rt_minf(tz1, ft);
        } else {
            nt = rt_maxf(tz1, nt);
            ft = rt_minf(tz2, ft);
        }
    } else if (rt_fabsf(o.z - 0.0f) > zs) {
        return 0;
    }
    if (nt > ft || ft < tmin) return rt_inff();
    if (nt < tmin) return ft;
    return nt;
}

/* box_normal (geometryFuncs.h:71-84): -p / |p| is exactly -1 or +1 for a finite non-zero p, so the
   division runs only for the rest (0 or infinite: NaN, as the reference's) */
__device__ __forceinline__ float neg_sign(float p)
{
    if (p != 0.0f && rt_fabsf(p) < rt_inff()) return p > 0.0f ? -1.0f : 1.0f;
    return -p / rt_fabsf(p);
}
__device__ __forceinline__ V3 box_normal_signs(V3 p, float xs, float ys, float zs)
{
    const float dx = rt_fabsf(rt_fabsf(p.x) - xs);
    const float dy = rt_fabsf(rt_fabsf(p.y) - ys);
    const float dz = rt_fabsf(rt_fabsf(p.z) - zs);
    if (dx < dy && dx < dz) return v3(neg_sign(p.x), 0.0f, 0.0f);
    if (dy < dz) return v3(0.0f, neg_sign(p.y), 0.0f);
    return v3(0.0f, 0.0f, neg_sign(p.z));
}

/* camera_dir for a group of G >= 8 lanes: the three divisions by the length on lanes 0-2 */
__device__ __forceinline__ V3 group_camera_dir(const rt_camera &cam, float a, float b, int sub, int gbase)
{
    const float x = (cam.view.x + cam.right.x * a) + cam.up.x * b;
    const float y = (cam.view.y + cam.right.y * a) + cam.up.y * b;
    const float z = (cam.view.z + cam.right.z * a) + cam.up.z * b;
    const float w = (cam.view.w + cam.right.w * a) + cam.up.w * b;
    const float len = rt_sqrtf(((x * x + y * y) + z * z) + w * w);
    const int kk = sub < 3 ? sub : 0;
    const float q = (kk == 0 ? x : kk == 1 ? y : z) / len;
    return v3(__shfl(q, gbase), __shfl(q, gbase + 1), __shfl(q, gbase + 2));
}

template <int G, bool RUNS = false> /* RUNS: the repair pass's runs of hit samples */
__global__ __launch_bounds__(RT_BLOCK, RT_TRIS_WAVES) void k_chain_seeds(RtTriLaunch a)
{
    static_assert(G >= 8 && G <= 64 && (G & (G - 1)) == 0, "the advance spreads 6 divisions over the group's lanes");
    __shared__ int s_stack[RT_STACK_DEPTH * RT_BLOCK];
    __shared__ uint4 s_erec[G][4]; /* per edge: its parent's record */
    __shared__ int s_par[G], s_slot[G];
    __shared__ int s_ne;
    if (box_items(a) == 0u) return; /* an empty list (the repair pass, mostly): no cut to make */
    const uint4 *__restrict__ qn = reinterpret_cast<const uint4 *>(a.nodes);
    if (threadIdx.x == 0) s_ne = chain_cut<G>(qn, a.n_nodes4, s_par, s_slot);
    __syncthreads();
    const int ne = s_ne;
    for (int i = (int)threadIdx.x; i < 4 * ne; i += RT_BLOCK) s_erec[i >> 2][i & 3] = qn[4 * s_par[i >> 2] + (i & 3)];
    __syncthreads();
    __builtin_amdgcn_s_setprio(3); /* the long chains run beside the chunk tasks and set when their own chunks start */

    Stack stk;
    stk.init(s_stack, a.spill, a.spill_cap);
    const int lane = (int)(threadIdx.x & 63), sub = lane & (G - 1), gbase = lane & ~(G - 1);
    const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
    const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(a.nodes);
    const float4 *__restrict__ tris = reinterpret_cast<const float4 *>(a.tris);
    const int eslot = sub < ne ? s_slot[sub] : 0;
    const uint32_t spp = a.sample_rate * a.sample_rate, fine = a.split_fine, nseed = a.split_nseed;
    const uint32_t plane = a.Wpad * a.Hpad;
    const uint32_t tiles_x = (a.W + 7u) >> 3;
    const uint32_t n_items = box_items(a);
    const uint32_t nl = a.n_lights;
    const float hw = uniform_f(((float)a.W) / 2.0f);
    const float hh = uniform_f(((float)a.H) / 2.0f);
    const float bw = (float)RT_BOX_WIDTH, bh = (float)RT_BOX_HEIGHT;
    const uint32_t gpw = a.split_gpw ? a.split_gpw : 64u / G;
    bool have = false, next = false, running = false, fin = false, drained = false, live = false, ghit = false;
    uint32_t x = 0, yl = 0, sample = 0, depth = 0, pslot = 0; /* pslot: the chain's seeds (pixel or slot) */
    uint32_t lpack = RT_LPACK_NONE;
    uint32_t bnext = 0, bend = 0;
    Seed seed = {0u, 0u};
    V3 qo = v3(0.0f, 0.0f, 0.0f), qd = v3(0.0f, 0.0f, 1.0f);
    TravState ts;
    ts.node = 0;
    ts.best = -1;
    ts.best_orig = -1;
    ts.best_t = kInf;
    ts.inv = qo;
    ts.oi = qo;
    uint32_t st_steps = 0, st_box = 0, st_t0 = 0, q_steps = 0;
    unsigned long long *const guard = a.counters + RT_CNT_GUARD;
    /* a query of the tree starts at the lane's edge of the cut; false: no lane of the group
       enters its child's box (no mesh hit, without a step) */
    auto start_tree = [&]() -> bool {
        live = false;
        if (sub < ne) {
            const uint4 p0 = s_erec[sub][0], p1 = s_erec[sub][1], p2 = s_erec[sub][2], p3 = s_erec[sub][3];
            if (edge_hit(p0, p1, p2, eslot, ts.inv, ts.oi, qd)) {
                live = true;
                ts.node = link_of(p3, eslot);
            }
        }
        return (__ballot(live) & gmask) != 0ull;
    };
    for (;;) {
        const unsigned long long idle = __ballot(!have && lane == gbase && (uint32_t)(lane / G) < gpw);
        if (idle && !drained) {
            uint32_t item = batch_take(a.split_counter, idle, bnext, bend, gpw);
            item = __shfl(item, gbase);
            drained = bnext >= n_items;
            if (!have && item < n_items) {
                const uint32_t p = a.split_box[a.split_item_base + item];
                pslot = a.split_seed_slot ? item : p;
                x = p % a.W;
                yl = p / a.W;
                const uint32_t slot = global_row(a, yl) * a.Wpad + x;
                seed.x = a.seeds[slot];
                seed.y = a.seeds[plane + slot];
                sample = 0;
                if (a.split_restart) { /* a repaired pixel: from its first missed chunk, whose seed the
                                          jump gives (every sample before it hit the mesh) */
                    const uint32_t ch = a.split_restart[p];
                    const uint32_t k = ch * a.split_restart_chunk * a.split_spec_draws;
                    seed.x = mwc_jump<36969u>(seed.x, k, a.split_spec_mul[2 * ch]);
                    seed.y = mwc_jump<18000u>(seed.y, k, a.split_spec_mul[2 * ch + 1]);
                    sample = ch * a.split_restart_chunk;
                }
                lpack = list_pack(a, x, yl, tiles_x);
                have = true;
                next = true;
                if (a.pixel_stats) {
                    st_steps = st_box = 0;
                    st_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
                }
            }
        }
        if (!__any(have)) {
            if (drained) break;
            continue;
        }
        /* the path advance (alike in the group's lanes), up to RT_CHAIN_IMM passes: a finished
           query's bounce (or the end of its sample), a new sample's camera ray, then at most one
           query start per pass — its ray answered at once when it enters no subtree's box.  The
           advance's IEEE divisions are spread over the group's lanes (one each, gathered) */
        for (int pass = 0;; ++pass) {
            bool start = false;
            if (fin) {
                fin = false;
                bool sample_done = true;
                if (ghit) { /* mesh hit: the light samples' draws, no bounce (rtcommon.h:411-421) */
                    for (uint32_t l = 0; l < nl; ++l) {
                        (void)frand(seed);
                        (void)frand(seed);
                    }
                } else { /* the enclosing box (rtcommon.h:425-466) */
                    const float hd = group_box(qo, qd, RT_SMALL_F, bw, bh, bw, sub, gbase);
                    if (depth == 0) ++st_box;
                    if (hd > RT_SMALL_F && hd < kInf) {
                        const V3 hp = v3(qo.x + qd.x * hd, qo.y + qd.y * hd, qo.z + qd.z * hd);
                        const V3 hn = box_normal_signs(hp, bw, bh, bw);
                        for (uint32_t l = 0; l < nl; ++l) {
                            (void)frand(seed);
                            (void)frand(seed);
                        }
                        const float r1 = frand(seed);
                        const float r2 = frand(seed);
                        const float ct = rt_sqrtf(1.0f - r1);
                        const float st = rt_sqrtf(1.0f - ct * ct);
                        const float phi = RT_M_2PI_F * r2;
                        float sphi, cphi;
                        rt_sincosf(phi, &sphi, &cphi);
                        qd = shading_to_world(v3(cphi * st, sphi * st, ct), hn);
                        qo = hp;
                        ++depth;
                        if (depth <= a.max_depth) {
                            sample_done = false;
                            start = true;
                        }
                    }
                }
                if (sample_done) {
                    if (!RUNS && a.split_hit_depth && lane == gbase) /* (not the repair pass: NULL there) */
                        a.split_hit_depth[(size_t)pslot * spp + sample] = ghit ? (uint8_t)depth : (uint8_t)0xffu;
                    ++sample;
                    next = true;
                }
            }
            bool run_on = false;
            if (RUNS && next && a.split_restart && sample < spp && lpack != RT_LPACK_NONE &&
                lpack != RT_LPACK_EMPTY) {
                /* the repair pass (a speculated pixel's chain): a run of up to G - 1 samples at once,
                   one per lane, each from the seed it has if every earlier sample of the run hit the
                   mesh (split_spec_draws numbers each, rtcommon.h:411-421), its camera ray tested
                   against the pixel's candidate list; the chain takes the run up to its first miss */
                const uint32_t D = a.split_spec_draws, rem = spp - sample;
                const uint32_t runmax = rem < (uint32_t)(G - 1) ? rem : (uint32_t)(G - 1);
                /* frand's state stepped sub x D draws on (rng.h:24-42): one multiplication by the
                   jump multiplier of the lane (mwc_jump) */
                Seed sl;
                sl.x = mwc_jump<36969u>(seed.x, (uint32_t)sub * D, a.split_run_mul[2 * sub]);
                sl.y = mwc_jump<18000u>(seed.y, (uint32_t)sub * D, a.split_run_mul[2 * sub + 1]);
                bool hit = false;
                if ((uint32_t)sub < runmax) {
                    const uint32_t s = sample + (uint32_t)sub;
                    Seed sc = sl;
                    const uint32_t sx = s / a.sample_rate, sy = s % a.sample_rate;
                    const float fa = (float)x + strat_rand(sc, (int)sx, (int)a.sample_rate);
                    const uint32_t y = global_row(a, yl);
                    const float fb = (float)y + strat_rand(sc, (int)sy, (int)a.sample_rate);
                    const V3 o = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
                    const V3 dd = camera_dir(a.cam, fa - hw, fb - hh);
                    const uint32_t pc = (lpack & (RT_LIST_MAX - 1u)) + 1u, first = (lpack >> RT_LIST_BITS) << 3;
                    for (uint32_t t = 0; t < pc && !hit; ++t) {
                        const uint32_t r = first + t;
                        float tt = 0.0f;
                        const bool h = mt_test(o, dd, tris[3 * r], tris[3 * r + 1], tris[3 * r + 2], tt);
                        hit = h && !(tt < RT_SMALL_F) && tt <= kInf; /* the closest-hit acceptance */
                    }
                }
                /* the run's hits before its first miss (64-bit: a group may be the whole wave; lane
                   runmax <= G - 1 never hits, so ~hm has a set bit) */
                const unsigned long long hm = (__ballot(hit) & gmask) >> gbase;
                uint32_t m = (uint32_t)__builtin_ctzll(~hm);
                if (m > runmax) { /* a defect: reported (rt_synchronize fails the render), the run taken as ended */
                    if (lane == gbase) atomicOr(guard, (unsigned long long)RT_GUARD_INDEX);
                    m = runmax;
                }
                if ((uint32_t)sub < m && (sample + (uint32_t)sub) % fine == 0u)
                    reinterpret_cast<uint2 *>(a.split_seed)[(size_t)pslot * nseed + (sample + (uint32_t)sub) / fine] =
                        make_uint2(sl.x, sl.y);
                seed.x = (uint32_t)__shfl((int)sl.x, gbase + (int)m);
                seed.y = (uint32_t)__shfl((int)sl.y, gbase + (int)m);
                sample += m;
                /* a whole run of hits: the next run in the next pass; else the missed sample (or the
                   chain's end) goes on below */
                run_on = m == runmax && sample < spp;
            }
            if (next && !run_on) {
                next = false;
                if ((sample == spp || sample % fine == 0u) && lane == gbase) {
                    const uint32_t c = sample == spp ? nseed - 1u : sample / fine;
                    reinterpret_cast<uint2 *>(a.split_seed)[(size_t)pslot * nseed + c] = make_uint2(seed.x, seed.y);
                }
                if (sample == spp) {
                    have = false;
                    if (a.pixel_stats && lane == gbase) {
                        uint32_t *ps = a.pixel_stats + 8 * ((size_t)yl * a.W + x);
                        ps[0] = st_t0;
                        ps[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        ps[2] = st_steps;
                        ps[3] = st_box;
                        ps[4] = 1u + (uint32_t)RT_SPLIT_BOX;
                    }
                } else {
                    /* strat_rand twice (rng.h:45-47): the two draws, then the divisions on two lanes */
                    const float f1 = frand(seed), f2 = frand(seed);
                    const uint32_t sx = sample / a.sample_rate, sy = sample % a.sample_rate;
                    const float num = (float)(sub & 1 ? sy : sx) + (sub & 1 ? f2 : f1);
                    const float qv = num / (float)a.sample_rate;
                    const float ua = __shfl(qv, gbase), ub = __shfl(qv, gbase + 1);
                    const float fa = (float)x + ua;
                    const uint32_t y = global_row(a, yl);
                    const float fb = (float)y + ub;
                    qo = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
                    qd = group_camera_dir(a.cam, fa - hw, fb - hh, sub, gbase);
                    depth = 0;
                    start = true;
                }
            }
            if (start) {
                trav_begin(ts, stk, qo, qd, kInf);
                q_steps = 0;
                running = true;
                if (depth == 0 && lpack == RT_LPACK_EMPTY) { /* no candidate: no mesh hit */
                    running = false;
                    ghit = false;
                    fin = true;
                } else if (depth == 0 && lpack != RT_LPACK_NONE) { /* the list's triangles in runs over the lanes */
                    const uint32_t pc = (lpack & (RT_LIST_MAX - 1u)) + 1u, first = (lpack >> RT_LIST_BITS) << 3;
                    const uint32_t bs = (pc + (uint32_t)G - 1u) / (uint32_t)G, s0 = (uint32_t)sub * bs;
                    live = s0 < pc;
                    const uint32_t cnt = live ? (pc - s0 < bs ? pc - s0 : bs) : 1u;
                    ts.node = ~(int)(((first + s0) << 3) | (cnt - 1u));
                } else if (!start_tree()) { /* misses every subtree's box: no mesh hit, at once */
                    running = false;
                    ghit = false;
                    fin = true;
                }
            }
            if (pass + 1 >= RT_CHAIN_IMM || !__any(next || fin)) break;
        }
        /* traversal steps: each live lane one record of its subtree; the group's query ends at
           its first accepted triangle or when no lane has a subtree left */
#pragma unroll
        for (int u = 0; u < RT_CHAIN_UNROLL; ++u) {
            bool found = false;
            if (running && live) {
                const int nd = ts.node;
                const uint32_t enc = ~(uint32_t)nd;
                const bool bad = nd < 0 ? (enc >> 3) + (enc & 7u) >= a.n_recs : (uint32_t)nd >= a.n_nodes4;
                if (bad) { /* a defect: reported (rt_synchronize fails the render), the lane ends */
                    atomicOr(guard, (unsigned long long)RT_GUARD_INDEX);
                    live = false;
                } else {
                    TravCounts tc = {0u, 0u, 0u};
                    const bool done = trav_step_q<false>(nodes, tris, ts, stk, qo, qd, RT_SMALL_F, false, tc);
                    found = ts.best >= 0;
                    if (done) live = false;
                }
            }
            const unsigned long long fb = __ballot(found), lb = __ballot(live);
            if (running) {
                ++q_steps;
                ++st_steps;
                const bool gf = (fb & gmask) != 0ull, gl = (lb & gmask) != 0ull;
                /* a query never takes 2^14 steps: a bound every wave reaches (reported) */
                if (q_steps > (1u << 14) && lane == gbase) atomicOr(guard, (unsigned long long)RT_GUARD_ROUNDS);
                if (gf || !gl || q_steps > (1u << 14)) {
                    running = false;
                    live = false;
                    fin = true;
                    ghit = gf;
                }
            }
        }
    }
}

/* ======================================================================== */
/* Triangle kernel: raytrace_tris + trace_path_tri (rtcommon.h:371-470).     */

constexpr int kMaxLights = 16;

enum : int { M_IDLE = 0, M_NEWSAMPLE = 1, M_CLOSEST = 2, M_SHADOW = 3, M_DONE = 4 };

/* Per-lane loop, one iteration:
     D  lanes whose ray query completed advance their path (trace_path_tri) and
        issue the next query, start the next sample, or write the pixel;
     A  idle lanes take the next pixels from the queue;
     B  camera ray of a new sample;
     C  ray queries.  BVH kinds: queries are resumable — newly issued queries
        start, then the wave steps every running query one node (or leaf) at a
        time until `fetch_k` lanes have completed (or none is running), so lanes
        whose query ended early go back to work instead of idling until the
        wave's longest query ends.  LINEAR: each query runs to completion inside
        the iteration (the reference loop, wave-uniform).
   SPLIT: a queue item is one chunk of a pixel's samples, started from the seed the seed pass
   (k_split_seeds) stored for it; each sample's radiance is stored for k_split_finish. */
/* path-advance passes that may answer an off-mesh box-path query in place (0 / 1 / all: bunny class
   0.484 / 0.457 / 0.594 ms, profiles/r05ag-r05ah); later ones at the stepping round's start, without a step */
constexpr int kOffMeshRedo = 1;
template <int TRAV, bool COUNT, bool SPLIT = false, bool MQ = false> /* MQ: the multi-head queue (mq_take) */
__global__ __launch_bounds__(RT_BLOCK, RT_TRIS_WAVES) void k_tris(RtTriLaunch a)
{
    constexpr bool RESUME = TRAV == RT_TRAV_BVH4 || TRAV == RT_TRAV_BVH4Q;
    __shared__ int s_stack[RT_STACK_DEPTH * RT_BLOCK];
    __shared__ float s_light[kMaxLights * 8];
    /* the pixel sum and the path throughput, touched once per sample / segment, live in LDS
       (6 floats per lane) instead of six registers across the stepping loop */
    __shared__ float s_state[6 * RT_BLOCK];
    /* the lane's pixel's candidate list (list_pack), read when it takes the pixel instead of before
       every camera ray (LDS budget: 5 blocks per CU beside the RT_STACK_DEPTH = 20-entry stack and
       the hit normal: 31,232 B per block) */
    __shared__ uint32_t s_list[RT_BLOCK];
    /* the closest hit's unnormalised normal, formed at its accept from the record in registers
       (trav_step_q), so the path advance needs no second fetch of the hit's edges */
    __shared__ float s_hn[3 * RT_BLOCK];
    lds_float *const st_hn = (lds_float *)(s_hn + threadIdx.x);
    float *const st_acc = s_state + threadIdx.x, *const st_prop = s_state + 3 * RT_BLOCK + threadIdx.x;
#define ACC_GET(k) st_acc[(k) * RT_BLOCK]
#define ACC_SET(k, v) (st_acc[(k) * RT_BLOCK] = (v))
#define PROP_GET(k) st_prop[(k) * RT_BLOCK]
#define PROP_SET(k, v) (st_prop[(k) * RT_BLOCK] = (v))

    /* emissive spheres: center.xyz, radius, emission.xyz (materials.h:232, rtcommon.h:97-99) */
    const uint32_t n_lights = a.n_lights < (uint32_t)kMaxLights ? a.n_lights : (uint32_t)kMaxLights;
    if (threadIdx.x < n_lights) {
        const rt_sphere &L = a.lights[threadIdx.x];
        float *dst = s_light + threadIdx.x * 8;
        dst[0] = L.center.x;
        dst[1] = L.center.y;
        dst[2] = L.center.z;
        dst[3] = L.radius;
        dst[4] = L.mat.emission.x;
        dst[5] = L.mat.emission.y;
        dst[6] = L.mat.emission.z;
        dst[7] = 0.0f;
    }
    __syncthreads();

    Stack stk;
    stk.init(s_stack, a.spill, a.spill_cap);
    const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(a.nodes);
    const float4 *__restrict__ tris = reinterpret_cast<const float4 *>(a.tris);
    float4 *__restrict__ out = reinterpret_cast<float4 *>(a.out);
    const uint32_t spp = a.sample_rate * a.sample_rate;
    const uint32_t plane = a.Wpad * a.Hpad;
    const uint32_t tiles_x = (a.W + 7u) >> 3;
    const uint32_t tiles_y = (a.Hl + 7u) >> 3;
    const uint32_t n_items = tiles_x * tiles_y * 64u;
    const uint32_t n_tasks =
        SPLIT ? (a.split_which == RT_SPLIT_BOX ? box_items(a) : n_items) * a.split_chunks
              : n_items;
    /* launch-uniform values pinned to SGPRs (readfirstlane), so they neither occupy nor
       spill vector registers */
    const float hw = uniform_f(((float)a.W) / 2.0f);
    const float hh = uniform_f(((float)a.H) / 2.0f);
    const float mix_t = uniform_f(a.progressive > 0 ? 1.0f / (float)a.progressive : 0.0f);
    const float bw = (float)RT_BOX_WIDTH, bh = (float)RT_BOX_HEIGHT;
    const int fetch_k_all = (int)a.fetch_k;

    int mode = M_IDLE;
    uint32_t x = 0, yl = 0; /* pixel column and local row (global row / seed slot derived) */
    Seed seed = {0u, 0u};
    float col_x = 0.0f, col_y = 0.0f, col_z = 0.0f; /* this path's radiance (trace_path_tri's pixelColor) */
    uint32_t sample = 0, depth = 0, light = 0;
    /* the query ray: a path segment (closest hit) or a shadow ray from the offset hit
       point (any hit) — one register set for both, the phases never overlap */
    V3 qo = v3(0.0f, 0.0f, 0.0f), qd = v3(0.0f, 0.0f, 1.0f);
    V3 hp = qo, hn = qo, direct = qo;
    float stmax = 0.0f;
    bool tri_hit = false;
    bool running = false; /* a resumable query is in flight */
    /* the pixel's class from the probe: -1 mesh pixel; a box pixel (long sample chain): -2, or
       its slot >= 0 among the long chains of a sample-split render */
    int pclass = -1;
    /* SPLIT over long chains with split_hit_depth: the depth of the sample's mesh hit (the closest
       queries above it meet only the box); 0 otherwise */
    int hit_depth = 0;
    bool fin = false;     /* the lane's query completed: ts.best / ts.best_t hold its result */
    TravState ts;
    ts.node = 0;
    ts.best = -1;
    ts.best_orig = -1;
    ts.best_t = kInf;
    ts.inv = qo;
    ts.oi = qo;
    unsigned long long cnt[RT_N_COUNTERS] = {};
    const unsigned long long t_k0 = COUNT ? wave_clock() : 0ull;
    /* counting launches: this pixel's start clock, queries and traversal steps */
    unsigned long long pix_t0 = 0, pix_q = 0, pix_steps = 0;
    /* counting launches with RT_PIXEL_STATS: this pixel's wall clocks by phase (path advance D,
       refill + camera ray A/B, stepping rounds C) and its loop iterations */
    unsigned long long pix_d = 0, pix_ab = 0, pix_c = 0, pix_it = 0;
    uint32_t pix_rt0 = 0; /* pixel start (s_memrealtime), RT_PIXEL_STATS diagnostics */
    uint32_t bnext = 0, bend = 0; /* the wave's batch of queue items (batch_take) */
    /* the multi-head queue (mq_take: launches of 64-item groups with batched takes) */
    const bool multi_q = MQ; /* multi-head queue: short frames' batched takes, long tasks' exact takes (batch 0)
                                and a split tile's mesh chunk tasks; never for RT_SPLIT_BOX launches */
    uint32_t qs = (blockIdx.x % RT_QHEADS) << 4;

    for (;;) {
        const unsigned long long t_d0 = (COUNT || RT_PLAIN_PIXEL_STATS) ? wave_clock() : 0ull;
        /* ---- D: advance the path (trace_path_tri, rtcommon.h:378-468) ---- */
        for (int redo_pass = 0;; ++redo_pass) {
        if (fin) {
            fin = false;
            bool want_shadow = false, seg_done = false, sample_done = false;
            if (mode == M_CLOSEST) {
                ++cnt[0];
                if (COUNT || RT_PLAIN_PIXEL_STATS) ++pix_q;
                bool surface = true;
                if (ts.best >= 0) {
                    const float qt = ts.best_t;
                    hp = v3(qo.x + qd.x * qt, qo.y + qd.y * qt, qo.z + qd.z * qt);
                    /* the unnormalised normal (rtcommon.h:389): written to LDS at the accept, the
                       same float operations on the same record (kept in registers instead it
                       measured 8 % slower, r01; a second fetch of the edges here is one more
                       dependent round trip per mesh hit) */
                    if (TRAV == RT_TRAV_BVH4Q) {
                        hn = v3(st_hn[0], st_hn[RT_BLOCK], st_hn[2 * RT_BLOCK]);
                    } else {
                        const float4 e1 = tris[3 * ts.best + 1];
                        const float4 e2 = tris[3 * ts.best + 2];
                        hn = cross3(v3(e2.x, e2.y, e2.z), v3(e1.x, e1.y, e1.z)); /* unnormalised, rtcommon.h:389 */
                    }
                    tri_hit = true;
                } else {
                    if (SPLIT && depth == 0 && a.split_spec && a.split_which == RT_SPLIT_MESH &&
                        sample / a.split_chunk + 1u < a.split_chunks) {
                        /* a speculated pixel's camera ray missed the mesh: its later chunks started
                           from wrong seeds — listed once for the repair pass, which restarts at the
                           first such chunk (rare path) */
                        const uint32_t p = yl * a.W + x;
                        if (atomicMin(a.split_dirty + p, sample / a.split_chunk) == ~0u)
                            a.split_repair[(uint32_t)atomicAdd(a.counters + RT_CNT_REPAIR, 1ull)] = p;
                    }
                    /* the enclosing box (rtcommon.h:427-433); ray.tmax is still INF */
                    const float hd = intersect_box(qo, qd, RT_SMALL_F, bw, bh, bw);
                    if (hd > RT_SMALL_F && hd < kInf) {
                        hp = v3(qo.x + qd.x * hd, qo.y + qd.y * hd, qo.z + qd.z * hd);
                        hn = box_normal(hp, bw, bh, bw);
                        tri_hit = false;
                    } else {
                        surface = false;
                        sample_done = true; /* path terminates (rtcommon.h:463-466) */
                    }
                }
                if (surface) { /* sample_direct_illumination_tri, rtcommon.h:78-105 */
                    /* the shadow-ray origin (so) becomes the query origin */
                    qo = v3(hp.x + hn.x * RT_SMALL_F, hp.y + hn.y * RT_SMALL_F, hp.z + hn.z * RT_SMALL_F);
                    direct = v3(0.0f, 0.0f, 0.0f);
                    light = 0;
                    if (n_lights > 0) want_shadow = true;
                    else seg_done = true;
                }
            } else {
                ++cnt[1];
                if (COUNT || RT_PLAIN_PIXEL_STATS) ++pix_q;
                if (ts.best < 0) { /* unoccluded: rtcommon.h:93-101 */
                    const float cw = qd.x * hn.x + qd.y * hn.y + qd.z * hn.z;
                    if (cw > 0) {
                        direct.x += s_light[light * 8 + 4] * cw;
                        direct.y += s_light[light * 8 + 5] * cw;
                        direct.z += s_light[light * 8 + 6] * cw;
                    }
                }
                ++light;
                if (light < n_lights) want_shadow = true;
                else seg_done = true;
            }
            bool bounce = false;
            if (seg_done) {
                const float scale = 1.0f * RT_M_1_PI_F;
                V3 prop = v3(PROP_GET(0), PROP_GET(1), PROP_GET(2));
                if (tri_hit) { /* rtcommon.h:411-421: no bounce off triangles */
                    col_x += prop.x * direct.x * scale * 0.7f;
                    col_y += prop.y * direct.y * scale * 0.7f;
                    col_z += prop.z * direct.z * scale * 0.7f;
                    sample_done = true;
                } else { /* rtcommon.h:435-461: albedo 0.7, Lambert bounce (drawn even at the last depth) */
                    prop.x *= 0.7f;
                    prop.y *= 0.7f;
                    prop.z *= 0.7f;
                    col_x += prop.x * direct.x * scale;
                    col_y += prop.y * direct.y * scale;
                    col_z += prop.z * direct.z * scale;
                    PROP_SET(0, prop.x);
                    PROP_SET(1, prop.y);
                    PROP_SET(2, prop.z);
                    qo = hp;
                    bounce = true;
                }
            }
            /* Next direction, light sample or Lambert bounce, through ONE code path: both
               draw r1 then r2 (rtcommon.h:92, :459), build (cos(phi) st, sin(phi) st, ct)
               with phi = 2 pi r2 and st = sqrt(1 - ct^2), and rotate it about an axis
               (shading_to_world) — sphereEmissiveRadiance (materials.h:232-271) about the
               direction to the light with ct = 1 + r1 (cos_max - 1), cos_sample_hemisphere
               (materials.h:21-35) about the normal with ct = sqrt(1 - r1).  Only ct and the
               axis differ, so lanes of both kinds share the sin/cos and the frame. */
            if (want_shadow || bounce) {
                const float r1 = frand(seed);
                const float r2 = frand(seed);
                V3 axis = hn;
                float ct = 0.0f;
                V3 lc = hn;
                float lr = 0.0f;
                if (want_shadow) {
                    lc = v3(s_light[light * 8 + 0], s_light[light * 8 + 1], s_light[light * 8 + 2]);
                    lr = s_light[light * 8 + 3];
                    V3 dir = v3(lc.x - qo.x, lc.y - qo.y, lc.z - qo.z);
                    const float inv = rt_rsqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
                    dir.x *= inv;
                    dir.y *= inv;
                    dir.z *= inv;
                    const float sin_max = lr * inv;
                    const float cos_max = rt_sqrtf(1.0f - sin_max * sin_max);
                    ct = 1.0f + r1 * (cos_max - 1.0f);
                    axis = dir;
                } else {
                    ct = rt_sqrtf(1.0f - r1);
                }
                const float st = rt_sqrtf(1.0f - ct * ct);
                const float phi = RT_M_2PI_F * r2;
                float sphi, cphi;
                rt_sincosf(phi, &sphi, &cphi);
                qd = shading_to_world(v3(cphi * st, sphi * st, ct), axis);
                if (want_shadow) {
                    stmax = intersect_sphere(qo, qd, RT_SMALL_F, lc, lr) - RT_SMALL_F;
                    mode = M_SHADOW;
                } else {
                    ++depth;
                    if (depth > a.max_depth) sample_done = true;
                    else mode = M_CLOSEST;
                }
            }
            if (SPLIT && sample_done) { /* the sample's radiance, summed in order by k_split_finish */
                hit_depth = 0; /* read per task: its first sample's */
                float *dst = a.split_col + ((size_t)sample * (a.W * a.Hl) + (yl * a.W + x)) * 3u;
                dst[0] = col_x;
                dst[1] = col_y;
                dst[2] = col_z;
                ++sample;
                mode = (sample >= spp || sample % a.split_chunk == 0u) ? M_IDLE : M_NEWSAMPLE;
                if (a.pixel_iter && mode == M_IDLE) /* the chunk task's finish */
                    a.pixel_iter[(size_t)a.W * a.Hl * a.split_chunks + (size_t)(yl * a.W + x) * a.split_chunks +
                                 (sample - 1u) / a.split_chunk] = (uint32_t)pix_steps;
                if (sample >= spp && !a.split_seed_slot) /* the pixel's final seed, from its last chunk's own draws
                                                            (a slotted long chain's: from its seed pass) */
                    reinterpret_cast<uint2 *>(a.split_seed)[(size_t)(yl * a.W + x) * a.split_nseed + a.split_nseed - 1u] =
                        make_uint2(seed.x, seed.y);
                if (mode == M_IDLE) {
                    pclass = -1;
                    if (COUNT && a.pixel_stats) { /* diagnostics: the pixel's queries and steps over its chunks */
                        uint32_t *ps = a.pixel_stats + 8 * ((size_t)yl * a.W + x);
                        atomicAdd(ps + 5, (uint32_t)pix_q);
                        atomicAdd(ps + 6, (uint32_t)pix_steps);
                    }
                }
            } else if (sample_done) {
                ACC_SET(0, ACC_GET(0) + col_x);
                ACC_SET(1, ACC_GET(1) + col_y);
                ACC_SET(2, ACC_GET(2) + col_z);
                ++sample;
                mode = M_NEWSAMPLE;
                if (sample >= spp) { /* raytracer.cl:234-242 */
                    {
                        const float n = (float)spp;
                        const float acc_x = ACC_GET(0), acc_y = ACC_GET(1), acc_z = ACC_GET(2);
                        float4 p = make_float4(acc_x / n, acc_y / n, acc_z / n, 0.0f / n);
                        float4 *dst = out + ((size_t)yl * a.W + x);
                        if (a.progressive > 0) {
                            const float4 old = *dst;
                            const float t = mix_t;
                            p.x = old.x + (p.x - old.x) * t;
                            p.y = old.y + (p.y - old.y) * t;
                            p.z = old.z + (p.z - old.z) * t;
                            p.w = old.w + (p.w - old.w) * t;
                        }
                        *dst = p;
                    }
                    const uint32_t slot = global_row(a, yl) * a.Wpad + x;
                    a.seeds[slot] = seed.x;
                    a.seeds[plane + slot] = seed.y;
                    if (a.pixel_iter) a.pixel_iter[a.W * a.Hl + yl * a.W + x] = (uint32_t)pix_steps;
                    mode = M_IDLE;
                    pclass = -1;
                    if ((COUNT || RT_PLAIN_PIXEL_STATS) && a.pixel_stats) { /* diagnostics (RT_PIXEL_STATS) */
                        uint32_t *ps = a.pixel_stats + 8 * ((size_t)yl * a.W + x);
                        ps[0] = pix_rt0;
                        ps[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        ps[2] = (COUNT || RT_PLAIN_PIXEL_STATS) ? (uint32_t)pix_q : 0u;
                        ps[3] = (COUNT || RT_PLAIN_PIXEL_STATS) ? (uint32_t)pix_steps : 0u;
                        ps[4] = (COUNT || RT_PLAIN_PIXEL_STATS) ? (uint32_t)(pix_d >> 6) : 0u;
                        ps[5] = (COUNT || RT_PLAIN_PIXEL_STATS) ? (uint32_t)(pix_ab >> 6) : 0u;
                        ps[6] = (COUNT || RT_PLAIN_PIXEL_STATS) ? (uint32_t)(pix_c >> 6) : 0u;
                        ps[7] = (COUNT || RT_PLAIN_PIXEL_STATS) ? (uint32_t)pix_it : 0u;
                    }
                    if (COUNT && !RT_DIAG_MIX && !RT_DIAG_RAYSPLIT) {
                        const unsigned long long dt = wave_clock() - pix_t0;
                        cnt[10] = dt > cnt[10] ? dt : cnt[10];
                        cnt[11] = pix_q > cnt[11] ? pix_q : cnt[11];
                        cnt[12] = pix_steps > cnt[12] ? pix_steps : cnt[12];
                    }
                }
            }
        }
        /* a shadow ray just issued whose answer is known without a traversal (the C-phase rule
           below: tmax <= tmin, or cos(wi) <= 0) is answered here and the path advanced again in
           this pass, instead of after a whole stepping round (-3.9 %, profiles/r01n) */
        const float cw_q = qd.x * hn.x + qd.y * hn.y + qd.z * hn.z;
        const bool issued = mode == M_SHADOW && !fin && !running;
        const bool need_trav = stmax > RT_SMALL_F && cw_q > 0;
        /* likewise a long chain's box segment (split_hit_depth): no triangle accepted */
        const bool known_miss = SPLIT && mode == M_CLOSEST && !fin && !running && (int)depth < hit_depth;
        /* and a box-path query (a bounce off the box, or a shadow ray leaving it) whose segment misses
           the mesh's padded bounds: no triangle accepted, whatever the traversal would visit */
        bool off_mesh = false;
        if (!SPLIT && redo_pass < kOffMeshRedo && a.mesh_bounds && !tri_hit && !fin && !running &&
            ((mode == M_SHADOW && need_trav) || (mode == M_CLOSEST && depth > 0)))
            off_mesh = segment_misses_box(qo, qd, RT_SMALL_F, mode == M_SHADOW ? stmax : kInf, a.mesh_lo, a.mesh_hi);
        const bool redo = (issued && !need_trav) || known_miss || off_mesh;
        if (!__any(redo)) break;
        if (redo) {
            ts.best = -1;
            fin = true;
            ++cnt[RT_CNT_SKIPPED];
        }
        }

        const unsigned long long t_d1 = (COUNT || RT_PLAIN_PIXEL_STATS) ? wave_clock() : 0ull;
        if (COUNT) cnt[RT_CNT_SHADE] += t_d1 - t_d0;
        if (COUNT || RT_PLAIN_PIXEL_STATS) { /* (the plain launch's phase clocks: RT_PLAIN_PIXEL_STATS builds) */
            pix_d += t_d1 - t_d0;
            ++pix_it;
        }
        /* ---- A: refill idle lanes from the pixel queue (wave-private batches: one atomic per
                64 items; bunny class 1024^2 at 1 spp 0.95 -> 0.55 ms, the dragon frame +-0.5 %) ---- */
        const unsigned long long idle = __ballot(mode == M_IDLE);
        if (idle) {
            const uint32_t item = multi_q ? mq_take(a.work_counter, n_tasks, idle, bnext, bend, qs,
                                                    a.take_exact ? 0u : a.queue_batch,
                                                    SPLIT ? 64u * a.split_chunks : 64u)
                                          : batch_take(a.work_counter, idle, bnext, bend, a.take_exact ? 0u : kBatch);
            if (mode == M_IDLE) {
                if (multi_q && item == ~0u) {
                    if ((qs >> 8) >= RT_QHEADS) mode = M_DONE; /* else: idle, takes again next iteration */
                } else if (item >= n_tasks) {
                    mode = M_DONE;
                } else {
                    /* 8 x 8 pixel tiles, row-major over the (local) frame; SPLIT over tiles: a
                       tile's chunk 0 of its 64 pixels, then chunk 1, ... (the mesh pixels only when
                       the box pixels run apart: the 16 chunk layers of a tile run side by side,
                       10 % faster than layer after layer over the frame); SPLIT over the box
                       pixels: a pixel's chunks in turn */
                    uint32_t tile = item >> 6, chunk = 0;
                    const uint32_t in = item & 63u;
                    uint32_t sbase = 0; /* the task's seeds in split_seed (x split_nseed): its pixel or its long-chain slot */
                    bool take;
                    if (SPLIT && a.split_which == RT_SPLIT_BOX) {
                        const uint32_t slot = item / a.split_chunks;
                        chunk = item - slot * a.split_chunks;
                        const uint32_t p = a.split_box[a.split_item_base + slot];
                        x = p % a.W;
                        yl = p / a.W;
                        sbase = a.split_seed_slot ? slot : p;
                        /* a repaired pixel: its chunks before the first missed one stand */
                        take = !a.split_restart || chunk * a.split_chunk >= a.split_restart[p] * a.split_restart_chunk;
                    } else {
                        if (SPLIT) {
                            chunk = tile % a.split_chunks;
                            tile = tile / a.split_chunks;
                        }
                        if (a.tile_order) tile = a.tile_order[tile];
                        x = (tile % tiles_x) * 8u + (in & 7u);
                        yl = (tile / tiles_x) * 8u + (in >> 3);
                        take = x < a.W && yl < a.Hl;
                        sbase = yl * a.W + x;
                        if (SPLIT && take && a.split_which == RT_SPLIT_MESH)
                            take = a.pixel_class[(size_t)yl * a.W + x] == -1;
                    }
                    if (RT_DIAG_ONE_PIXEL) { /* diagnostics build: the target pixel and the diag_k - 1 pixels
                                                after it in its 8 x 8 tile (in-tile order, wrapping) */
                        const uint32_t dx = a.diag_pixel % a.W, dy = a.diag_pixel / a.W;
                        const uint32_t in0 = (dy & 7u) * 8u + (dx & 7u);
                        take = take && (x >> 3) == (dx >> 3) && (yl >> 3) == (dy >> 3) && ((in - in0) & 63u) < a.diag_k;
                    }
                    if (take) s_list[threadIdx.x] = list_pack(a, x, yl, tiles_x);
                    if (SPLIT && take && a.split_spec && a.split_which == RT_SPLIT_MESH) {
                        /* a speculated mesh pixel: the chunk's first seed jumped ahead from the
                           frame seed (split_spec_draws numbers per sample before it) */
                        const uint32_t slot = global_row(a, yl) * a.Wpad + x;
                        const uint32_t k = chunk * a.split_chunk * a.split_spec_draws;
                        seed.x = mwc_jump<36969u>(a.seeds[slot], k, a.split_spec_mul[2 * chunk]);
                        seed.y = mwc_jump<18000u>(a.seeds[plane + slot], k, a.split_spec_mul[2 * chunk + 1]);
                    } else if (SPLIT && take) { /* the chunk's first seed, from the seed pass */
                        const uint2 sd = reinterpret_cast<const uint2 *>(
                            a.split_seed)[(size_t)sbase * a.split_nseed + chunk * a.split_chunk / a.split_fine];
                        seed.x = sd.x;
                        seed.y = sd.y;
                    }
                    if (SPLIT && take) {
                        if (a.pixel_iter) /* a mesh pixel's chunk task: its take (pixel_iter, whole pixels: below) */
                            a.pixel_iter[(size_t)(yl * a.W + x) * a.split_chunks + chunk] = 0u;
                        sample = chunk * a.split_chunk;
                        if (a.split_hit_depth) hit_depth = a.split_hit_depth[(size_t)sbase * spp + sample];
                        pclass = a.pixel_class ? a.pixel_class[(size_t)yl * a.W + x] : -1;
                        mode = M_NEWSAMPLE;
                        pix_q = pix_steps = 0;
                    } else if (take) {
                        const uint32_t slot = global_row(a, yl) * a.Wpad + x;
                        /* raytracer.cl:207-209: unshifted seed slot */
                        seed.x = a.seeds[slot];
                        seed.y = a.seeds[plane + slot];
                        if (a.pixel_iter) a.pixel_iter[yl * a.W + x] = 0u;
                        if ((COUNT || RT_PLAIN_PIXEL_STATS) && a.pixel_stats)
                            pix_rt0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        if (COUNT) pix_t0 = wave_clock();
                        pix_q = pix_steps = pix_d = pix_ab = pix_c = pix_it = 0;
                        ACC_SET(0, 0.0f);
                        ACC_SET(1, 0.0f);
                        ACC_SET(2, 0.0f);
                        const float acc_x = 0.0f, acc_y = 0.0f, acc_z = 0.0f;
                        sample = 0;
                        /* some of the probe's rays missed the mesh: box paths, long chains */
                        pclass = a.pixel_class ? a.pixel_class[(size_t)yl * a.W + x] : -1;
                        if (RT_DIAG_SKIP && (RT_DIAG_SKIP == 1 ? pclass != -1 : pclass == -1)) {
                            mode = M_IDLE; /* diagnostics builds: the mesh / box pixels alone (wrong frames) */
                            pclass = -1;
                        } else if (spp > 0) {
                            mode = M_NEWSAMPLE;
                        } else { /* no samples: 0/0 pixels, seeds untouched (raytracer.cl:234-242) */
                            const float n = 0.0f;
                            float4 p = make_float4(acc_x / n, acc_y / n, acc_z / n, 0.0f / n);
                            float4 *dst = out + ((size_t)yl * a.W + x);
                            if (a.progressive > 0) {
                                const float4 old = *dst;
                                const float t = mix_t;
                                p.x = old.x + (p.x - old.x) * t;
                                p.y = old.y + (p.y - old.y) * t;
                                p.z = old.z + (p.z - old.z) * t;
                                p.w = old.w + (p.w - old.w) * t;
                            }
                            *dst = p;
                        }
                    }
                }
            }
        }
        if (!__any(mode != M_DONE)) break;

        /* ---- B: camera ray of a new sample (raytracer.cl:216-224; sx outer,
                sy inner, the x draw before the y draw) ---- */
        if (mode == M_NEWSAMPLE) {
            const uint32_t sx = sample / a.sample_rate, sy = sample % a.sample_rate;
            const float fa = (float)x + strat_rand(seed, (int)sx, (int)a.sample_rate);
            const uint32_t y = global_row(a, yl);
            const float fb = (float)y + strat_rand(seed, (int)sy, (int)a.sample_rate);
            qo = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
            qd = camera_dir(a.cam, fa - hw, fb - hh);
            PROP_SET(0, 1.0f);
            PROP_SET(1, 1.0f);
            PROP_SET(2, 1.0f);
            col_x = col_y = col_z = 0.0f;
            depth = 0;
            mode = M_CLOSEST;
        }

        /* ---- C: ray queries ---- */
        /* the waves that hold box pixels (the long serial chains that end the frame) issue
           at top priority (measured against graded priorities: DESIGN.md §5); scheduling only */
        if (__any(pclass != -1)) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);
        const bool pending = (mode == M_CLOSEST || mode == M_SHADOW) && !running && !fin;
        if (RESUME) {
            if (pending) {
                const bool shadow = (mode == M_SHADOW);
                const float qt = shadow ? stmax : kInf;
                /* Shadow rays whose answer cannot change the pixel are not traversed:
                   tmax <= tmin (the sample missed the light) can hit nothing
                   (visibility_test_tri returns true), and with cos(wi) <= 0 the light's
                   term is dropped whatever the visibility (rtcommon.h:93-95 tests
                   cosWi > 0 after the visibility test; the ray is const there, and
                   both draws were already made).  Same pixel, same seeds. */
                if ((shadow && (!(qt > RT_SMALL_F) || !(qd.x * hn.x + qd.y * hn.y + qd.z * hn.z > 0))) ||
                    (SPLIT && !shadow && (int)depth < hit_depth) || /* a long chain's box segment */
                    (!SPLIT && a.mesh_bounds && !tri_hit && (shadow || depth > 0) && /* (short frames: never split) */
                     segment_misses_box(qo, qd, RT_SMALL_F, qt, a.mesh_lo, a.mesh_hi))) { /* off the mesh */
                    ts.best = -1;
                    fin = true;
                    ++cnt[RT_CNT_SKIPPED];
                } else {
                    trav_begin(ts, stk, qo, qd, qt);
                    if (shadow) ts.node = (int)a.shadow_root; /* the shadow queries' tree */
                    running = true;
                    if (!shadow && depth == 0) { /* a camera ray: the pixel's candidate list */
                        const uint32_t lpack = s_list[threadIdx.x];
                        const uint32_t pc = (lpack & (RT_LIST_MAX - 1u)) + 1u, first = (lpack >> RT_LIST_BITS) << 3;
                        if (lpack == RT_LPACK_EMPTY) {
                            running = false;
                            ts.best = -1;
                            fin = true;
                        } else if (lpack != RT_LPACK_NONE) {
                            for (uint32_t b = (pc - 1u) >> 3; b > 0u; --b) {
                                const uint32_t k = pc - 8u * b < 8u ? pc - 8u * b : 8u;
                                stk.push(~(int)(((first + 8u * b) << 3) | (k - 1u)));
                            }
                            ts.node = ~(int)((first << 3) | ((pc < 8u ? pc : 8u) - 1u));
                        }
                    }
                }
            }
            const unsigned long long t_c0 = (COUNT || RT_PLAIN_PIXEL_STATS) ? wave_clock() : 0ull;
            if (COUNT || RT_PLAIN_PIXEL_STATS) pix_ab += t_c0 - t_d1;
            /* The exit threshold follows the wave's live queries: with few lanes left (the
               frame's tail, or a small tile) a fixed fetch_k is never reached, and every lane
               would wait for the wave's longest query before its path moves on — the long
               serial chains then run at the pace of their slowest neighbours. */
            int fetch_k = fetch_k_all;
            if (a.fetch_frac) {
                const int live = __popcll(__ballot(running || fin));
                const int k_live = (live * (int)a.fetch_frac + 63) >> 6;
                fetch_k = fetch_k < k_live ? fetch_k : (k_live > 1 ? k_live : 1);
            }
            for (;;) {
                /* RT_STEP_UNROLL steps per exit check (fewer wave-level ballots and branches) */
#pragma unroll
                for (int u = 0; u < RT_STEP_UNROLL; ++u) {
#if RT_DIAG_MIX
                    if (COUNT) { /* diagnostics build: wave-steps holding node and leaf lanes / nodes only / leaves only */
                        const unsigned long long bn = __ballot(running && ts.node >= 0), bl = __ballot(running && ts.node < 0);
                        if ((threadIdx.x & 63) == 0) {
                            cnt[10] += (bn && bl) ? 1u : 0u;
                            cnt[11] += (bn && !bl) ? 1u : 0u;
                            cnt[12] += (!bn && bl) ? 1u : 0u;
                        }
                    }
#endif
                    if (running) {
                        const bool shadow = (mode == M_SHADOW);
                        TravCounts tc = {0u, 0u, 0u};
                        if (trav_step<TRAV, COUNT>(nodes, tris, ts, stk, qo, qd, RT_SMALL_F, shadow, tc,
                                                   shadow && tri_hit, st_hn)) {
                            running = false;
                            fin = true;
                        }
                        if (COUNT) {
                            cnt[2] += tc.nodes;
                            cnt[3] += tc.tests;
                            cnt[4] += tc.leaves;
                            pix_steps += tc.nodes + tc.leaves;
                            if (RT_DIAG_RAYSPLIT) {
                                const int k = shadow ? (tri_hit ? 10 : 11) : (depth == 0 ? 12 : -1);
                                if (k >= 0) cnt[k] += tc.nodes + tc.leaves;
                            }
                        } else {
                            ++pix_steps; /* (the measured cost, pixel_iter: trav_step calls) */
                        }
                    }
                    if (COUNT) ++cnt[5];
                }
                if (!__any(running)) break;
                const unsigned long long fin_lanes = __ballot(fin);
                if (__popcll(fin_lanes) >= fetch_k) break;
            }
            if (COUNT || RT_PLAIN_PIXEL_STATS) {
                const unsigned long long dc = wave_clock() - t_c0;
                if (COUNT) cnt[6] += dc;
                pix_c += dc;
            }
        } else if (pending) {
            const bool shadow = (mode == M_SHADOW);
            ts.best_t = shadow ? stmax : kInf;
            ts.best = -1;
            TravCounts tc = {0u, 0u, 0u};
            if (!shadow || ts.best_t > RT_SMALL_F)
                ts.best = traverse<TRAV, COUNT>(nodes, tris, a.n_tris, qo, qd, RT_SMALL_F, ts.best_t, shadow, stk, tc);
            fin = true;
            if (COUNT) {
                cnt[2] += tc.nodes;
                cnt[3] += tc.tests;
            }
        }
    }
    if (COUNT) cnt[7] = wave_clock() - t_k0;
    flush_counters(a.counters, cnt, COUNT);
}
#undef ACC_GET
#undef ACC_SET
#undef PROP_GET
#undef PROP_SET

/* ======================================================================== */
/* Sphere kernel: raytrace (SS = false) / raytrace_ss (SS = true)            */
/* (raytracer.cl:46-166, trace_path rtcommon.h:267-365).                     */

__device__ V3 trace_path(PathRay &r, const rt_sphere *__restrict__ sph, uint32_t n, uint32_t max_depth, Seed &seed,
                         unsigned long long &n_closest, unsigned long long &n_shadow,
                         unsigned long long &n_skipped)
{
    const float bw = (float)RT_BOX_WIDTH, bh = (float)RT_BOX_HEIGHT;
    V3 color = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t depth = 0; depth <= max_depth; ++depth) {
        ++n_closest;
        /* scene_intersection, rtcommon.h:107-121 */
        int hit = -1;
        for (uint32_t i = 0; i < n; ++i) {
            const float dd = intersect_sphere(r.o, r.d, r.tmin, v3f(sph[i].center), sph[i].radius);
            if (dd > r.tmin && dd < r.tmax) {
                hit = (int)i;
                r.tmax = dd;
            }
        }
        V3 hp, hn;
        float kd = 0.0f;
        V3 diff = v3(0.0f, 0.0f, 0.0f);
        if (hit >= 0) {
            const rt_sphere &s = sph[hit];
            hp = v3(r.o.x + r.d.x * r.tmax, r.o.y + r.d.y * r.tmax, r.o.z + r.d.z * r.tmax);
            const float inv_r = 1.0f / s.radius; /* sphereNormal, geometryFuncs.h:58-69 */
            hn = v3((hp.x - s.center.x) * inv_r, (hp.y - s.center.y) * inv_r, (hp.z - s.center.z) * inv_r);
            if (r.ext.x > 0.0f) r.prop.x *= rt_expf(rt_logf(r.ext.x) * r.tmax);
            if (r.ext.y > 0.0f) r.prop.y *= rt_expf(rt_logf(r.ext.y) * r.tmax);
            if (r.ext.z > 0.0f) r.prop.z *= rt_expf(rt_logf(r.ext.z) * r.tmax);
            if (!r.diffuse && s.mat.emission_power != 0) {
                color.x += r.prop.x * s.mat.emission.x;
                color.y += r.prop.y * s.mat.emission.y;
                color.z += r.prop.z * s.mat.emission.z;
            }
            kd = s.mat.kd;
            diff = v3f(s.mat.diffuse);
        } else {
            const float hd = intersect_box(r.o, r.d, r.tmin, bw, bh, bw);
            if (!(hd > r.tmin && hd < r.tmax)) break;
            r.tmax = hd;
            hp = v3(r.o.x + r.d.x * r.tmax, r.o.y + r.d.y * r.tmax, r.o.z + r.d.z * r.tmax);
            hn = box_normal(hp, bw, bh, bw);
        }
        /* sample_direct_illumination, rtcommon.h:148-174 (box, or kd > 0) */
        V3 direct = v3(0.0f, 0.0f, 0.0f);
        if (hit < 0 || kd > 0.0f) {
            const V3 so = v3(hp.x + hn.x * RT_SMALL_F, hp.y + hn.y * RT_SMALL_F, hp.z + hn.z * RT_SMALL_F);
            const float inv_samples = 1.0f / (float)RT_LIGHT_SAMPLES;
            for (uint32_t k = 0; k < n; ++k) {
                if (sph[k].mat.emission_power != 0) {
                    const V3 lc = v3f(sph[k].center);
                    const float lr = sph[k].radius;
                    for (int i = 0; i < (int)RT_LIGHT_SAMPLES; ++i) {
                        const float r1 = frand(seed);
                        const float r2 = strat_rand(seed, i, (int)RT_LIGHT_SAMPLES);
                        float stmax;
                        const V3 sd = sphere_light_dir(so, lc, lr, r1, r2, stmax);
                        ++n_shadow;
                        /* the light term needs cos(wi) > 0 AND visibility (rtcommon.h:160-167);
                           the const shadow ray is tested only when cos(wi) > 0 — same result */
                        const float cw = sd.x * hn.x + sd.y * hn.y + sd.z * hn.z;
                        bool vis = cw > 0; /* visibility_test, rtcommon.h:128-138 */
                        if (!vis) ++n_skipped;
                        for (uint32_t j = 0; vis && j < n; ++j) {
                            const float dd = intersect_sphere(so, sd, RT_SMALL_F, v3f(sph[j].center), sph[j].radius);
                            if (dd > RT_SMALL_F && dd < stmax) vis = false;
                        }
                        if (vis) {
                            {
                                direct.x += sph[k].mat.emission.x * cw * inv_samples;
                                direct.y += sph[k].mat.emission.y * cw * inv_samples;
                                direct.z += sph[k].mat.emission.z * cw * inv_samples;
                            }
                        }
                    }
                }
            }
        }
        if (hit >= 0) {
            if (kd > 0.0f) {
                const float scale = kd * RT_M_1_PI_F;
                color.x += r.prop.x * direct.x * diff.x * scale;
                color.y += r.prop.y * direct.y * diff.y * scale;
                color.z += r.prop.z * direct.z * diff.z * scale;
            }
            if (depth == max_depth) break;
            if (!sample_material(r, hp, hn, sph[hit].mat, seed)) break;
        } else {
            const float scale = RT_M_1_PI_F;
            r.prop.x *= 0.7f;
            r.prop.y *= 0.7f;
            r.prop.z *= 0.7f;
            color.x += r.prop.x * direct.x * scale;
            color.y += r.prop.y * direct.y * scale;
            color.z += r.prop.z * direct.z * scale;
            r.o = hp;
            r.tmin = RT_SMALL_F;
            r.tmax = kInf;
            const float r1 = frand(seed);
            const float r2 = frand(seed);
            r.d = shading_to_world(cos_sample_hemisphere(r1, r2), hn);
            r.diffuse = 1;
        }
    }
    return color;
}

template <bool SS>
#ifndef RT_SPH_TILE
#define RT_SPH_TILE 16 /* pixel tile per block, RT_SPH_TILE^2 threads (A/B: 8) */
#endif
__global__ __launch_bounds__(RT_SPH_TILE * RT_SPH_TILE) void k_spheres(RtSphLaunch a)
{
    /* RT_SPH_TILE x RT_SPH_TILE pixel tile per block; a wave covers 64 consecutive pixels of it */
    const uint32_t x = blockIdx.x * RT_SPH_TILE + (threadIdx.x % RT_SPH_TILE);
    const uint32_t yl = blockIdx.y * RT_SPH_TILE + (threadIdx.x / RT_SPH_TILE);
    unsigned long long n_closest = 0, n_shadow = 0, n_skipped = 0;
    if (x < a.W && yl < a.Hl) {
        const uint32_t y = global_row(a, yl);
        const uint32_t plane = a.Wpad * a.Hpad;
        /* get_seed (raytracer.cl:20-24): rows shifted by `progressive`; raytrace_ss unshifted */
        const uint32_t slot = SS ? (y * a.Wpad + x) : (((y + a.progressive) % a.Hpad) * a.Wpad + x);
        Seed seed = {a.seeds[slot], a.seeds[plane + slot]};
        const float hw = ((float)a.W) / 2.0f, hh = ((float)a.H) / 2.0f;
        float4 pc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (SS) {
            const float fa = (float)x + frand(seed);
            const float fb = (float)y + frand(seed);
            PathRay r;
            r.o = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
            r.d = camera_dir(a.cam, fa - hw, fb - hh);
            r.tmin = RT_SMALL_F;
            r.tmax = kInf;
            r.prop = v3(1.0f, 1.0f, 1.0f);
            r.ext = v3(0.0f, 0.0f, 0.0f);
            r.diffuse = 0;
            const V3 c = trace_path(r, a.spheres, a.n_spheres, a.max_depth, seed, n_closest, n_shadow, n_skipped);
            pc = make_float4(c.x, c.y, c.z, 0.0f);
        } else {
            const uint32_t sr = a.sample_rate;
            for (uint32_t sx = 0; sx < sr; ++sx) {
                for (uint32_t sy = 0; sy < sr; ++sy) {
                    const float fa = (float)x + strat_rand(seed, (int)sx, (int)sr);
                    const float fb = (float)y + strat_rand(seed, (int)sy, (int)sr);
                    PathRay r;
                    r.o = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
                    r.d = camera_dir(a.cam, fa - hw, fb - hh);
                    r.tmin = RT_SMALL_F;
                    r.tmax = kInf;
                    r.prop = v3(1.0f, 1.0f, 1.0f);
                    r.ext = v3(0.0f, 0.0f, 0.0f);
                    r.diffuse = 0;
                    const V3 c = trace_path(r, a.spheres, a.n_spheres, a.max_depth, seed, n_closest, n_shadow, n_skipped);
                    pc.x += c.x;
                    pc.y += c.y;
                    pc.z += c.z;
                }
            }
            const float n = (float)(sr * sr);
            pc.x /= n;
            pc.y /= n;
            pc.z /= n;
            pc.w /= n;
        }
        float4 *dst = reinterpret_cast<float4 *>(a.out) + ((size_t)yl * a.W + x);
        if (a.progressive > 0) {
            const float4 old = *dst;
            const float t = 1.0f / (float)a.progressive;
            pc.x = old.x + (pc.x - old.x) * t;
            pc.y = old.y + (pc.y - old.y) * t;
            pc.z = old.z + (pc.z - old.z) * t;
            pc.w = old.w + (pc.w - old.w) * t;
        }
        *dst = pc;
        a.seeds[slot] = seed.x;
        a.seeds[plane + slot] = seed.y;
    }
    unsigned long long cnt[RT_N_COUNTERS] = {};
    cnt[0] = n_closest;
    cnt[1] = n_shadow;
    cnt[RT_CNT_SKIPPED] = n_skipped;
    flush_counters(a.counters, cnt, false);
}

/* ======================================================================== */
/* Batch ray queries (hit-index parity).                                     */
template <int TRAV, bool COUNT>
__global__ __launch_bounds__(RT_BLOCK) void k_trace_rays(const float4 *__restrict__ nodes,
                                                         const float4 *__restrict__ tris, uint32_t n_tris,
                                                         const rt_ray *__restrict__ rays, uint32_t n, int any_hit,
                                                         int32_t *spill, uint32_t spill_cap,
                                                         int32_t *__restrict__ out_idx, float *__restrict__ out_t,
                                                         unsigned long long *__restrict__ counters)
{
    __shared__ int s_stack[RT_STACK_DEPTH * RT_BLOCK];
    const uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x;
    if (i >= n) return;
    const rt_ray r = rays[i];
    float t = r.tmax;
    TravCounts tc = {0u, 0u, 0u};
    Stack stk;
    stk.init(s_stack, spill, spill_cap);
    const int s = traverse<TRAV, COUNT>(nodes, tris, n_tris, v3f(r.o), v3f(r.d), r.tmin, t, any_hit != 0, stk, tc);
    if (COUNT) { /* counting calls (rt_set_counting): records visited, summed over the rays */
        atomicAdd(&counters[any_hit ? 1 : 0], 1ull);
        atomicAdd(&counters[2], (unsigned long long)tc.nodes);
        atomicAdd(&counters[3], (unsigned long long)tc.tests);
        atomicAdd(&counters[4], (unsigned long long)tc.leaves);
    }
    if (any_hit) {
        out_idx[i] = (s >= 0) ? 1 : 0;
        if (out_t) out_t[i] = r.tmax;
    } else {
        out_idx[i] = (s >= 0) ? __float_as_int(tris[3 * s].w) : -1;
        if (out_t) out_t[i] = t;
    }
}

/* Cost probe for the LPT pixel queue (rt_host.cpp tile_order): per pixel, an n x n grid
   (probe_n, default 2) of camera rays (the pixel's samples are stratified over its area, so silhouette pixels mix
   mesh and box paths) — each ray's closest-hit query and, when it hits the mesh, one shadow
   query per light from the hit point toward the light's centre — with the per-lane
   compressed traversal of the real kernel, counting its steps.
   out[p] = (mesh hits, 0..n^2) << RT_PROBE_HIT_SHIFT | steps of all those queries.  A persistent grid (the
   main kernel's) with grid-stride pixels, so the main kernel's traversal spill area serves
   it.  Scheduling only: no result depends on it. */
__global__ __launch_bounds__(RT_BLOCK, RT_TRIS_WAVES) void k_probe_cost(RtTriLaunch a, uint32_t *__restrict__ out)
{
    __shared__ int s_stack[RT_STACK_DEPTH * RT_BLOCK];
    Stack stk;
    stk.init(s_stack, a.spill, a.spill_cap);
    const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(a.nodes);
    const float4 *__restrict__ tris = reinterpret_cast<const float4 *>(a.tris);
    const uint32_t npx = a.W * a.Hl;
    const uint32_t stride = gridDim.x * RT_BLOCK;
    const uint32_t rounds = (npx + stride - 1) / stride; /* uniform trip count: whole waves iterate together */
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t p = r * stride + blockIdx.x * RT_BLOCK + threadIdx.x;
        const bool valid = p < npx;
        const uint32_t x = valid ? p % a.W : 0u, yl = valid ? p / a.W : 0u;
        const uint32_t y = global_row(a, yl);
        const V3 o = v3(a.cam.position.x, a.cam.position.y, a.cam.position.z);
        uint32_t steps = 0, hits = 0;
        const uint32_t pn = a.probe_n;
        const float step = 1.0f / (float)pn;
        for (uint32_t k = 0; k < pn * pn; ++k) {
            const float fx = (float)x + ((float)(k % pn) + 0.5f) * step, fy = (float)y + ((float)(k / pn) + 0.5f) * step;
            const V3 d = camera_dir(a.cam, fx - ((float)a.W) / 2.0f, fy - ((float)a.H) / 2.0f);
            TravCounts tc = {0u, 0u, 0u};
            float t = kInf;
            const int hit = traverse<RT_TRAV_BVH4Q, true>(nodes, tris, a.n_tris, o, d, RT_SMALL_F, t, false, stk, tc);
            steps += tc.nodes + tc.leaves;
            if (hit < 0) continue;
            ++hits;
            const float4 e1 = tris[3 * hit + 1], e2 = tris[3 * hit + 2];
            const V3 hn = cross3(v3(e2.x, e2.y, e2.z), v3(e1.x, e1.y, e1.z));
            const V3 so = v3(o.x + d.x * t + hn.x * RT_SMALL_F, o.y + d.y * t + hn.y * RT_SMALL_F,
                             o.z + d.z * t + hn.z * RT_SMALL_F);
            for (uint32_t l = 0; l < a.n_lights; ++l) {
                const rt_sphere &L = a.lights[l];
                const V3 lc = v3(L.center.x, L.center.y, L.center.z);
                V3 sd = v3(lc.x - so.x, lc.y - so.y, lc.z - so.z);
                const float il = rt_rsqrtf(sd.x * sd.x + sd.y * sd.y + sd.z * sd.z);
                sd = v3(sd.x * il, sd.y * il, sd.z * il);
                float st = intersect_sphere(so, sd, RT_SMALL_F, lc, L.radius) - RT_SMALL_F;
                if (st > RT_SMALL_F && sd.x * hn.x + sd.y * hn.y + sd.z * hn.z > 0.0f) {
                    TravCounts ts = {0u, 0u, 0u};
                    (void)traverse<RT_TRAV_BVH4Q, true>(nodes, tris, a.n_tris, so, sd, RT_SMALL_F, st, true, stk, ts);
                    steps += ts.nodes + ts.leaves;
                }
            }
        }
        if (valid) out[p] = (hits << RT_PROBE_HIT_SHIFT) | (steps < RT_PROBE_STEP_MASK ? steps : RT_PROBE_STEP_MASK);
    }
}

template <int G>
__global__ __launch_bounds__(RT_BLOCK, RT_TRIS_WAVES) void k_split_seeds(RtTriLaunch a)
{
    __shared__ int s_stack[RT_STACK_DEPTH * RT_BLOCK];
    seed_pass<G>(a, s_stack);
}

/* Sample-split tiles, step 3 (per part: the long chains after their chunks on the second stream,
   the clean mesh pixels after theirs on a third, the repaired after the repair pass): per pixel,
   the samples' radiance summed in sample order
   (raytracer.cl:228-230: the same additions on the same values as one lane's loop), the
   pixel written (:234-240) and its final seed (:241-242). */
__global__ __launch_bounds__(RT_BLOCK) void k_split_finish(RtTriLaunch a)
{
    const uint32_t npx = a.W * a.Hl;
    /* every pixel, or the clean mesh pixels (RT_FIN_MESH), over a grid-stride loop */
    const uint32_t n = npx;
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < n; i += gridDim.x * RT_BLOCK) {
        const uint32_t p = i;
        if (p >= npx) continue;
        if (a.finish_part == RT_FIN_MESH && (a.pixel_class[p] >= 0 || (a.split_dirty && a.split_dirty[p] != ~0u)))
            continue; /* the mesh pixels no chunk of which missed */
        const uint32_t spp = a.sample_rate * a.sample_rate;
        float acc_x = 0.0f, acc_y = 0.0f, acc_z = 0.0f;
        /* 16 samples' loads issued together, then added in sample order (a part's few pixels are
           latency-bound: one load per add would wait out each) */
        for (uint32_t s0 = 0; s0 < spp; s0 += 16u) {
            float v[48];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t s = s0 + (uint32_t)j < spp ? s0 + (uint32_t)j : spp - 1u;
                const float *c = a.split_col + ((size_t)s * npx + p) * 3u;
                v[3 * j] = c[0];
                v[3 * j + 1] = c[1];
                v[3 * j + 2] = c[2];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (s0 + (uint32_t)j < spp) {
                    acc_x += v[3 * j];
                    acc_y += v[3 * j + 1];
                    acc_z += v[3 * j + 2];
                }
            }
        }
        const float nf = (float)spp;
        float4 px = make_float4(acc_x / nf, acc_y / nf, acc_z / nf, 0.0f / nf);
        float4 *dst = reinterpret_cast<float4 *>(a.out) + p;
        if (a.progressive > 0) {
            const float4 old = *dst;
            const float t = 1.0f / (float)a.progressive;
            px.x = old.x + (px.x - old.x) * t;
            px.y = old.y + (px.y - old.y) * t;
            px.z = old.z + (px.z - old.z) * t;
            px.w = old.w + (px.w - old.w) * t;
        }
        *dst = px;
        const uint32_t x = p % a.W, yl = p / a.W;
        const uint32_t slot = global_row(a, yl) * a.Wpad + x;
        const uint2 sd = reinterpret_cast<const uint2 *>(a.split_seed)[(size_t)p * a.split_nseed + a.split_nseed - 1u];
        a.seeds[slot] = sd.x;
        a.seeds[a.Wpad * a.Hpad + slot] = sd.y;
    }
}

/* The in-order sums of a part's listed pixels (the long chains, the repaired): a wave per pixel —
   its lanes load the samples together (4 each per 256), then the wave adds them in sample order
   through readlane, the same additions as k_split_finish's loop.  A part is a few thousand pixels
   at most, latency-bound when one lane walks a pixel's samples. */
__global__ __launch_bounds__(RT_BLOCK) void k_split_finish_list(RtTriLaunch a)
{
    const uint32_t npx = a.W * a.Hl, lane = threadIdx.x & 63u;
    const uint32_t n = box_items(a);
    const uint32_t spp = a.sample_rate * a.sample_rate;
    for (uint32_t i = blockIdx.x * (RT_BLOCK / 64u) + (threadIdx.x >> 6); i < n; i += gridDim.x * (RT_BLOCK / 64u)) {
        const uint32_t p = a.split_box[a.split_item_base + i];
        if (p >= npx) continue;
        float acc_x = 0.0f, acc_y = 0.0f, acc_z = 0.0f;
        for (uint32_t b = 0; b < spp; b += 256u) {
            float v[12];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t s = b + lane * 4u + (uint32_t)j;
                const float *c = a.split_col + ((size_t)(s < spp ? s : 0u) * npx + p) * 3u;
                v[3 * j] = c[0];
                v[3 * j + 1] = c[1];
                v[3 * j + 2] = c[2];
            }
            const uint32_t lanes = (spp - b + 3u) / 4u < 64u ? (spp - b + 3u) / 4u : 64u;
            for (uint32_t l = 0; l < lanes; ++l) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (b + l * 4u + (uint32_t)j < spp) {
                        acc_x += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[3 * j]), (int)l));
                        acc_y += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[3 * j + 1]), (int)l));
                        acc_z += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[3 * j + 2]), (int)l));
                    }
                }
            }
        }
        if (lane != 0u) continue;
        const float nf = (float)spp;
        float4 px = make_float4(acc_x / nf, acc_y / nf, acc_z / nf, 0.0f / nf);
        float4 *dst = reinterpret_cast<float4 *>(a.out) + p;
        if (a.progressive > 0) {
            const float4 old = *dst;
            const float t = 1.0f / (float)a.progressive;
            px.x = old.x + (px.x - old.x) * t;
            px.y = old.y + (px.y - old.y) * t;
            px.z = old.z + (px.z - old.z) * t;
            px.w = old.w + (px.w - old.w) * t;
        }
        *dst = px;
        const uint32_t x = p % a.W, yl = p / a.W;
        const uint32_t slot = global_row(a, yl) * a.Wpad + x;
        const uint2 sd = reinterpret_cast<const uint2 *>(a.split_seed)[(size_t)(a.split_seed_slot ? i : p) * a.split_nseed + a.split_nseed - 1u];
        a.seeds[slot] = sd.x;
        a.seeds[a.Wpad * a.Hpad + slot] = sd.y;
    }
}


/* Camera-ray candidate lists.  A pixel's sampleRate^2 camera rays share the camera position
   and leave through the pixel's square (strat_rand offsets in [0, 1], raytracer.cl:216-224), so
   one conservative traversal of that narrow frustum finds every triangle any of them could
   accept: directions bounded component-wise by the four corner rays (camera_dir, the kernel's
   own arithmetic) padded by 1e-5; boxes tested with interval slabs in binary64 (per axis the
   earliest entry and latest exit over the direction interval — a necessary condition for a
   hit); nodes whose normal box keeps |d . N| below the determinant threshold for every
   direction skipped (rt_quant.h); triangles kept if their padded box (the builder's pad) meets
   the frustum and some direction could give |det| >= 1e-4 (with det's float error).  Up to
   RT_LIST_MAX survivors are copied into the pixel's list slots; k_tris then answers each camera
   query by testing only them (a virtual leaf: the same tests and accept rule on the same
   records, so the same closest hit), and an empty list answers "no mesh hit" outright.  Pixels
   with more candidates (or a stack overflow) keep the BVH. */
struct Frustum {
    double o[3];           /* the rays' origin (the camera) */
    double dlo[3], dhi[3]; /* their directions (component-wise interval) */
    double ilo[3], ihi[3]; /* 1 / dlo, 1 / dhi */
    double l1;             /* max |d|_1 */
    /* the pixel in the camera's own coordinates: P - o = s0 view + s1 right + s2 up (minv: that
       basis inverted), a ray of the pixel through P has a = s1 / s0 in [a0, a1], b = s2 / s0 in
       [b0, b1] (pixel_square); proj false: no such test */
    double minv[9];
    double a0, a1, b0, b1;
    bool proj;
};

/* The pixel's square in the camera's (a, b) coordinates, padded for the float evaluation of
   camera_dir: its rays are o + t (view + right a + up b) exactly for a in [ax, ax + 1], b in
   [by, by + 1] (the strat_rand offsets, raytracer.cl:216-224; the subtraction of W / 2 is exact),
   and the float direction strays from that ray by a few ulp of |view| + |right a| + |up b|,
   which moves (a, b) by that over |right| or |up| plus (|a| + |b|) times it over |view|: the pad
   covers it 20 times over. */
__device__ __forceinline__ void pixel_square(Frustum &f, const rt_camera &cam, float ax, float by)
{
    const double c[3][3] = {{cam.view.x, cam.right.x, cam.up.x}, {cam.view.y, cam.right.y, cam.up.y},
                            {cam.view.z, cam.right.z, cam.up.z}};
    const double det = c[0][0] * (c[1][1] * c[2][2] - c[1][2] * c[2][1]) - c[0][1] * (c[1][0] * c[2][2] - c[1][2] * c[2][0]) +
                       c[0][2] * (c[1][0] * c[2][1] - c[1][1] * c[2][0]);
    const double nv = sqrt(c[0][0] * c[0][0] + c[1][0] * c[1][0] + c[2][0] * c[2][0]);
    const double nr = sqrt(c[0][1] * c[0][1] + c[1][1] * c[1][1] + c[2][1] * c[2][1]);
    const double nu = sqrt(c[0][2] * c[0][2] + c[1][2] * c[1][2] + c[2][2] * c[2][2]);
    f.proj = fabs(det) > 1e-6 * nv * nr * nu && fmin(nr, nu) > 0.0 &&
             (double)cam.view.w == 0.0 && (double)cam.right.w == 0.0 && (double)cam.up.w == 0.0;
    if (!f.proj) return;
    const double id = 1.0 / det;
    f.minv[0] = (c[1][1] * c[2][2] - c[1][2] * c[2][1]) * id;
    f.minv[1] = (c[0][2] * c[2][1] - c[0][1] * c[2][2]) * id;
    f.minv[2] = (c[0][1] * c[1][2] - c[0][2] * c[1][1]) * id;
    f.minv[3] = (c[1][2] * c[2][0] - c[1][0] * c[2][2]) * id;
    f.minv[4] = (c[0][0] * c[2][2] - c[0][2] * c[2][0]) * id;
    f.minv[5] = (c[0][2] * c[1][0] - c[0][0] * c[1][2]) * id;
    f.minv[6] = (c[1][0] * c[2][1] - c[1][1] * c[2][0]) * id;
    f.minv[7] = (c[0][1] * c[2][0] - c[0][0] * c[2][1]) * id;
    f.minv[8] = (c[0][0] * c[1][1] - c[0][1] * c[1][0]) * id;
    const double mag = nv + nr * (fabs((double)ax) + 1.0) + nu * (fabs((double)by) + 1.0);
    const double pad = 0.01 + 64.0 * 0x1p-24 * mag * (1.0 / fmin(nr, nu) + (fabs((double)ax) + fabs((double)by) + 2.0) / nv);
    f.a0 = (double)ax - pad;
    f.a1 = (double)ax + 1.0 + pad;
    f.b0 = (double)by - pad;
    f.b1 = (double)by + 1.0 + pad;
}

/* Can a camera ray of the pixel meet the triangle v0 + u e1 + v e2 (the record's float values, as
   mt_test reads them) where the float test could accept?  The triangle is widened to u, v >= -eps,
   u + v <= 1 + 2 eps, eps bounding the float test's barycentric error (a few ulp of |e| |o - v0|
   and |e1| |e2| over |det| >= 1e-4, 7x margin), projected through the camera onto the pixel's
   (a, b) plane, and tested against the padded square by separating axes (the square's two and the
   triangle's three edge normals).  A vertex at or behind the camera's plane keeps the triangle.
   Culling only; false means no ray of the pixel can accept it. */
__device__ __forceinline__ bool tri_meets_pixel(const Frustum &f, float4 r0, float4 r1, float4 r2, double dist)
{
    if (!f.proj) return true;
    const double e1[3] = {r1.x, r1.y, r1.z}, e2[3] = {r2.x, r2.y, r2.z};
    const double n1 = fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2]), n2 = fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2]);
    const double eps = 8.0 * 16.0 * 0x1p-24 * ((n1 + n2) * dist + n1 * n2) / 1e-4 + 1e-6;
    const double uv[3][2] = {{-eps, -eps}, {1.0 + 3.0 * eps, -eps}, {-eps, 1.0 + 3.0 * eps}};
    double pa[3], pb[3];
    for (int i = 0; i < 3; ++i) {
        double q[3];
        for (int k = 0; k < 3; ++k)
            q[k] = ((double)(k == 0 ? r0.x : k == 1 ? r0.y : r0.z) + uv[i][0] * e1[k] + uv[i][1] * e2[k]) - f.o[k];
        const double s0 = f.minv[0] * q[0] + f.minv[1] * q[1] + f.minv[2] * q[2];
        const double s1 = f.minv[3] * q[0] + f.minv[4] * q[1] + f.minv[5] * q[2];
        const double s2 = f.minv[6] * q[0] + f.minv[7] * q[1] + f.minv[8] * q[2];
        if (!(s0 > 1e-9 * (fabs(s1) + fabs(s2) + fabs(s0)))) return true; /* at or behind the camera's plane */
        pa[i] = s1 / s0;
        pb[i] = s2 / s0;
    }
    if (fmax(pa[0], fmax(pa[1], pa[2])) < f.a0 || fmin(pa[0], fmin(pa[1], pa[2])) > f.a1) return false;
    if (fmax(pb[0], fmax(pb[1], pb[2])) < f.b0 || fmin(pb[0], fmin(pb[1], pb[2])) > f.b1) return false;
    const double cx[4] = {f.a0, f.a1, f.a0, f.a1}, cy[4] = {f.b0, f.b0, f.b1, f.b1};
    for (int i = 0; i < 3; ++i) {
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        double nx = -(pb[j] - pb[i]), ny = pa[j] - pa[i];
        if (nx * (pa[k] - pa[i]) + ny * (pb[k] - pb[i]) < 0.0) {
            nx = -nx;
            ny = -ny;
        }
        bool out = true;
        for (int q = 0; q < 4 && out; ++q) out = nx * (cx[q] - pa[i]) + ny * (cy[q] - pb[i]) < 0.0;
        if (out) return false;
    }
    return true;
}

__device__ __forceinline__ void frustum_init(Frustum &f)
{
    f.l1 = 0.0;
    for (int k = 0; k < 3; ++k) {
        f.ilo[k] = 1.0 / f.dlo[k];
        f.ihi[k] = 1.0 / f.dhi[k];
        f.l1 += fmax(fabs(f.dlo[k]), fabs(f.dhi[k]));
    }
}

__device__ __forceinline__ bool frustum_slab(const Frustum &f, const double lo[3], const double hi[3],
                                             double *tin_out = nullptr)
{
    /* rays o + t d with d in [dlo, dhi]: per axis (P - o) / d is monotonic in d (of one sign), so
       its range is spanned by the two end quotients (as products with the reciprocals: a
       relative 1e-16 against boxes padded by 1e-6 and more) */
    double tin = -1e300, tout = 1e300;
    for (int k = 0; k < 3; ++k) {
        const double a = f.dlo[k], b = f.dhi[k], o = f.o[k];
        if (!(a > 0.0 || b < 0.0)) {
            /* d straddles 0 on this axis: at t >= 0 the rays' coordinate spans
               [o + t a, o + t b], which must reach [lo, hi] (a lower bound on t) */
            if (a < 0.0) tin = fmax(tin, (hi[k] - o) * f.ilo[k]);
            else if (o > hi[k]) return false;
            if (b > 0.0) tin = fmax(tin, (lo[k] - o) * f.ihi[k]);
            else if (o < lo[k]) return false;
            continue;
        }
        const double ne = (a > 0.0 ? lo[k] : hi[k]) - o, fa = (a > 0.0 ? hi[k] : lo[k]) - o;
        const double ia = f.ilo[k], ib = f.ihi[k];
        tin = fmax(tin, fmin(ne * ia, ne * ib));
        tout = fmin(tout, fmax(fa * ia, fa * ib));
    }
    tin = fmax(tin, -1e-3); /* accepted hits have t > tmin > 0 */
    if (tin_out) *tin_out = tin;
    return tin <= tout;
}

/* max over the direction box of |d . n| for n in [nlo, nhi] */
__device__ __forceinline__ double frustum_det(const double dlo[3], const double dhi[3], const double nlo[3],
                                              const double nhi[3])
{
    double mx = 0.0, mn = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double c0 = dlo[k] * nlo[k], c1 = dlo[k] * nhi[k], c2 = dhi[k] * nlo[k], c3 = dhi[k] * nhi[k];
        mx += fmax(fmax(c0, c1), fmax(c2, c3));
        mn += fmin(fmin(c0, c1), fmin(c2, c3));
    }
    return fmax(mx, -mn);
}

/* The builder's padded triangle box (rt_bvh.cpp: extent / 512 + 1e-6 (1 + |coord|), doubled
   here), from a record's vertices, and the largest |N| component of its normal e2 x e1. */
__device__ __forceinline__ void tri_padded_box(float4 r0, float4 r1, float4 r2, double lo[3], double hi[3],
                                               double &nmax)
{
    const float vx[3] = {r0.x, r0.x + r1.x, r0.x + r2.x}, vy[3] = {r0.y, r0.y + r1.y, r0.y + r2.y},
                vz[3] = {r0.z, r0.z + r1.z, r0.z + r2.z};
    const float *vv[3] = {vx, vy, vz};
    float bl[3], bh[3], mabs = 0.0f;
    for (int q = 0; q < 3; ++q) {
        bl[q] = fminf(vv[q][0], fminf(vv[q][1], vv[q][2]));
        bh[q] = fmaxf(vv[q][0], fmaxf(vv[q][1], vv[q][2]));
        mabs = fmaxf(mabs, fmaxf(fabsf(bl[q]), fabsf(bh[q])));
    }
    const float ext = fmaxf(bh[0] - bl[0], fmaxf(bh[1] - bl[1], bh[2] - bl[2]));
    const double pad = 2.0 * ((double)ext * (1.0 / 512.0) + 1e-6 * (1.0 + mabs));
    for (int q = 0; q < 3; ++q) {
        lo[q] = bl[q] - pad;
        hi[q] = bh[q] + pad;
    }
    const double e1[3] = {r1.x, r1.y, r1.z}, e2[3] = {r2.x, r2.y, r2.z};
    nmax = fmax(fabs(e2[1] * e1[2] - e2[2] * e1[1]),
                fmax(fabs(e2[2] * e1[0] - e2[0] * e1[2]), fabs(e2[0] * e1[1] - e2[1] * e1[0])));
}

/* the pre-pass's per-lane traversal stack, in LDS (it was 256 B of scratch per lane): 48 entries
   cover a 4-wide tree of depth 15 (the dragon needs 35); deeper, the pixel takes the tree */
constexpr int kFrustumStack = 48;

__device__ bool frustum_list(const float *__restrict__ nodes4, const uint32_t *__restrict__ q4,
                             const float4 *__restrict__ tris, const Frustum &f, int *slots, float *keys, uint32_t cap,
                             uint32_t &n, lds_int *stack);

/* The component-wise box of the unit directions normalize(view + right a + up b) over a pixel's
   square a in [ax, ax + 1], b in [by, by + 1] (strat_rand offsets, raytracer.cl:216-224).  The
   four corner rays (camera_dir, the kernel's own float arithmetic) span it only up to the
   curvature of the normalisation: an interior direction leaves the corners' box by about
   1 / (8 L^2), L = (W / 2) / tan(fov / 2) (2e-5 at W = 64).  Bound: d = v / |v| has
   |D^2 d[w, w]| <= 6 |w|^2 / |v|^2, and a C^2 function on the unit square differs from the
   bilinear interpolation of its corners (whose range is the corners' box) by at most
   (1/8)(max |d_aa| + max |d_bb|) = 0.75 (|right|^2 + |up|^2) / min|v|^2, with min|v| over the
   square at least the smallest corner |v| less |right| + |up|.  The pad on top covers the
   float evaluation of camera_dir (a few ulp of a unit vector). */
__device__ __forceinline__ void pixel_dir_box(const rt_camera &cam, float ax, float by, double dlo[3], double dhi[3])
{
    double nmin = 1e300;
    for (int k = 0; k < 3; ++k) {
        dlo[k] = 1e300;
        dhi[k] = -1e300;
    }
    for (int c = 0; c < 4; ++c) {
        const float a = ax + (float)(c & 1), b = by + (float)(c >> 1);
        const V3 d = camera_dir(cam, a, b);
        const double dv[3] = {d.x, d.y, d.z};
        for (int k = 0; k < 3; ++k) {
            dlo[k] = fmin(dlo[k], dv[k]);
            dhi[k] = fmax(dhi[k], dv[k]);
        }
        const double vx = (double)cam.view.x + (double)cam.right.x * a + (double)cam.up.x * b;
        const double vy = (double)cam.view.y + (double)cam.right.y * a + (double)cam.up.y * b;
        const double vz = (double)cam.view.z + (double)cam.right.z * a + (double)cam.up.z * b;
        nmin = fmin(nmin, sqrt(vx * vx + vy * vy + vz * vz));
    }
    const double r2 = (double)cam.right.x * cam.right.x + (double)cam.right.y * cam.right.y +
                      (double)cam.right.z * cam.right.z;
    const double u2 = (double)cam.up.x * cam.up.x + (double)cam.up.y * cam.up.y + (double)cam.up.z * cam.up.z;
    nmin -= sqrt(r2) + sqrt(u2);
    const double bulge = nmin > 1e-3 ? 0.75 * (r2 + u2) / (nmin * nmin) : 2.0; /* 2: the whole direction range */
    const double pad = 1e-5 + bulge;
    for (int k = 0; k < 3; ++k) {
        dlo[k] -= pad;
        dhi[k] += pad;
    }
}

__global__ __launch_bounds__(RT_BLOCK) void k_pixel_lists(RtTriLaunch a, const float *__restrict__ nodes4,
                                                          const uint32_t *__restrict__ q4, uint16_t *__restrict__ codes,
                                                          uint32_t *__restrict__ tile_base)
{
    /* one wave per 8 x 8 pixel tile: neighbouring frusta walk the same nodes */
    __shared__ int s_fstack[kFrustumStack * RT_BLOCK];
    const uint32_t item = blockIdx.x * RT_BLOCK + threadIdx.x, tiles_x = (a.W + 7u) / 8u;
    const uint32_t tile = item >> 6, in = item & 63u;
    const uint32_t x = (tile % tiles_x) * 8u + (in & 7u), yl = (tile / tiles_x) * 8u + (in >> 3);
    const bool valid = x < a.W && yl < a.Hl;
    const uint32_t p = yl * a.W + x;
    const float4 *__restrict__ tris = reinterpret_cast<const float4 *>(a.tris);
    int slot[RT_LIST_MAX];
    float key[RT_LIST_MAX];
    uint32_t n = 0;
    bool ok = false;
    if (valid) {
        const uint32_t y = global_row(a, yl);
        /* a = fa - W/2 with fa in [x, x + 1] (the kernel's float subtraction, exact at these
           magnitudes), likewise b */
        const float ax = (float)x - ((float)a.W) / 2.0f, by = (float)y - ((float)a.H) / 2.0f;
        Frustum f;
        pixel_dir_box(a.cam, ax, by, f.dlo, f.dhi);
        pixel_square(f, a.cam, ax, by);
        for (int k = 0; k < 3; ++k) f.o[k] = k == 0 ? a.cam.position.x : k == 1 ? a.cam.position.y : a.cam.position.z;
        frustum_init(f);
        ok = frustum_list(nodes4, q4, tris, f, slot, key, RT_LIST_MAX, n, (lds_int *)(s_fstack + threadIdx.x));
    }
    /* The tile's lists are one block of the list area (one atomic per wave), in lane order, each
       list starting on a 128-B line (a multiple of 8 records of 48 B; the area's base is one too):
       the first records of a list — most camera queries read one to three — then share lines
       (r02's fixed 32-slot layout had that by accident: it read 0.45G fewer lines per frame than
       lists at arbitrary offsets) */
    const uint32_t want = ok ? (n + 7u) & ~7u : 0u;
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t incl = want;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
    }
    const uint32_t total = __shfl(incl, 63);
    uint32_t base = 0;
    if (lane == 0 && total) base = atomicAdd(a.list_alloc, total);
    base = __shfl(base, 0);
    /* no room left in the list area: the tile's camera rays take the tree (wave-uniform) */
    if ((uint64_t)base + total > a.list_cap) ok = false;
    const uint32_t n_tiles = tiles_x * ((a.Hl + 7u) / 8u);
    if (lane == 0 && tile < n_tiles) tile_base[tile] = a.list_base + base;
    if (!valid) return;
    const uint32_t rel = incl - want; /* < 64 * RT_LIST_MAX, a multiple of 8 */
    codes[p] = (uint16_t)(!ok ? RT_LIST_NONE : n == 0 ? RT_LIST_EMPTY : ((rel >> 3) << RT_LIST_BITS) | (n - 1u));
    if (!ok || n == 0) return;
    float4 *__restrict__ lst = const_cast<float4 *>(tris) + 3ull * (a.list_base + (size_t)base + rel);
    /* The records in order of their earliest accept t, each one's r1.w carrying the NEXT
       record's bound (+inf on the last): a closest-hit query whose best t is already below
       it has its answer (trav_step_q ends the list there — the accept rule needs t < best_t,
       or t == best_t). */
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t r = 0;
        float next = kInf;
        for (uint32_t j = 0; j < n; ++j) {
            const bool before = key[j] < key[i] || (key[j] == key[i] && j < i);
            r += before ? 1u : 0u;
            if (!before && j != i) next = fminf(next, key[j]);
        }
        const int s = slot[i];
        const float4 e1 = tris[3 * s + 1];
        lst[3 * r] = tris[3 * s];
        lst[3 * r + 1] = make_float4(e1.x, e1.y, e1.z, next);
        lst[3 * r + 2] = tris[3 * s + 2];
    }
}

/* Conservative traversal for k_pixel_lists: every triangle some ray o + t d of the frustum
   could accept under intersects_triangle's tests is listed (`cap` at most: false on
   overflow): its slot, and the earliest t of such an accept.  (Kept in registers and ranked
   afterwards: 4.85 ms per dragon frame, against 5.6 ms for an insertion sort in the list
   itself at 109 instead of 164 VGPRs.) */
__device__ bool frustum_list(const float *__restrict__ nodes4, const uint32_t *__restrict__ q4,
                             const float4 *__restrict__ tris, const Frustum &fr, int *slots, float *keys, uint32_t cap,
                             uint32_t &n, lds_int *stack)
{
    const double *dlo = fr.dlo, *dhi = fr.dhi, *olo = fr.o;
    const double l1 = fr.l1;
    int sp = 0, node = 0;
    n = 0;
    bool ok = true;
    for (;;) {
        const float *f = nodes4 + 32ull * (uint32_t)node;
        for (int k = 0; k < 4 && ok; ++k) {
            const int c = __float_as_int(f[24 + k]);
            if (c == RT_EMPTY_CHILD) continue;
            const double lo[3] = {f[0 + k], f[8 + k], f[16 + k]}, hi[3] = {f[4 + k], f[12 + k], f[20 + k]};
            if (!frustum_slab(fr, lo, hi)) continue;
            if (c >= 0) {
                if (q4) { /* the child's normal box (determinant cull) */
                    const uint32_t wl = q4[(size_t)RT_QNODE_DWORDS * (uint32_t)c + 10];
                    const uint32_t wh = q4[(size_t)RT_QNODE_DWORDS * (uint32_t)c + 11];
                    const double sc = ldexp(1.0, (int)(wl >> 24) - 128);
                    const double nlo[3] = {((int)(wl & 255u) - 128) * sc, ((int)((wl >> 8) & 255u) - 128) * sc,
                                           ((int)((wl >> 16) & 255u) - 128) * sc};
                    const double nhi[3] = {((int)(wh & 255u) - 128) * sc, ((int)((wh >> 8) & 255u) - 128) * sc,
                                           ((int)((wh >> 16) & 255u) - 128) * sc};
                    if (frustum_det(dlo, dhi, nlo, nhi) * 1.02 + 5e-7 * l1 < 1e-4) continue;
                }
                if (sp >= kFrustumStack) {
                    ok = false;
                    break;
                }
                stack[RT_BLOCK * sp++] = c;
                continue;
            }
            const int enc = ~c, first = enc >> 3, cnt = (enc & 7) + 1;
            for (int j = 0; j < cnt; ++j) {
                const int s = first + j;
                const float4 r0 = tris[3 * s], r1 = tris[3 * s + 1], r2 = tris[3 * s + 2];
                double lo[3], hi[3], nmax, tin;
                tri_padded_box(r0, r1, r2, lo, hi, nmax);
                if (!frustum_slab(fr, lo, hi, &tin)) continue;
                const double e1[3] = {r1.x, r1.y, r1.z}, e2[3] = {r2.x, r2.y, r2.z};
                const double nv[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                                      e2[0] * e1[1] - e2[1] * e1[0]};
                const double el = (fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2])) * (fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2]));
                if (frustum_det(dlo, dhi, nv, nv) * (1.0 + 1e-6) + 8.0 * 0x1p-24 * l1 * el < 1e-4) continue;
                double tf2 = 0.0;
                for (int k = 0; k < 3; ++k) {
                    const double u = fmax(fabs(lo[k] - olo[k]), fabs(hi[k] - olo[k]));
                    tf2 += u * u;
                }
                if (!tri_meets_pixel(fr, r0, r1, r2, sqrt(tf2))) continue;
                if (n >= cap) {
                    ok = false;
                    break;
                }
                /* the earliest t any ray could accept this triangle at: the box entry less the
                   error of the float t (relative ~gamma |e1| |e2| |d| / |det|, |det| >= 1e-4;
                   30x margin), at the farthest t the box allows; kept in the spare r1.w */
                const double le1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
                const double le2 = sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
                const double terr = sqrt(tf2) * (2e-6 * le1 * le2 * l1 / 1e-4 + 1e-6) * l1 + 1e-5;
                /* the float t estimates the exact ray parameter of the triangle's plane, q / (N . d)
                   with q = N . (v0 - o): over the direction box N . d lies in [mlo, mhi], so where
                   that keeps one sign with q, t >= q / mhi (q, mlo > 0) or q / mlo (q, mhi < 0) —
                   for a triangle facing the pixel far later than its box's entry */
                double tpl = -1e300;
                {
                    double mlo = 0.0, mhi = 0.0, q = 0.0;
                    for (int k = 0; k < 3; ++k) {
                        const double a0 = nv[k] * dlo[k], a1 = nv[k] * dhi[k];
                        mlo += fmin(a0, a1);
                        mhi += fmax(a0, a1);
                        q += nv[k] * ((double)(k == 0 ? r0.x : k == 1 ? r0.y : r0.z) - olo[k]);
                    }
                    const double qe = 1e-12 * (fabs(nv[0]) + fabs(nv[1]) + fabs(nv[2])) * (1.0 + sqrt(tf2));
                    if (mlo > 0.0 && q - qe > 0.0) tpl = (q - qe) / (mhi * (1.0 + 1e-12));
                    else if (mhi < 0.0 && q + qe < 0.0) tpl = (q + qe) / (mlo * (1.0 + 1e-12));
                }
                slots[n] = s;
                keys[n] = __double2float_rd(fmax(tin, tpl) - terr);
                ++n;
            }
        }
        if (!ok || sp == 0) break;
        node = stack[RT_BLOCK * --sp];
    }
    return ok;
}

/* Seed-row halo pack / unpack (multi-GPU progressive sphere frames). */
__global__ __launch_bounds__(RT_BLOCK) void k_seed_rows(uint32_t *__restrict__ seeds, uint32_t wpad, uint32_t hpad,
                                                        const uint32_t *__restrict__ rows, uint32_t n,
                                                        uint32_t *__restrict__ buf, int unpack)
{
    const size_t idx = (size_t)blockIdx.x * RT_BLOCK + threadIdx.x;
    const size_t per_plane = (size_t)n * wpad;
    if (idx >= 2 * per_plane) return;
    const uint32_t p = (uint32_t)(idx / per_plane);
    const uint32_t i = (uint32_t)((idx % per_plane) / wpad);
    const uint32_t x = (uint32_t)(idx % wpad);
    uint32_t *s = seeds + (size_t)p * wpad * hpad + (size_t)rows[i] * wpad + x;
    if (unpack) *s = buf[idx];
    else buf[idx] = *s;
}

} // namespace

/* ======================================================================== */
/* Launchers                                                                 */

int rt_launch_seed_rows(uint32_t *seeds, uint32_t wpad, uint32_t hpad, const uint32_t *rows, uint32_t n,
                        uint32_t *buf, bool unpack, void *stream)
{
    const size_t total = 2ull * n * wpad;
    if (!total) return 0;
    dim3 grid((unsigned)((total + RT_BLOCK - 1) / RT_BLOCK)), block(RT_BLOCK);
    hipLaunchKernelGGL(k_seed_rows, grid, block, 0, (hipStream_t)stream, seeds, wpad, hpad, rows, n, buf,
                       unpack ? 1 : 0);
    return (int)hipGetLastError();
}

template <typename K>
static int occupancy(K kern, int *per_cu)
{
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kern, RT_BLOCK, 0);
}

int rt_launch_tris(const RtTriLaunch &a, int trav, bool count, int grid_blocks, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)grid_blocks), block(RT_BLOCK);
    /* the multi-head queue: its own instantiations (its take costs the others registers) */
    const bool mq = a.queue_batch && trav == RT_TRAV_BVH4Q && a.split_which != RT_SPLIT_BOX;
#define RT_LAUNCH_TRIS(T, S)                                                                                           \
    do {                                                                                                               \
        if (mq && count) hipLaunchKernelGGL((k_tris<RT_TRAV_BVH4Q, true, S, true>), grid, block, 0, st, a);            \
        else if (mq) hipLaunchKernelGGL((k_tris<RT_TRAV_BVH4Q, false, S, true>), grid, block, 0, st, a);               \
        else if (count) hipLaunchKernelGGL((k_tris<T, true, S>), grid, block, 0, st, a);                               \
        else hipLaunchKernelGGL((k_tris<T, false, S>), grid, block, 0, st, a);                                         \
    } while (0)
    /* the sample-split form only where it is used (its code costs a full frame 1 %) */
    if (trav == RT_TRAV_BVH4Q && a.split_chunks) {
        /* the chunk tasks (queue cursor a.work_counter — or the multi-head queue's heads — reset here) */
        const size_t words = mq ? (size_t)RT_QSTRIDE * RT_QHEADS : 1u;
        const hipError_t e = hipMemsetAsync(a.work_counter, 0, words * sizeof(uint32_t), st);
        if (e != hipSuccess) return (int)e;
        RT_LAUNCH_TRIS(RT_TRAV_BVH4Q, true);
    } else if (trav == RT_TRAV_LINEAR) RT_LAUNCH_TRIS(RT_TRAV_LINEAR, false);
    else if (trav == RT_TRAV_BVH4Q) RT_LAUNCH_TRIS(RT_TRAV_BVH4Q, false);
    else RT_LAUNCH_TRIS(RT_TRAV_BVH4, false);
#undef RT_LAUNCH_TRIS
    return (int)hipGetLastError();
}

/* The end of a render: its counters (n_cnt words) written straight into the host's pinned, mapped
   copy, and the counters and queue cursors (n_zero words from `dev`, the counters first) zeroed for
   the next render — one small kernel on the render's stream instead of a copy-engine transfer
   plus a fill at the next render's start.  `totals` (RT_COUNTER_WORDS + 1 words, device) keeps the
   context's running totals over renders, whose counters are otherwise overwritten render by
   render when renders are enqueued back to back (rt_counter_totals): sums for the summed counters
   and the repair count, maxima for the per-pixel maxima, the OR of the guard words, and the
   number of renders in the last word.  host == nullptr: totals only (the copy-engine path). */
__global__ __launch_bounds__(256) void k_counters_out(unsigned long long *__restrict__ dev,
                                                      unsigned long long *__restrict__ host,
                                                      unsigned long long *__restrict__ totals, uint32_t n_cnt,
                                                      uint32_t n_zero)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n_cnt) {
        const unsigned long long v = dev[i];
        if (host) host[i] = v;
        if (totals) {
            if (i < RT_N_SUM_COUNTERS || i == RT_CNT_REPAIR) totals[i] += v;
            else if (i == RT_CNT_GUARD) totals[i] |= v;
            else totals[i] = totals[i] > v ? totals[i] : v;
        }
    }
    if (totals && i == 0) totals[RT_COUNTER_WORDS] += 1ull;
    if (i < n_zero) dev[i] = 0ull;
}

int rt_launch_counters_out(unsigned long long *dev, unsigned long long *host_mapped, unsigned long long *totals,
                           uint32_t n_cnt, uint32_t n_zero, void *stream)
{
    const uint32_t n = n_cnt > n_zero ? n_cnt : n_zero;
    hipLaunchKernelGGL(k_counters_out, dim3((n + 255u) / 256u), dim3(256), 0, (hipStream_t)stream, dev, host_mapped,
                       totals, n_cnt, n_zero);
    return (int)hipGetLastError();
}

int rt_launch_split_seeds(const RtTriLaunch &a, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const hipError_t e = hipMemsetAsync(a.split_counter, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return (int)e;
    const dim3 g(a.split_seed_blocks), b(RT_BLOCK);
    if (a.split_which == RT_SPLIT_BOX && a.split_coop >= 8) { /* subtree-parallel */
        if (a.split_coop == 64 && a.split_restart) hipLaunchKernelGGL((k_chain_seeds<64, true>), g, b, 0, st, a);
        else if (a.split_coop == 32 && a.split_restart) hipLaunchKernelGGL((k_chain_seeds<32, true>), g, b, 0, st, a);
        else if (a.split_coop == 16 && a.split_restart) hipLaunchKernelGGL((k_chain_seeds<16, true>), g, b, 0, st, a);
        else if (a.split_coop == 8 && a.split_restart) hipLaunchKernelGGL((k_chain_seeds<8, true>), g, b, 0, st, a);
        else if (a.split_coop == 8) hipLaunchKernelGGL(k_chain_seeds<8>, g, b, 0, st, a);
        else if (a.split_coop == 32) hipLaunchKernelGGL(k_chain_seeds<32>, g, b, 0, st, a);
        else if (a.split_coop == 64) hipLaunchKernelGGL(k_chain_seeds<64>, g, b, 0, st, a);
        else hipLaunchKernelGGL(k_chain_seeds<16>, g, b, 0, st, a);
    } else if (a.split_coop == RT_SEED_COOP4) hipLaunchKernelGGL(k_split_seeds<4>, g, b, 0, st, a);
    else hipLaunchKernelGGL(k_split_seeds<1>, g, b, 0, st, a);
    return (int)hipGetLastError();
}

int rt_launch_split_finish(const RtTriLaunch &a, void *stream)
{
    if (a.finish_part == RT_FIN_LIST) { /* a wave per listed pixel */
        const uint32_t n = a.split_n_dev ? 4096u : a.split_n_box; /* a count on the device: grid-stride */
        const uint32_t blocks = std::min(2048u, std::max(1u, (n + 3u) / 4u));
        hipLaunchKernelGGL(k_split_finish_list, dim3(blocks), dim3(RT_BLOCK), 0, (hipStream_t)stream, a);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_split_finish, dim3((a.W * a.Hl + RT_BLOCK - 1) / RT_BLOCK), dim3(RT_BLOCK), 0,
                       (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

int rt_launch_spheres(const RtSphLaunch &a, bool single_sample, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    constexpr uint32_t T = RT_SPH_TILE;
    dim3 grid((a.W + T - 1u) / T, (a.Hl + T - 1u) / T), block(T * T);
    if (single_sample) hipLaunchKernelGGL((k_spheres<true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((k_spheres<false>), grid, block, 0, st, a);
    return (int)hipGetLastError();
}

int rt_launch_trace_rays(const float *nodes, const float *tris, uint32_t n_tris, const rt_ray *rays, uint32_t n,
                         int any_hit, int trav, int32_t *spill, uint32_t spill_cap, int32_t *out_idx, float *out_t,
                         unsigned long long *counters, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((n + RT_BLOCK - 1) / RT_BLOCK), block(RT_BLOCK);
    const float4 *nd = reinterpret_cast<const float4 *>(nodes);
    const float4 *tr = reinterpret_cast<const float4 *>(tris);
#define RT_LAUNCH_TRACE(T)                                                                                             \
    do {                                                                                                               \
        if (counters)                                                                                                  \
            hipLaunchKernelGGL((k_trace_rays<T, true>), grid, block, 0, st, nd, tr, n_tris, rays, n, any_hit, spill,   \
                               spill_cap, out_idx, out_t, counters);                                                   \
        else                                                                                                           \
            hipLaunchKernelGGL((k_trace_rays<T, false>), grid, block, 0, st, nd, tr, n_tris, rays, n, any_hit, spill,  \
                               spill_cap, out_idx, out_t, counters);                                                   \
    } while (0)
    if (trav == RT_TRAV_LINEAR) RT_LAUNCH_TRACE(RT_TRAV_LINEAR);
    else if (trav == RT_TRAV_BVH4Q) RT_LAUNCH_TRACE(RT_TRAV_BVH4Q);
    else RT_LAUNCH_TRACE(RT_TRAV_BVH4);
#undef RT_LAUNCH_TRACE
    return (int)hipGetLastError();
}

int rt_tris_grid_blocks(int device, int trav, bool count, int form, int *blocks)
{
    int per_cu = 0;
    int e;
    if (trav == RT_TRAV_LINEAR)
        e = count ? occupancy(k_tris<RT_TRAV_LINEAR, true>, &per_cu) : occupancy(k_tris<RT_TRAV_LINEAR, false>, &per_cu);
    else if (trav == RT_TRAV_BVH4Q && form == RT_FORM_SPLIT)
        e = count ? occupancy(k_tris<RT_TRAV_BVH4Q, true, true>, &per_cu)
                  : occupancy(k_tris<RT_TRAV_BVH4Q, false, true>, &per_cu);
    else if (trav == RT_TRAV_BVH4Q)
        e = count ? occupancy(k_tris<RT_TRAV_BVH4Q, true>, &per_cu) : occupancy(k_tris<RT_TRAV_BVH4Q, false>, &per_cu);
    else
        e = count ? occupancy(k_tris<RT_TRAV_BVH4, true>, &per_cu) : occupancy(k_tris<RT_TRAV_BVH4, false>, &per_cu);
    if (e) return e;
    int n_cu = 0;
    const hipError_t he = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (he != hipSuccess) return (int)he;
    if (getenv("RT_DEBUG_LAUNCH"))
        fprintf(stderr, "[rtmi] occupancy: trav %d count %d per_cu %d n_cu %d (device %d, err %d)\n", trav, (int)count,
                per_cu, n_cu, device, e);
    if (per_cu < 1) per_cu = 1;
    *blocks = per_cu * n_cu;
    return 0;
}

int rt_launch_pixel_lists(const RtTriLaunch &a, const float *nodes4, const uint32_t *q4, uint16_t *codes,
                          uint32_t *tile_base, void *stream)
{
    const uint32_t items = ((a.W + 7u) / 8u) * ((a.Hl + 7u) / 8u) * 64u;
    if (!a.W || !a.Hl) return 0;
    hipError_t e = hipMemsetAsync(a.list_alloc, 0, sizeof(uint32_t), (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_pixel_lists, dim3((items + RT_BLOCK - 1) / RT_BLOCK), dim3(RT_BLOCK), 0, (hipStream_t)stream,
                       a, nodes4, q4, codes, tile_base);
    return (int)hipGetLastError();
}

int rt_launch_probe_cost(const RtTriLaunch &a, int grid_blocks, uint32_t *out, void *stream)
{
    hipLaunchKernelGGL(k_probe_cost, dim3((unsigned)grid_blocks), dim3(RT_BLOCK), 0, (hipStream_t)stream, a, out);
    return (int)hipGetLastError();
}

/* Per stripe of a whole-frame probe (rt_partition_stripes): one block per stripe, its pixels'
   box flags and mesh-pixel steps summed over the block (integer sums: the same on every GPU). */
__global__ __launch_bounds__(256) void k_stripe_costs(const uint32_t *__restrict__ probe, uint32_t W, uint32_t H,
                                                      uint32_t stripe_rows, uint32_t pn2,
                                                      unsigned long long *__restrict__ out)
{
    __shared__ unsigned long long s_box[256], s_steps[256];
    const uint32_t s = blockIdx.x;
    const uint32_t y0 = s * stripe_rows, y1 = min(H, y0 + stripe_rows);
    unsigned long long box = 0, steps = 0;
    for (uint32_t p = y0 * W + threadIdx.x; p < y1 * W; p += 256u) {
        const uint32_t w = probe[p];
        if ((w >> RT_PROBE_HIT_SHIFT) < pn2) ++box;
        else steps += w & RT_PROBE_STEP_MASK;
    }
    s_box[threadIdx.x] = box;
    s_steps[threadIdx.x] = steps;
    __syncthreads();
    for (uint32_t k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) {
            s_box[threadIdx.x] += s_box[threadIdx.x + k];
            s_steps[threadIdx.x] += s_steps[threadIdx.x + k];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[2 * s] = s_box[0];
        out[2 * s + 1] = s_steps[0];
    }
}

int rt_launch_stripe_costs(const uint32_t *probe, uint32_t W, uint32_t H, uint32_t stripe_rows, uint32_t pn2,
                           unsigned long long *out, void *stream)
{
    const uint32_t ns = (H + stripe_rows - 1u) / stripe_rows;
    hipLaunchKernelGGL(k_stripe_costs, dim3(ns), dim3(256), 0, (hipStream_t)stream, probe, W, H, stripe_rows, pn2, out);
    return (int)hipGetLastError();
}

