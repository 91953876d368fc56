/*
 * rt_quant.h — the compressed 4-wide node (64 B), built identically by the host SAH
 * builder (rt_bvh.cpp) and the GPU builder (rt_build_gpu.hip) from a full-precision
 * 4-wide node whose inner children are numbered consecutively and whose leaf children
 * cover consecutive triangle slots, in child order.
 *
 * Layout (16 dwords, fetched as 4 x dwordx4; two nodes per 128-B line):
 *   d[0..2]  origin.xyz (float): the minimum corner of the children's boxes
 *   d[3]     bits 0-4 / 5-9 / 10-14: per-axis grid exponent e + 24 (e in [-24, 7]);
 *            bits 16-31: 4 bits per child k at 16 + 4k:
 *              bit 3 set: leaf, bits 0-2 = triangle count - 1;
 *              bit 3 clear: inner node, bits 0-1 = rank among the inner children
 *   d[4..9]  8-bit planes lo.x, hi.x, lo.y, hi.y, lo.z, hi.z (child k in byte k);
 *            plane = origin + q * 2^e, rounded outward (floor / ceil, checked in binary64)
 *            so the box contains the exact child box; an unused slot is the inverted
 *            box lo = 255 > hi = 0, which no ray enters
 *   d[10..11] the node's normal box (determinant cull, below): the box of the reference's
 *            unnormalised normals N = e2 x e1 over every triangle of the subtree, bytes
 *            b = q + 128 for q * 2^(E - 128), q in [-128, 127]: d[10] = lo.x | lo.y << 8 |
 *            lo.z << 16 | E << 24, d[11] = hi.x | hi.y << 8 | hi.z << 16 (E = 255: no cull)
 *   d[12..15] the four child links written out (rt_internal.h encoding)
 *
 * Determinant cull.  intersects_triangle rejects |det| < 1e-4 (geometryFuncs.h:167), and
 * det = (d x e2) . e1 = d . N exactly, so no triangle under a node can be accepted by a ray
 * whose max over the node's normal box of |d . N| is below 1e-4 minus the float error of
 * det (<= 8u |d|_1 max(|e1|_1 |e2|_1), which the builder keeps below 5e-7 |d|_1 for every
 * cullable node).  The traversal then skips the node's subtree: the same hits, the same
 * occlusion answers, fewer steps (rays that pass through the dragon-class mesh at moderate
 * incidence cross hundreds of leaf boxes of triangles too small to accept them). 
 * (A 48-B form without d[12..15], links decoded from d[3] / d[10] / d[11], measured 4.9 %
 * slower per frame — the decode's per-child branches cost more than the fourth load — and
 * was removed)
 */
#ifndef RT_QUANT_H
#define RT_QUANT_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "rt_internal.h"

#define RT_QNODE_DWORDS 16 /* dwords per compressed node */
#define RT_QEXP_MIN (-24)
#define RT_QEXP_MAX 7

#if defined(__HIPCC__)
#define RT_QHD __host__ __device__
#else
#define RT_QHD
#endif

/* f: 32 floats of a full-precision 4-wide node (rt_internal.h); q: RT_QNODE_DWORDS out.
   Returns false if a child's layout breaks the contiguity rules or an axis needs a grid
   step beyond 2^RT_QEXP_MAX (extent > 255 * 128). */
RT_QHD inline bool rt_quantize_node4(const float *f, uint32_t *q)
{
    int32_t code[4];
    for (int k = 0; k < 4; ++k) memcpy(&code[k], &f[24 + k], 4);
    uint32_t exps = 0, meta = 0;
    uint32_t planes[6] = {0, 0, 0, 0, 0, 0};
    int32_t inner_base = 0, tri_base = 0;
    int n_inner = 0, n_leaf_tris = 0;
    bool seen_empty = false;
    for (int k = 0; k < 4; ++k) {
        const int32_t c = code[k];
        if (c == RT_EMPTY_CHILD) {
            seen_empty = true;
            continue;
        }
        if (seen_empty) return false; /* unused slots must trail */
        if (c >= 0) {
            if (n_inner == 0) inner_base = c;
            else if (c != inner_base + n_inner) return false;
            meta |= (uint32_t)n_inner << (16 + 4 * k);
            ++n_inner;
        } else {
            const int32_t enc = ~c;
            const int32_t first = enc >> 3, count = (enc & 7) + 1;
            if (n_leaf_tris == 0) tri_base = first;
            else if (first != tri_base + n_leaf_tris) return false;
            meta |= (uint32_t)(8 | (count - 1)) << (16 + 4 * k);
            n_leaf_tris += count;
        }
    }
    for (int ax = 0; ax < 3; ++ax) {
        const float *lo = f + 8 * ax, *hi = f + 8 * ax + 4;
        float omin = INFINITY, omax = -INFINITY;
        for (int k = 0; k < 4; ++k)
            if (code[k] != RT_EMPTY_CHILD) {
                omin = fminf(omin, lo[k]);
                omax = fmaxf(omax, hi[k]);
            }
        if (!(omin <= omax)) omin = omax = 0.0f;
        const float origin = omin;
        int e = RT_QEXP_MIN;
        const double ext = (double)omax - (double)origin;
        if (ext > 0) {
            const int want = (int)ceil(log2(ext / 255.0));
            e = want > RT_QEXP_MIN ? want : RT_QEXP_MIN;
        }
        for (;; ++e) {
            if (e > RT_QEXP_MAX) return false;
            const double step = ldexp(1.0, e);
            bool ok = true;
            uint32_t wl = 0, wh = 0;
            for (int k = 0; k < 4; ++k) {
                int32_t l = 255, h = 0;
                if (code[k] != RT_EMPTY_CHILD) {
                    l = (int32_t)floor(((double)lo[k] - origin) / step);
                    h = (int32_t)ceil(((double)hi[k] - origin) / step);
                    if (l < 0) l = 0;
                    if (h > 255) ok = false;
                    if ((double)origin + l * step > (double)lo[k] || (double)origin + h * step < (double)hi[k])
                        ok = false;
                }
                wl |= (uint32_t)l << (8 * k);
                wh |= (uint32_t)(h & 255) << (8 * k);
            }
            if (ok) {
                planes[2 * ax] = wl;
                planes[2 * ax + 1] = wh;
                break;
            }
        }
        memcpy(&q[ax], &origin, 4);
        exps |= (uint32_t)(e - RT_QEXP_MIN) << (5 * ax);
    }
    q[3] = exps | meta;
    for (int i = 0; i < 6; ++i) q[4 + i] = planes[i];
    (void)inner_base;
    (void)tri_base;
    q[10] = 255u << 24; /* no cull until rt_qnode_set_nbox: [-128, 127] * 2^127 */
    q[11] = 0xffu << 16 | 0xffu << 8 | 0xffu;
    for (int k = 0; k < 4; ++k) q[12 + k] = (uint32_t)code[k]; /* explicit links */
    return true;
}

/* Encode a node's normal box (exact bounds in double) into d[10..11]; `err` is the node's
   max |e1|_1 |e2|_1, so 8u * err bounds det's float error per unit |d|_1.  Nodes whose error
   bound or range the encoding cannot honour keep the no-cull box. */
RT_QHD inline void rt_qnode_set_nbox(uint32_t *q, const double lo[3], const double hi[3], double err)
{
    if (!(8.0 * 0x1p-24 * err <= 5e-7)) return;
    double m = 0.0;
    for (int k = 0; k < 3; ++k) {
        if (!(lo[k] <= hi[k])) return;
        m = fmax(m, fmax(fabs(lo[k]), fabs(hi[k])));
    }
    int e = (m > 0.0) ? (int)ceil(log2(m / 127.0)) : -120;
    if (e < -120) e = -120; /* scales stay normal floats */
    for (;; ++e) {
        if (e > 126) return;
        const double step = ldexp(1.0, e);
        int32_t ql[3], qh[3];
        bool ok = true;
        for (int k = 0; k < 3; ++k) {
            ql[k] = (int32_t)floor(lo[k] / step);
            qh[k] = (int32_t)ceil(hi[k] / step);
            if (ql[k] < -128 || qh[k] > 127 || ql[k] * step > lo[k] || qh[k] * step < hi[k]) ok = false;
        }
        if (!ok) continue;
        q[10] = (uint32_t)(ql[0] + 128) | (uint32_t)(ql[1] + 128) << 8 | (uint32_t)(ql[2] + 128) << 16 |
                (uint32_t)(e + 128) << 24;
        q[11] = (uint32_t)(qh[0] + 128) | (uint32_t)(qh[1] + 128) << 8 | (uint32_t)(qh[2] + 128) << 16;
        return;
    }
}

#endif /* RT_QUANT_H */
