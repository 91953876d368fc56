/*
 * rt_build_gpu.hip — BVH build on the GPU ("the step before the
 * path").  Produces the same 4-wide layouts the traversal reads (rt_internal.h: 128-B
 * float nodes (the full-precision traversal), 64-B compressed nodes for the
 * default traversal) and the leaf-ordered triangle records, from the mesh arrays of
 * raytrace_tris (tri_verts / tri_vert_idx, raytracer.cl:184-188).
 *
 *   1. per triangle: padded box (the host builder's pad: ext/512 + 1e-6(1+|coord|)) and
 *      centroid; centroid bounds by ordered-integer atomics;
 *   2. 63-bit Morton codes (21 bits per axis) of the centroids, radix-sorted (hipCUB)
 *      with the triangle index as payload;
 *   3. binary radix tree over the sorted codes (Karras 2012; equal codes broken by the
 *      slot index), one thread per inner node; every node covers a contiguous slot range;
 *   4. boxes bottom-up: one thread per leaf climbs, the second arrival at a node merges;
 *   5. collapse to the 4-wide tree top-down, one launch per level (largest-area child
 *      expanded first, as the host collapse; a subtree of <= kLeafMax triangles becomes a
 *      leaf over its slot range), nodes numbered breadth-first (root 0);
 *   6. quantisation of every node (same rounding rule as rt_bvh.cpp) and the triangle
 *      records in slot order, e1/e2 formed by the reference's get_triangle subtraction.
 *
 * The traversal contract is unchanged (conservative boxes, the accept rule in the leaf
 * test), so results equal the linear loop exactly; only the tree shape — and therefore
 * speed — differs from the host SAH build.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cmath>
#include <string>
#include <vector>

#include "rt_internal.h"
#include "rt_quant.h"

#pragma clang fp contract(off)

namespace {

constexpr int kB = 256;
constexpr uint32_t kLeafMax = 4; /* largest slot range emitted as one leaf */

__device__ __forceinline__ uint32_t f2key(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

/* 1. padded triangle boxes + centroids; bounds[0..2] = min key, [3..5] = max key */
__global__ void k_prep(const float *__restrict__ verts, const int32_t *__restrict__ idx, uint32_t n,
                       float *__restrict__ tbox, float *__restrict__ cent, uint32_t *__restrict__ bounds)
{
    const uint32_t t = blockIdx.x * kB + threadIdx.x;
    float c[3] = {0, 0, 0};
    bool ok = t < n;
    if (ok) {
        float lo[3], hi[3], maxabs = 0.0f;
        for (int a = 0; a < 3; ++a) {
            lo[a] = INFINITY;
            hi[a] = -INFINITY;
        }
        for (int k = 0; k < 3; ++k) {
            const float *p = verts + 3ull * (uint32_t)idx[3ull * t + k];
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(lo[a], p[a]);
                hi[a] = fmaxf(hi[a], p[a]);
                maxabs = fmaxf(maxabs, fabsf(p[a]));
            }
        }
        float ext = 0.0f;
        for (int a = 0; a < 3; ++a) ext = fmaxf(ext, hi[a] - lo[a]);
        const float pad = ext * (1.0f / 512.0f) + 1e-6f * (1.0f + maxabs);
        for (int a = 0; a < 3; ++a) {
            c[a] = 0.5f * (lo[a] + hi[a]);
            cent[3ull * t + a] = c[a];
            tbox[6ull * t + a] = lo[a] - pad;
            tbox[6ull * t + 3 + a] = hi[a] + pad;
        }
    }
    /* block reduction of the centroid bounds, one atomic per block and bound */
    __shared__ uint32_t s_lo[3], s_hi[3];
    if (threadIdx.x < 3) {
        s_lo[threadIdx.x] = 0xFFFFFFFFu;
        s_hi[threadIdx.x] = 0u;
    }
    __syncthreads();
    if (ok)
        for (int a = 0; a < 3; ++a) {
            atomicMin(&s_lo[a], f2key(c[a]));
            atomicMax(&s_hi[a], f2key(c[a]));
        }
    __syncthreads();
    if (threadIdx.x < 3) {
        atomicMin(&bounds[threadIdx.x], s_lo[threadIdx.x]);
        atomicMax(&bounds[3 + threadIdx.x], s_hi[threadIdx.x]);
    }
}

__device__ __forceinline__ uint64_t spread21(uint64_t v)
{
    v &= 0x1FFFFFull;
    v = (v | (v << 32)) & 0x1F00000000FFFFull;
    v = (v | (v << 16)) & 0x1F0000FF0000FFull;
    v = (v | (v << 8)) & 0x100F00F00F00F00Full;
    v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
    v = (v | (v << 2)) & 0x1249249249249249ull;
    return v;
}

/* 2. Morton codes + identity payload */
__global__ void k_morton(const float *__restrict__ cent, uint32_t n, const uint32_t *__restrict__ bounds,
                         uint64_t *__restrict__ keys, uint32_t *__restrict__ vals)
{
    const uint32_t t = blockIdx.x * kB + threadIdx.x;
    if (t >= n) return;
    uint64_t code = 0;
    for (int a = 0; a < 3; ++a) {
        const float lo = key2f(bounds[a]), hi = key2f(bounds[3 + a]);
        const float ext = hi - lo;
        float u = ext > 0.0f ? (cent[3ull * t + a] - lo) / ext : 0.0f;
        u = fminf(fmaxf(u, 0.0f), 1.0f);
        const uint64_t q = (uint64_t)fminf(u * 2097152.0f, 2097151.0f);
        code |= spread21(q) << (2 - a);
    }
    keys[t] = code;
    vals[t] = t;
}

/* 3. radix tree.  Inner node i in [0, n-2]; child c >= 0 inner, c < 0 leaf ~slot. */
__device__ __forceinline__ int delta(const uint64_t *__restrict__ k, int n, int i, int j)
{
    if (j < 0 || j >= n) return -1;
    const uint64_t a = k[i], b = k[j];
    if (a == b) return 64 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clzll((long long)(a ^ b));
}

__global__ void k_radix_tree(const uint64_t *__restrict__ k, int n, int2 *__restrict__ child,
                             int2 *__restrict__ range, int *__restrict__ parent_inner, int *__restrict__ parent_leaf)
{
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(k, n, i, j);
    int s = 0;
    int t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int g = i + s * d + (d < 0 ? -1 : 0);
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    const int left = (lo == g) ? ~g : g;
    const int right = (hi == g + 1) ? ~(g + 1) : g + 1;
    child[i] = make_int2(left, right);
    range[i] = make_int2(lo, hi);
    if (left >= 0) parent_inner[left] = i;
    else parent_leaf[~left] = i;
    if (right >= 0) parent_inner[right] = i;
    else parent_leaf[~right] = i;
}

/* 4. bottom-up boxes */
__global__ void k_boxes(const float *__restrict__ tbox, const uint32_t *__restrict__ perm, int n,
                        const int2 *__restrict__ child, const int *__restrict__ parent_inner,
                        const int *__restrict__ parent_leaf, float *__restrict__ nbox, int *__restrict__ flags)
{
    const int s = blockIdx.x * kB + threadIdx.x;
    if (s >= n || n < 2) return;
    int node = parent_leaf[s];
    while (node >= 0) {
        __threadfence();
        if (atomicAdd(&flags[node], 1) == 0) return; /* the sibling finishes this node */
        __threadfence();
        const int2 c = child[node];
        float b[6];
        for (int q = 0; q < 2; ++q) {
            const int ci = q ? c.y : c.x;
            const float *src = ci >= 0 ? nbox + 6ull * ci : tbox + 6ull * perm[~ci];
            /* the sibling's box was written by another workgroup: L1-bypassing loads */
            float v[6];
            for (int a = 0; a < 6; ++a)
                v[a] = __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t *>(src + a),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (q == 0)
                for (int a = 0; a < 6; ++a) b[a] = v[a];
            else
                for (int a = 0; a < 3; ++a) {
                    b[a] = fminf(b[a], v[a]);
                    b[3 + a] = fmaxf(b[3 + a], v[3 + a]);
                }
        }
        for (int a = 0; a < 6; ++a) nbox[6ull * node + a] = b[a];
        node = node == 0 ? -1 : parent_inner[node];
    }
}

__device__ __forceinline__ float box_area(const float *b)
{
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    if (!(dx >= 0.0f) || !(dy >= 0.0f) || !(dz >= 0.0f)) return 0.0f;
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

struct Frontier {
    int bin;   /* binary inner node (or ~slot for a single-triangle mesh) */
    int out;   /* 4-wide node index */
    int stack; /* traversal stack entries live on entry */
};

/* 5. one level of the top-down collapse */
__global__ void k_collapse(const Frontier *__restrict__ cur, const uint32_t *__restrict__ n_cur,
                           Frontier *__restrict__ next, uint32_t *__restrict__ n_next, uint32_t *__restrict__ n_nodes,
                           uint32_t *__restrict__ max_stack, const int2 *__restrict__ child,
                           const int2 *__restrict__ range, const float *__restrict__ nbox,
                           const float *__restrict__ tbox, const uint32_t *__restrict__ perm, int n,
                           float *__restrict__ nodes4, uint32_t *__restrict__ n_tris_out,
                           uint32_t *__restrict__ perm2)
{
    const uint32_t e = blockIdx.x * kB + threadIdx.x;
    if (e >= *n_cur) return;
    const Frontier f = cur[e];
    int kids[4] = {0, 0, 0, 0};
    int nk = 0;
    auto size_of = [&](int c) -> int { return c >= 0 ? range[c].y - range[c].x + 1 : 1; };
    auto expandable = [&](int c) -> bool { return c >= 0 && size_of(c) > (int)kLeafMax; };
    if (f.bin < 0 || n < 2 || size_of(f.bin) <= (int)kLeafMax) {
        kids[nk++] = f.bin; /* the whole (small) mesh as one leaf */
    } else {
        kids[nk++] = child[f.bin].x;
        kids[nk++] = child[f.bin].y;
        while (nk < 4) {
            int best = -1;
            float best_a = -1.0f;
            for (int i = 0; i < nk; ++i)
                if (expandable(kids[i])) {
                    const float a = box_area(nbox + 6ull * kids[i]);
                    if (a > best_a) {
                        best_a = a;
                        best = i;
                    }
                }
            if (best < 0) break;
            const int c = kids[best];
            kids[best] = child[c].x;
            kids[nk++] = child[c].y;
        }
    }
    const int stk = f.stack + (nk > 0 ? nk - 1 : 0);
    atomicMax(max_stack, (uint32_t)stk);
    /* inner children get consecutive node indices, leaf children consecutive
       triangle slots (rt_quant.h), allocated as one block each */
    int n_in = 0;
    uint32_t n_leaf_tris = 0;
    for (int k = 0; k < nk; ++k) {
        const int c = kids[k];
        if (c >= 0 && n >= 2 && expandable(c)) ++n_in;
        else n_leaf_tris += (c < 0 && n >= 2) ? 1u : (n >= 2 && c >= 0 ? (uint32_t)size_of(c) : (uint32_t)n);
    }
    const uint32_t node_base = n_in ? atomicAdd(n_nodes, (uint32_t)n_in) : 0u;
    const uint32_t tri_base = n_leaf_tris ? atomicAdd(n_tris_out, n_leaf_tris) : 0u;
    uint32_t next_node = node_base, next_tri = tri_base;
    float *nd = nodes4 + 32ull * f.out;
    for (int k = 0; k < 4; ++k) {
        int32_t code = RT_EMPTY_CHILD;
        float b[6] = {0, 0, 0, 0, 0, 0};
        if (k < nk) {
            const int c = kids[k];
            if (c >= 0 && n >= 2 && expandable(c)) {
                for (int a = 0; a < 6; ++a) b[a] = nbox[6ull * c + a];
                const uint32_t id = next_node++;
                code = (int32_t)id;
                const uint32_t q = atomicAdd(n_next, 1u);
                next[q] = Frontier{c, (int)id, stk};
            } else {
                /* a leaf: one triangle (binary leaf), a small subtree's slot range, or
                   the whole mesh of <= kLeafMax triangles */
                uint32_t first_old = 0, count = (uint32_t)n;
                if (c < 0 && n >= 2) {
                    first_old = (uint32_t)(~c);
                    count = 1;
                    for (int a = 0; a < 6; ++a) b[a] = tbox[6ull * perm[first_old] + a];
                } else if (n >= 2) {
                    first_old = (uint32_t)range[c].x;
                    count = (uint32_t)(range[c].y - range[c].x + 1);
                    for (int a = 0; a < 6; ++a) b[a] = nbox[6ull * c + a];
                } else {
                    for (int a = 0; a < 6; ++a) b[a] = tbox[6ull * perm[0] + a];
                }
                const uint32_t first = next_tri;
                next_tri += count;
                for (uint32_t q = 0; q < count; ++q) perm2[first + q] = first_old + q;
                code = ~(int32_t)((first << 3) | (count - 1));
            }
        }
        nd[0 + k] = b[0];
        nd[4 + k] = b[3];
        nd[8 + k] = b[1];
        nd[12 + k] = b[4];
        nd[16 + k] = b[2];
        nd[20 + k] = b[5];
        nd[24 + k] = __int_as_float(code);
        nd[28 + k] = 0.0f;
    }
}

/* 6a. compressed nodes (rt_quant.h, the host builder's encoder); flag = 1 if any
   node cannot be encoded (the traversal then uses the full-precision nodes) */
__global__ void k_quantize(const float *__restrict__ nodes4, uint32_t n_nodes, uint32_t *__restrict__ q4,
                           uint32_t *__restrict__ fail)
{
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= n_nodes) return;
    if (!rt_quantize_node4(nodes4 + 32ull * i, q4 + (uint64_t)RT_QNODE_DWORDS * i)) atomicOr(fail, 1u);
}

/* 6b. triangle records in slot order: (v0, orig), (v1 - v0), (v2 - v0) (rtcommon.h:20-37) */
__global__ void k_tri_records(const float *__restrict__ verts, const int32_t *__restrict__ idx,
                              const uint32_t *__restrict__ perm, const uint32_t *__restrict__ perm2, uint32_t n,
                              float *__restrict__ tris)
{
    const uint32_t s = blockIdx.x * kB + threadIdx.x;
    if (s >= n) return;
    const uint32_t t = perm[perm2[s]];
    const float *a = verts + 3ull * (uint32_t)idx[3ull * t];
    const float *p1 = verts + 3ull * (uint32_t)idx[3ull * t + 1];
    const float *p2 = verts + 3ull * (uint32_t)idx[3ull * t + 2];
    float *o = tris + 12ull * s;
    o[0] = a[0];
    o[1] = a[1];
    o[2] = a[2];
    o[3] = __int_as_float((int32_t)t);
    o[4] = p1[0] - a[0];
    o[5] = p1[1] - a[1];
    o[6] = p1[2] - a[2];
    o[7] = 0.0f;
    o[8] = p2[0] - a[0];
    o[9] = p2[1] - a[1];
    o[10] = p2[2] - a[2];
    o[11] = 0.0f;
}

/* 6c. normal boxes of the compressed nodes (rt_quant.h determinant cull), one level of the
   4-wide tree per launch from the deepest up: a node's inner children (the next level) are
   done, its leaf children's triangles are read from the records.  binary64, as the host
   builder. */
struct NBox {
    double lo[3], hi[3], err;
};
__global__ void k_nbox(const float *__restrict__ nodes4, uint32_t first, uint32_t last, const float *__restrict__ tris,
                       NBox *__restrict__ nb, uint32_t *__restrict__ q4)
{
    const uint32_t i = first + blockIdx.x * kB + threadIdx.x;
    if (i >= last) return;
    NBox b;
    for (int a = 0; a < 3; ++a) {
        b.lo[a] = __builtin_huge_val();
        b.hi[a] = -__builtin_huge_val();
    }
    b.err = 0.0;
    const float *f = nodes4 + 32ull * i;
    for (int k = 0; k < 4; ++k) {
        const int32_t c = __float_as_int(f[24 + k]);
        if (c == RT_EMPTY_CHILD) continue;
        if (c >= 0) {
            const NBox &cb = nb[c];
            for (int a = 0; a < 3; ++a) {
                b.lo[a] = fmin(b.lo[a], cb.lo[a]);
                b.hi[a] = fmax(b.hi[a], cb.hi[a]);
            }
            b.err = fmax(b.err, cb.err);
            continue;
        }
        const int32_t enc = ~c, lf = enc >> 3, cnt = (enc & 7) + 1;
        for (int32_t j = 0; j < cnt; ++j) {
            const float *o = tris + 12ull * (uint32_t)(lf + j);
            const double e1[3] = {o[4], o[5], o[6]}, e2[3] = {o[8], o[9], o[10]};
            const double n[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                                 e2[0] * e1[1] - e2[1] * e1[0]};
            for (int a = 0; a < 3; ++a) {
                b.lo[a] = fmin(b.lo[a], n[a]);
                b.hi[a] = fmax(b.hi[a], n[a]);
            }
            b.err = fmax(b.err, (fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2])) * (fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2])));
        }
    }
    nb[i] = b;
    rt_qnode_set_nbox(q4 + (uint64_t)RT_QNODE_DWORDS * i, b.lo, b.hi, b.err);
}

unsigned blocks_for(uint64_t n) { return (unsigned)((n + kB - 1) / kB); }

/* RAII scratch */
struct DevBuf {
    void *p = nullptr;
    ~DevBuf()
    {
        if (p) (void)hipFree(p);
    }
};

} // namespace

#define GCHK(x)                                                                                                        \
    do {                                                                                                               \
        const hipError_t e_ = (x);                                                                                     \
        if (e_ != hipSuccess) {                                                                                        \
            err = std::string(#x) + ": " + hipGetErrorString(e_);                                                      \
            return (int)e_;                                                                                            \
        }                                                                                                              \
    } while (0)

int rt_build_bvh_gpu(const float *verts_h, uint32_t n_verts, const int32_t *idx_h, uint32_t n_tris, RtGpuBvh &out,
                     std::string &err, void *stream, bool det_cull)
{
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t st = (hipStream_t)stream;
    const int n = (int)n_tris;
    DevBuf d_verts, d_idx, d_tbox, d_cent, d_bounds, d_keys, d_keys2, d_vals, d_perm, d_child, d_range, d_pin,
        d_pleaf, d_nbox, d_flags, d_front[2], d_counts, d_tmp, d_perm2;
    GCHK(hipMalloc(&d_verts.p, 12ull * n_verts));
    GCHK(hipMalloc(&d_idx.p, 12ull * n_tris));
    GCHK(hipMemcpyAsync(d_verts.p, verts_h, 12ull * n_verts, hipMemcpyHostToDevice, st));
    GCHK(hipMemcpyAsync(d_idx.p, idx_h, 12ull * n_tris, hipMemcpyHostToDevice, st));
    GCHK(hipMalloc(&d_tbox.p, 24ull * n_tris));
    GCHK(hipMalloc(&d_cent.p, 12ull * n_tris));
    GCHK(hipMalloc(&d_bounds.p, 6 * sizeof(uint32_t)));
    const uint32_t init_bounds[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    GCHK(hipMemcpyAsync(d_bounds.p, init_bounds, sizeof(init_bounds), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_prep, dim3(blocks_for(n_tris)), dim3(kB), 0, st, (const float *)d_verts.p,
                       (const int32_t *)d_idx.p, n_tris, (float *)d_tbox.p, (float *)d_cent.p,
                       (uint32_t *)d_bounds.p);
    GCHK(hipGetLastError());

    GCHK(hipMalloc(&d_keys.p, 8ull * n_tris));
    GCHK(hipMalloc(&d_keys2.p, 8ull * n_tris));
    GCHK(hipMalloc(&d_vals.p, 4ull * n_tris));
    GCHK(hipMalloc(&d_perm.p, 4ull * n_tris));
    hipLaunchKernelGGL(k_morton, dim3(blocks_for(n_tris)), dim3(kB), 0, st, (const float *)d_cent.p, n_tris,
                       (const uint32_t *)d_bounds.p, (uint64_t *)d_keys.p, (uint32_t *)d_vals.p);
    GCHK(hipGetLastError());
    size_t tmp_bytes = 0;
    GCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (uint64_t *)d_keys.p, (uint64_t *)d_keys2.p,
                                            (uint32_t *)d_vals.p, (uint32_t *)d_perm.p, n, 0, 63, st));
    GCHK(hipMalloc(&d_tmp.p, tmp_bytes));
    GCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tmp_bytes, (uint64_t *)d_keys.p, (uint64_t *)d_keys2.p,
                                            (uint32_t *)d_vals.p, (uint32_t *)d_perm.p, n, 0, 63, st));

    const uint64_t n_inner = n >= 2 ? (uint64_t)n - 1 : 1;
    GCHK(hipMalloc(&d_child.p, 8ull * n_inner));
    GCHK(hipMalloc(&d_range.p, 8ull * n_inner));
    GCHK(hipMalloc(&d_pin.p, 4ull * n_inner));
    GCHK(hipMalloc(&d_pleaf.p, 4ull * n_tris));
    GCHK(hipMalloc(&d_nbox.p, 24ull * n_inner));
    GCHK(hipMalloc(&d_flags.p, 4ull * n_inner));
    GCHK(hipMemsetAsync(d_flags.p, 0, 4ull * n_inner, st));
    GCHK(hipMemsetAsync(d_pin.p, 0xFF, 4ull * n_inner, st));
    if (n >= 2) {
        hipLaunchKernelGGL(k_radix_tree, dim3(blocks_for(n - 1)), dim3(kB), 0, st, (const uint64_t *)d_keys2.p, n,
                           (int2 *)d_child.p, (int2 *)d_range.p, (int *)d_pin.p, (int *)d_pleaf.p);
        GCHK(hipGetLastError());
        hipLaunchKernelGGL(k_boxes, dim3(blocks_for(n_tris)), dim3(kB), 0, st, (const float *)d_tbox.p,
                           (const uint32_t *)d_perm.p, n, (const int2 *)d_child.p, (const int *)d_pin.p,
                           (const int *)d_pleaf.p, (float *)d_nbox.p, (int *)d_flags.p);
        GCHK(hipGetLastError());
    }

    /* collapse: the 4-wide tree has fewer nodes than the binary tree has inner nodes */
    const uint64_t cap4 = n_inner + 1;
    float *nodes4 = nullptr;
    GCHK(hipMalloc(&nodes4, 128ull * cap4));
    out.nodes4 = nodes4;
    GCHK(hipMalloc(&d_front[0].p, sizeof(Frontier) * cap4));
    GCHK(hipMalloc(&d_front[1].p, sizeof(Frontier) * cap4));
    GCHK(hipMalloc(&d_counts.p, 8 * sizeof(uint32_t)));
    GCHK(hipMalloc(&d_perm2.p, 4ull * n_tris));
    /* counts: [0] frontier A size, [1] frontier B size, [2] nodes, [3] max stack,
       [4] triangle slots handed out, [5] quantisation failure flag */
    const Frontier root = {n >= 2 ? 0 : ~0, 0, 0};
    GCHK(hipMemcpyAsync(d_front[0].p, &root, sizeof(root), hipMemcpyHostToDevice, st));
    const uint32_t init_counts[8] = {1u, 0u, 1u, 0u, 0u, 0u, 0u, 0u};
    GCHK(hipMemcpyAsync(d_counts.p, init_counts, sizeof(init_counts), hipMemcpyHostToDevice, st));
    uint32_t *cnt = (uint32_t *)d_counts.p;
    uint32_t level_size = 1, depth = 0;
    int cur = 0;
    std::vector<uint32_t> level_end{1}; /* node ids of level L: [level_end[L-1], level_end[L]) */
    while (level_size > 0) {
        ++depth;
        GCHK(hipMemsetAsync(cnt + (1 - cur), 0, sizeof(uint32_t), st));
        hipLaunchKernelGGL(k_collapse, dim3(blocks_for(level_size)), dim3(kB), 0, st,
                           (const Frontier *)d_front[cur].p, cnt + cur, (Frontier *)d_front[1 - cur].p,
                           cnt + (1 - cur), cnt + 2, cnt + 3, (const int2 *)d_child.p, (const int2 *)d_range.p,
                           (const float *)d_nbox.p, (const float *)d_tbox.p, (const uint32_t *)d_perm.p, n, nodes4,
                           cnt + 4, (uint32_t *)d_perm2.p);
        GCHK(hipGetLastError());
        GCHK(hipMemcpyAsync(&level_size, cnt + (1 - cur), sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        uint32_t n_alloc = 0;
        GCHK(hipMemcpyAsync(&n_alloc, cnt + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        GCHK(hipStreamSynchronize(st));
        if (level_size > 0) level_end.push_back(n_alloc);
        cur = 1 - cur;
        if (depth > 4096) {
            err = "GPU BVH collapse did not terminate";
            return -1;
        }
    }
    uint32_t counts[8];
    GCHK(hipMemcpyAsync(counts, cnt, sizeof(counts), hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    out.n_nodes4 = counts[2];
    out.depth4 = depth;
    out.stack4 = counts[3];

    if (counts[4] != n_tris) {
        err = "GPU BVH collapse lost triangles";
        return -1;
    }
    uint32_t *q4 = nullptr;
    GCHK(hipMalloc(&q4, 4ull * RT_QNODE_DWORDS * out.n_nodes4));
    out.nodes4q = q4;
    hipLaunchKernelGGL(k_quantize, dim3(blocks_for(out.n_nodes4)), dim3(kB), 0, st, (const float *)nodes4,
                       out.n_nodes4, q4, cnt + 5);
    GCHK(hipGetLastError());
    float *tris = nullptr;
    GCHK(hipMalloc(&tris, 48ull * n_tris));
    out.tris = tris;
    hipLaunchKernelGGL(k_tri_records, dim3(blocks_for(n_tris)), dim3(kB), 0, st, (const float *)d_verts.p,
                       (const int32_t *)d_idx.p, (const uint32_t *)d_perm.p, (const uint32_t *)d_perm2.p, n_tris,
                       tris);
    GCHK(hipGetLastError());
    if (det_cull) {
        DevBuf d_nb;
        GCHK(hipMalloc(&d_nb.p, sizeof(NBox) * out.n_nodes4));
        for (size_t L = level_end.size(); L-- > 0;) {
            const uint32_t a = L ? level_end[L - 1] : 0u, b = level_end[L];
            if (b <= a) continue;
            hipLaunchKernelGGL(k_nbox, dim3(blocks_for(b - a)), dim3(kB), 0, st, (const float *)nodes4, a, b,
                               (const float *)tris, (NBox *)d_nb.p, q4);
            GCHK(hipGetLastError());
        }
        GCHK(hipStreamSynchronize(st));
    }
    uint32_t qfail = 0;
    GCHK(hipMemcpyAsync(&qfail, cnt + 5, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    if (qfail) { /* not encodable: full-precision nodes only */
        (void)hipFree(q4);
        out.nodes4q = nullptr;
    }
    out.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}
