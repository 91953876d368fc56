/*
 * rt_sched.hip — the triangle kernel's pixel-queue schedule, computed on the device.
 *
 * The reference launches one work-item per pixel and lets the runtime order them
 * (raytracer.cl:184-243); a pixel's sampleRate^2 samples are one serial chain, so the
 * persistent k_tris takes 8 x 8 pixel tiles from a queue, and the order of that queue
 * sets how long the launch's tail is.  From the cost probe (k_probe_cost: per pixel the
 * mesh hits of a grid of probe rays and the traversal steps of their queries) this file
 * computes, without a host round trip:
 *   1. the frame's mean steps per probed query (k_probe_sums),
 *   2. each tile's estimated cost (k_tile_cost: a blend of its costliest pixel — the
 *      tile's last lane finishes with it — and its mean; a probe ray that misses the mesh
 *      stands for a box path of (1 + lights) x (maxDepth + 1) queries),
 *   3. the LPT order: tiles by cost, most expensive first (hipCUB radix sort, stable),
 *   4. the pixel classes (k_classify): mesh pixel -1; box pixel (some probe ray missed,
 *      or — for a sample-split render — a mesh pixel whose probe took over 96 steps per ray)
 *      with a slot >= 0 in pixel order up to the slot budget (an exclusive scan of the box
 *      flags), -2 beyond it; a sample-split render runs the slotted long chains apart.
 * Scheduling only: no pixel's result depends on when or where it is rendered.  This
 * replaced an 8 MB device-to-host copy, a host loop and a host sort per camera change
 * (every arrow key or drag of GlutCLWindow.cpp:229-279 restarts the refinement).
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>

#include "rt_internal.h"

namespace {

/* the probe-cost model's constants (measured on the dragon frame, DESIGN.md §5: a box-path
   query costs 1.4x the mean probed query; the tile key weighs its costliest pixel 0.75) */
constexpr double kBoxFactor = 1.4;
constexpr double kLptMax = 0.75;

__global__ __launch_bounds__(256) void k_probe_sums(const uint32_t *__restrict__ flags, uint32_t npx,
                                                    unsigned long long *__restrict__ sums)
{
    unsigned long long steps = 0, hits = 0;
    for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < npx; p += gridDim.x * 256u) {
        const uint32_t v = flags[p];
        steps += v & RT_PROBE_STEP_MASK;
        hits += v >> RT_PROBE_HIT_SHIFT;
    }
    for (int off = 32; off > 0; off >>= 1) {
        steps += __shfl_xor(steps, off);
        hits += __shfl_xor(hits, off);
    }
    if ((threadIdx.x & 63u) == 0) {
        atomicAdd(&sums[0], steps);
        atomicAdd(&sums[1], hits);
    }
}

/* one thread per 8 x 8 tile */
__global__ __launch_bounds__(256) void k_tile_cost(const uint32_t *__restrict__ flags, uint32_t W, uint32_t hl,
                                                   uint32_t pn2, uint32_t n_lights, uint32_t max_depth,
                                                   const unsigned long long *__restrict__ sums,
                                                   float *__restrict__ keys, uint32_t *__restrict__ idx)
{
    const uint32_t tx = (W + 7u) / 8u, n_t = tx * ((hl + 7u) / 8u);
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n_t) return;
    const uint64_t npx = (uint64_t)W * hl, nl = n_lights;
    const uint64_t hit_steps = sums[0], n_hit = sums[1];
    /* mean steps of one probed query: a hit ray's closest-hit + shadow queries, or a missing
       ray's closest-hit query */
    double q = n_hit ? (double)hit_steps / (double)(n_hit * (1 + nl) + ((uint64_t)pn2 * npx - n_hit)) : 20.0;
    if (q < 1.0) q = 1.0;
    const double c_box = (double)((1 + nl) * (uint64_t)(max_depth + 1)) * q * kBoxFactor;
    const uint32_t x0 = (t % tx) * 8u, y0 = (t / tx) * 8u;
    double sum = 0.0, mx = 0.0;
    for (uint32_t dy = 0; dy < 8u; ++dy) {
        const uint32_t y = y0 + dy;
        if (y >= hl) break;
        for (uint32_t dx = 0; dx < 8u; ++dx) {
            const uint32_t x = x0 + dx;
            if (x >= W) break;
            const uint32_t v = flags[(size_t)y * W + x];
            const double pc = ((double)(v & RT_PROBE_STEP_MASK) + (double)(pn2 - (v >> RT_PROBE_HIT_SHIFT)) * c_box) *
                                  (4.0 / (double)pn2) +
                              1.0;
            sum += pc;
            mx = mx > pc ? mx : pc;
        }
    }
    keys[t] = (float)((1.0 - kLptMax) * sum / 64.0 + kLptMax * mx);
    idx[t] = t;
}

/* The same key from a rendered frame: a pixel's cost is the number of its wave's loop iterations
   it was in flight (take to finish) — its queries, plus the stepping rounds its longer queries
   span — which, unlike the probe's few rays, sees every sample's light and bounce directions (the
   probe's shadow rays aim at the light centres); a sample-split frame's pixel: the sum over its nch
   chunk tasks (0 for pixels that ran elsewhere: the long chains) */
__global__ __launch_bounds__(256) void k_tile_cost_measured(const uint32_t *__restrict__ iters, uint32_t W,
                                                            uint32_t hl, uint32_t nch, float wmax,
                                                            float *__restrict__ keys, uint32_t *__restrict__ idx)
{
    const uint32_t tx = (W + 7u) / 8u, n_t = tx * ((hl + 7u) / 8u);
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n_t) return;
    const size_t n = (size_t)W * hl * nch;
    const uint32_t x0 = (t % tx) * 8u, y0 = (t / tx) * 8u;
    double sum = 0.0, mx = 0.0;
    for (uint32_t dy = 0; dy < 8u; ++dy) {
        const uint32_t y = y0 + dy;
        if (y >= hl) break;
        for (uint32_t dx = 0; dx < 8u; ++dx) {
            const uint32_t x = x0 + dx;
            if (x >= W) break;
            const size_t p = ((size_t)y * W + x) * nch;
            double pc = 1.0;
            for (uint32_t k = 0; k < nch; ++k) pc += (double)(iters[n + p + k] - iters[p + k]);
            sum += pc;
            mx = mx > pc ? mx : pc;
        }
    }
    keys[t] = (float)((1.0 - wmax) * sum / 64.0 + wmax * mx);
    idx[t] = t;
}

/* box[p] = 1 if some probe ray missed the mesh, or (step_max > 0) its probe queries took more
   than step_max steps in all (a long chain on the mesh: grazing camera rays without a candidate
   list); box[npx] = 0 (the scan's total) */
__global__ __launch_bounds__(256) void k_box_flags(const uint32_t *__restrict__ flags, uint32_t npx, uint32_t pn2,
                                                   uint32_t step_max, uint32_t row, uint32_t *__restrict__ box)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p < npx) {
        const uint32_t v = flags[p];
        bool b = (v >> RT_PROBE_HIT_SHIFT) < pn2 || (step_max && (v & RT_PROBE_STEP_MASK) > step_max);
        if (row && !b) {
            /* speculated mesh pixels (row = the tile's width): a pixel next to one whose probe
               missed the mesh (a silhouette) runs as a long chain instead — its camera rays may
               miss too, and a speculated pixel that does costs a repair */
            const uint32_t x = p % row, y = p / row, rows = npx / row;
            for (int dy = -1; dy <= 1 && !b; ++dy)
                for (int dx = -1; dx <= 1 && !b; ++dx) {
                    const int xx = (int)x + dx, yy = (int)y + dy;
                    if (xx < 0 || yy < 0 || xx >= (int)row || yy >= (int)rows) continue;
                    b = (flags[(uint32_t)yy * row + (uint32_t)xx] >> RT_PROBE_HIT_SHIFT) < pn2;
                }
        }
        box[p] = b ? 1u : 0u;
    } else if (p == npx) {
        box[p] = 0u;
    }
}

__global__ __launch_bounds__(256) void k_classify(const uint32_t *__restrict__ box, const uint32_t *__restrict__ scan,
                                                  uint32_t npx, uint32_t slots, int32_t *__restrict__ cls,
                                                  uint32_t *__restrict__ slot_pixel)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= npx) return;
    int32_t c = -1;
    if (box[p]) {
        const uint32_t s = scan[p];
        if (s < slots) {
            c = (int32_t)s;
            slot_pixel[s] = p;
        } else {
            c = -2;
        }
    }
    cls[p] = c;
}

} // namespace

void rt_sched_free(RtSchedScratch &s)
{
    for (void *p : {(void *)s.tmp, (void *)s.keys, (void *)s.keys_sorted, (void *)s.idx, (void *)s.box, (void *)s.scan,
                    (void *)s.sums})
        if (p) (void)hipFree(p);
    s = RtSchedScratch{};
}

static int reserve(RtSchedScratch &s, uint32_t n_t, uint32_t npx)
{
    hipError_t e = hipSuccess;
    if (!s.sums) e = hipMalloc(&s.sums, 2 * sizeof(unsigned long long));
    if (e == hipSuccess && s.cap_tiles < n_t) {
        if (s.keys) (void)hipFree(s.keys);
        if (s.keys_sorted) (void)hipFree(s.keys_sorted);
        if (s.idx) (void)hipFree(s.idx);
        s.keys = s.keys_sorted = nullptr;
        s.idx = nullptr;
        s.cap_tiles = 0;
        e = hipMalloc(&s.keys, n_t * sizeof(float));
        if (e == hipSuccess) e = hipMalloc(&s.keys_sorted, n_t * sizeof(float));
        if (e == hipSuccess) e = hipMalloc(&s.idx, n_t * sizeof(uint32_t));
        if (e == hipSuccess) s.cap_tiles = n_t;
    }
    if (e == hipSuccess && s.cap_px < npx) {
        if (s.box) (void)hipFree(s.box);
        if (s.scan) (void)hipFree(s.scan);
        s.box = s.scan = nullptr;
        s.cap_px = 0;
        e = hipMalloc(&s.box, (npx + 1) * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc(&s.scan, (npx + 1) * sizeof(uint32_t));
        if (e == hipSuccess) s.cap_px = npx;
    }
    if (e != hipSuccess) return (int)e;
    size_t sort_bytes = 0, scan_bytes = 0;
    e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, sort_bytes, s.keys, s.keys_sorted, s.idx, s.idx, (int)n_t);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, s.box, s.scan, (int)npx + 1);
    if (e != hipSuccess) return (int)e;
    const size_t need = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
    if (s.tmp_bytes < need) {
        if (s.tmp) (void)hipFree(s.tmp);
        s.tmp = nullptr;
        s.tmp_bytes = 0;
        e = hipMalloc(&s.tmp, need);
        if (e != hipSuccess) return (int)e;
        s.tmp_bytes = need;
    }
    return 0;
}

int rt_sched_order(RtSchedScratch &s, const uint32_t *flags, uint32_t W, uint32_t hl, uint32_t pn2, uint32_t n_lights,
                   uint32_t max_depth, uint32_t *order, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const uint32_t n_t = ((W + 7u) / 8u) * ((hl + 7u) / 8u), npx = W * hl;
    if (!n_t) return 0;
    int r = reserve(s, n_t, npx);
    if (r) return r;
    hipError_t e = hipMemsetAsync(s.sums, 0, 2 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return (int)e;
    const uint32_t sum_blocks = std::min<uint32_t>(1024u, (npx + 255u) / 256u);
    hipLaunchKernelGGL(k_probe_sums, dim3(sum_blocks), dim3(256), 0, st, flags, npx, s.sums);
    hipLaunchKernelGGL(k_tile_cost, dim3((n_t + 255u) / 256u), dim3(256), 0, st, flags, W, hl, pn2, n_lights,
                       max_depth, s.sums, s.keys, s.idx);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    size_t bytes = s.tmp_bytes;
    e = hipcub::DeviceRadixSort::SortPairsDescending(s.tmp, bytes, s.keys, s.keys_sorted, s.idx, order, (int)n_t, 0,
                                                     (int)(sizeof(float) * 8), st);
    return (int)e;
}

int rt_sched_order_measured(RtSchedScratch &s, const uint32_t *iters, uint32_t W, uint32_t hl, uint32_t nch,
                            uint32_t *order, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const uint32_t n_t = ((W + 7u) / 8u) * ((hl + 7u) / 8u);
    if (!n_t) return 0;
    int r = reserve(s, n_t, W * hl);
    if (r) return r;
    /* the tile key's weight of its costliest pixel: the probe key's */
    const float wmax = (float)kLptMax;
    hipLaunchKernelGGL(k_tile_cost_measured, dim3((n_t + 255u) / 256u), dim3(256), 0, st, iters, W, hl, nch, wmax,
                       s.keys, s.idx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    size_t bytes = s.tmp_bytes;
    e = hipcub::DeviceRadixSort::SortPairsDescending(s.tmp, bytes, s.keys, s.keys_sorted, s.idx, order, (int)n_t, 0,
                                                     (int)(sizeof(float) * 8), st);
    return (int)e;
}

int rt_sched_box_scan(RtSchedScratch &s, const uint32_t *flags, uint32_t npx, uint32_t pn2, uint32_t step_max,
                      uint32_t row, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_box_flags, dim3((npx + 1u + 255u) / 256u), dim3(256), 0, st, flags, npx, pn2, step_max, row,
                       s.box);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    size_t bytes = s.tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(s.tmp, bytes, s.box, s.scan, (int)npx + 1, st);
    return (int)e;
}

int rt_sched_classify(const RtSchedScratch &s, uint32_t npx, uint32_t slots, int32_t *cls, uint32_t *slot_pixel,
                      void *stream)
{
    hipLaunchKernelGGL(k_classify, dim3((npx + 255u) / 256u), dim3(256), 0, (hipStream_t)stream, s.box, s.scan, npx,
                       slots, cls, slot_pixel);
    return (int)hipGetLastError();
}
