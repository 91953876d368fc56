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

/* No C++ exception crosses the C ABI (the reference lets cl::Error escape,
   RayTracerCL.cpp:102-107): every extern "C" entry that can allocate or parse is a
   function-try-block ending in RT_CATCH(err), which maps the exception in flight to a status —
   std::bad_alloc / std::length_error to RT_ERR_ALLOC, any other std::exception to RT_ERR_ARG,
   anything else to RT_ERR_STATE — and stores its message in *err (may be NULL). */
int rt_exception_status(std::string *err) noexcept;
#define RT_CATCH(err_ptr)                                                                                              \
    catch (...) { return rt_exception_status(err_ptr); }

/* Traversal stack entries per lane kept in LDS (20 x 256 lanes x 4 B = 20 KB per block, which
   with k_tris's other per-lane LDS — pixel sum and throughput, list word, hit normal: 31,232 B
   per block in all — keeps 5 blocks per CU; one block more of LDS measured 3.5 % slower:
   profiles/r03z, r03zb); deeper entries go to a per-lane global spill tail sized from the tree
   (rt_host.cpp spill_cap). */
#ifndef RT_STACK_DEPTH
#define RT_STACK_DEPTH 20
#endif
/* Inner depth bound of the binary tree (median splits below it). */
#define RT_BVH_MAX_DEPTH 33
#define RT_BLOCK 256
/* waves per SIMD the triangle kernel is compiled for (register budget 512 / waves) */
/* cost-probe word: hits (0..25) in the top 5 bits, traversal steps below */
#define RT_PROBE_HIT_SHIFT 27
#define RT_PROBE_STEP_MASK ((1u << RT_PROBE_HIT_SHIFT) - 1u)
#ifndef RT_STEP_UNROLL
#define RT_STEP_UNROLL 4 /* traversal steps per exit check in k_tris (round 6, dragon frame: 3 / 4 / 5 / 6 / 8:
                            76.8 / 76.3-76.5 / 77.2 / 77.6-77.8 / 80.4 ms, profiles/r06zz; r01: 6 best) */
#endif
#ifndef RT_DIAG_ONE_PIXEL
#define RT_DIAG_ONE_PIXEL 0 /* diagnostics build: k_tris renders only the pixel RT_DIAG_PIXEL=x,y names (the
                               others are skipped), so its serial chain runs alone in its wave */
#endif
#ifndef RT_PLAIN_PIXEL_STATS
#define RT_PLAIN_PIXEL_STATS 0 /* RT_PIXEL_STATS clocks in plain (not only counting) launches: a
                                  diagnostics build (costs registers: 0.5 %) */
#endif
#ifndef RT_TRIS_WAVES
#define RT_TRIS_WAVES 5
#endif
#define RT_LEAF_MAX 8
/* device counters: rays_closest, rays_shadow, nodes, tris, leaves, lane slots,
   traversal-loop clocks, kernel clocks (the last two: per lane, summed), shadow rays
   answered without a traversal, path-advance (shading) clocks — summed over lanes; then
   per-pixel maxima: clocks, queries, traversal steps of the costliest pixel */
#define RT_N_SUM_COUNTERS 10
#define RT_N_COUNTERS 13
#define RT_CNT_SKIPPED 8
#define RT_CNT_SHADE 9
/* past the counters: the long chains' seed-pass defect guards (atomicOr of RT_GUARD_*), then the
   count of speculated pixels to repair (sample-split renders, split_spec); the device counter
   buffer holds RT_COUNTER_WORDS words */
#define RT_CNT_GUARD RT_N_COUNTERS
#define RT_CNT_REPAIR (RT_N_COUNTERS + 1)
#define RT_COUNTER_WORDS (RT_N_COUNTERS + 2)
enum { RT_GUARD_INDEX = 1, RT_GUARD_STACK = 2, RT_GUARD_ROUNDS = 4 };

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
/* 4-wide node = 8 x float4 = 128 B (one cache line), children in SoA:
     f[0] = lo.x[0..3], f[1] = hi.x[0..3], f[2] = lo.y[0..3], f[3] = hi.y[0..3],
     f[4] = lo.z[0..3], f[5] = hi.z[0..3], f[6] = child[0..3] (int bits), f[7] = 0
   child >= 0: 4-wide node index; child < 0: leaf ~((first << 3) | (count - 1));
   RT_EMPTY_CHILD marks an unused slot.  Collapsed from the binary SAH tree
   (largest-area child expanded first). */
#define RT_EMPTY_CHILD 0x7fffffff
/* Compressed 4-wide node = 12 dwords = 48 B: see rt_quant.h.  The 4-wide trees are
   numbered breadth-first with each node's inner children consecutive, and the
   triangles laid out so each node's leaf children cover consecutive slots. */

struct RtBvh {
    std::vector<float> nodes; /* binary: 16 floats per node */
    std::vector<float> tris;  /* 12 floats per triangle */
    uint32_t n_nodes = 0;
    uint32_t n_leaves = 0;
    uint32_t depth = 0;
    std::vector<float> nodes4;     /* 4-wide: 32 floats per node */
    std::vector<uint32_t> nodes4q; /* 4-wide, compressed: 12 dwords per node (empty: not encodable) */
    uint32_t n_nodes4 = 0;
    uint32_t depth4 = 0;
    uint32_t stack4 = 0; /* worst-case traversal stack entries of the 4-wide tree */
    double build_seconds = 0.0;
    bool cull_unhittable = true; /* in: leave triangles no ray can hit out of the tree (rt_bvh.cpp never_hit) */
    bool det_cull = true;        /* in: normal boxes in the compressed nodes (rt_quant.h determinant cull) */
    std::vector<float> light_centres; /* in: the scene's lights (3 floats each): the cost area leans toward them */
    float light_cost_weight = 0.6f;   /* in: their share of the cost area (rt_bvh.cpp Builder::area) */
    uint32_t n_hit = 0;          /* out: triangles in the tree (slots [0, n_hit)) */
};

/* Builds a binned-SAH BVH over the mesh (rt_bvh.cpp).  Returns false and sets
   err on invalid input. */
bool rt_build_bvh(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris, RtBvh &out,
                  std::string &err);

/* GPU build (rt_build_gpu.hip): LBVH over 63-bit Morton codes collapsed to the 4-wide
   layouts; device buffers owned by the caller afterwards (hipFree).  No binary-tree
   layout is produced.  Returns a hipError_t as int (or -1), err set. */
struct RtGpuBvh {
    float *nodes4 = nullptr;     /* 32 floats per node */
    uint32_t *nodes4q = nullptr; /* 12 dwords per node (nullptr: not encodable) */
    float *tris = nullptr;       /* 12 floats per triangle, leaf order */
    uint32_t n_nodes4 = 0, depth4 = 0, stack4 = 0;
    double build_seconds = 0.0;
};
int rt_build_bvh_gpu(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris, RtGpuBvh &out,
                     std::string &err, void *stream, bool det_cull = true);
/* Input checks shared by both builders (finite coordinates, indices in range, size limit). */
bool rt_validate_mesh(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris, std::string &err);

/* ---- kernel launchers (rt_kernels.hip) ---- */
#ifndef RT_QHEADS
#define RT_QHEADS 8 /* heads of the multi-head pixel queue (k_tris mq_take) */
#endif
#ifndef RT_QSTRIDE
#define RT_QSTRIDE 1024 /* words between the heads (4 KB: apart in the memory channels the device-scope atomics go to) */
#endif
struct RtTriLaunch {
    float *out;
    uint32_t *seeds;
    const float *nodes;
    uint32_t shadow_root; /* the shadow queries' root node (BVH4Q: the lights' tree after the closest-hit tree's nodes; 0: one tree) */
    const float *tris;
    uint32_t n_tris;
    const rt_sphere *lights; /* emissive spheres only, scene order */
    uint32_t n_lights;
    rt_camera cam;
    uint32_t W, H, Wpad, Hpad, Hl;
    uint32_t sample_rate, max_depth, progressive;
    uint32_t stripe, n_ranks, rank;
    const uint32_t *stripe_map; /* tile-local stripe -> the frame's stripe (an owner-map partition,
                                   rt_tile.stripe_owner); NULL: interleaved, (yl / stripe) * n_ranks + rank */
    uint32_t map_key;           /* host only: the serial of stripe_map's contents (0: none), in the schedule key */
    uint32_t *work_counter;
    unsigned long long *counters; /* [RT_COUNTER_WORDS]: the counters, then the guard word (RT_CNT_GUARD) */
    int32_t *spill;      /* per-lane stack overflow (4-wide traversal), spill_cap entries per lane */
    uint32_t spill_cap;
    const uint32_t *tile_order; /* queue position -> 8x8 tile index (NULL: row-major) */
    uint32_t fetch_k;           /* resumable queries: completed lanes that end a stepping round */
    const uint32_t *pixel_flags; /* cost probe per pixel: mesh hits of its probe rays << RT_PROBE_HIT_SHIFT |
                                    their steps (NULL: no probe) */
    uint32_t probe_n;            /* probe rays per pixel: probe_n x probe_n (<= 5) */
    uint32_t fetch_frac;        /* stepping-round exit at ceil(live lanes x fetch_frac / 64) completed
                                   queries when that is below fetch_k (0: fetch_k only) */
    uint32_t diag_pixel;        /* RT_DIAG_ONE_PIXEL builds: yl * W + x of the target pixel, and how many */
    uint32_t diag_k;            /* pixels of its 8 x 8 tile are rendered (from it on, in-tile order) */
    uint32_t *pixel_stats;      /* diagnostics (counting launches, RT_PIXEL_STATS): per pixel 4 x u32 =
                                   start / finish (s_memrealtime, 100 MHz, low 32 bits), queries, steps */
    const int32_t *pixel_class; /* per pixel (W x Hl): -1 mesh pixel, -2 box pixel, >= 0 a long chain's slot
                                   in a sample-split render (NULL: no probe) */
    /* Camera-ray candidate lists (k_pixel_lists): per pixel the triangles any of its sample
       rays could accept, RT_LIST_MAX at most, their records copied into the triangle buffer's
       slots [list_base, list_base + list_cap).  Each 8x8 tile's lists are one block (one
       allocation per pre-pass wave, list_alloc): list_tile[tile] = the block's first slot,
       list_code[pixel] = its list's offset in the block / 8 << 5 | (count - 1) (lists start on
       128-B lines: 8-record multiples from an 8-aligned list_base), or RT_LIST_EMPTY (no
       candidate: no mesh hit possible) or RT_LIST_NONE (no list: the pixel's camera rays take
       the tree).  2 B per pixel + 4 B per tile: small enough to stay in L2 beside the tree. */
    const uint16_t *list_code;
    const uint32_t *list_tile;
    uint32_t list_base;
    uint32_t list_cap;
    uint32_t *list_alloc;
    /* Sample-split tiles: a pixel's random numbers depend only on its closest
       hits, so a seed pass (k_split_seeds) walks every pixel's samples with the closest-hit
       queries alone and stores the seed at the first sample of each chunk; k_tris then renders
       the chunks as independent tasks, each sample's radiance stored, and k_split_finish sums
       them in sample order and writes the pixel and its final seed. */
    uint32_t split_chunks;    /* chunks per pixel of this launch (0: pixels are whole tasks) */
    uint32_t split_chunk;     /* samples per chunk of this launch (a multiple of split_fine) */
    uint32_t split_fine;      /* samples between the stored seeds */
    uint32_t split_nseed;     /* stored seeds per pixel: one per split_fine samples, then the final seed */
    uint32_t *split_seed;     /* per pixel (yl * W + x): split_nseed seeds of 2 words */
    float *split_col;         /* per sample s and pixel p: radiance at ((s * W * Hl) + p) * 3 */
    uint32_t *split_counter;  /* the seed pass's queue cursor */
    uint32_t split_seed_blocks; /* grid of the seed pass */
    uint32_t split_which;     /* RT_SPLIT_ALL, or the mesh pixels / the box pixels of a two-stream split */
    const uint32_t *split_box; /* RT_SPLIT_BOX: the box pixels (yl * W + x), split_n_box of them */
    uint32_t split_n_box;
    uint32_t split_coop;      /* seed pass: lanes per long-chain query, 4 (0: one) */
    uint32_t n_nodes4, n_recs; /* compressed nodes and triangle records (mesh + lists): the cooperative
                                  seed pass checks every index against them */
    uint32_t split_gpw;       /* seed pass: queries (chains) per wave, 0 = all lanes / groups */
    int32_t coop_multi_sp;    /* cooperative seed pass: rounds take 4 stack items while the group's stack holds
                                 at most this many entries, else one (coop_round) */
    /* Speculated mesh pixels: a mesh pixel whose every camera ray hits the mesh
       draws exactly split_spec_draws random numbers per sample (two for the camera ray, two per
       light), so its chunks' first seeds follow from its frame seed by jumping each MWC
       generator ahead (x_{n+k} = a^k x_n mod a 2^16 - 1) — no seed pass.  A chunk that meets a
       camera ray missing the mesh marks the pixel (split_dirty) and lists it (split_repair,
       counted in counters[RT_CNT_REPAIR]) for a repair pass: the long chains' seed pass and
       chunks over that list, whose length they read from split_n_dev. */
    uint32_t split_spec;          /* RT_SPLIT_MESH: the mesh pixels' chunk seeds by jump-ahead */
    uint32_t split_spec_draws;    /* random numbers per sample of a speculated pixel */
    const uint32_t *split_spec_mul; /* per chunk c: a_x^(c chunk D) mod m_x, a_y^(c chunk D) mod m_y */
    const uint32_t *split_run_mul;  /* per lane j < 64: a_x^(j D) mod m_x, a_y^(j D) mod m_y (the repair's runs) */
    uint32_t *split_dirty;        /* per pixel: the first chunk that saw a camera ray miss (~0u: none) */
    uint32_t *split_repair;       /* the marked pixels (yl * W + x) */
    const uint32_t *split_n_dev;  /* RT_SPLIT_BOX: the item count from device memory (NULL: split_n_box) */
    const uint32_t *split_restart; /* the repair pass: per pixel the first chunk (of split_restart_chunk samples)
                                      whose camera ray missed — the chain restarts there from the jumped seed,
                                      the chunks before it stand (NULL: from the frame seed) */
    uint32_t split_restart_chunk;
    uint32_t finish_part; /* k_split_finish: RT_FIN_ALL, or the pixels of one part (pixel_class, split_dirty) */
    uint32_t split_seed_slot; /* RT_SPLIT_BOX: split_seed indexed by the item (the chain's slot in its list, minus
                                 split_item_base: its own buffer, a seed per split_fine samples), not by pixel */
    uint32_t split_item_base, split_item_cap; /* RT_SPLIT_BOX: the items split_box[base ...], at most cap (0: all) */
    /* per pixel the wave's loop iteration at its take ([p]) and at its finish ([W x Hl + p]) — the
       measured cost a view's next schedule is sorted by; a sample-split launch's mesh chunk tasks:
       per pixel and chunk, [p x split_chunks + c] and [W x Hl x split_chunks + ...] (NULL: not
       recorded) */
    uint32_t *pixel_iter;
    uint32_t take_exact; /* k_tris: queue takes of exactly the idle lanes' items, no wave-private batch */
    /* the mesh's bounds padded by 1e-3 of its extent (rt_host.cpp mesh_bounds): a box-path query
       (a bounce off the box or a shadow ray leaving it) whose segment misses them meets no
       triangle and is answered in the path advance, without a traversal (0: not used) */
    uint32_t mesh_bounds;
    float mesh_lo[3], mesh_hi[3];
    uint32_t queue_batch; /* k_tris: items per take from the multi-head queue (mq_take, exact takes when take_exact; work_counter then points
                             at RT_QHEADS heads RT_QSTRIDE words apart); 0: one head (batch_take) */
    /* RT_SPLIT_BOX, slotted seeds, one sample per task: per slot and sample (slot x spp + sample) the
       depth of the segment whose closest-hit query meets the mesh, 0xff for a path that meets only
       the box — written by the subtree-parallel seed pass, which answers that very question for
       every segment; the chunk tasks answer the closest-hit queries above it (box segments: no
       triangle accepted) without a traversal.  NULL: every query traverses. */
    uint8_t *split_hit_depth;
};
enum { RT_SPLIT_ALL = 0, RT_SPLIT_MESH = 1, RT_SPLIT_BOX = 2 };
/* k_split_finish parts: every pixel; a list's pixels (split_box: the long chains, the repaired); the mesh
   pixels no chunk of which missed */
enum { RT_FIN_ALL = 0, RT_FIN_LIST = 1, RT_FIN_MESH = 2 };
#define RT_SEED_COOP4 3 /* split_coop: the 4-lane cooperative seed pass (coop_round) */
#define RT_COOP_STACK (RT_STACK_DEPTH * 4) /* LDS stack entries of a 4-lane query group (k_split_seeds) */
#ifndef RT_LIST_MAX
#define RT_LIST_MAX 64
#endif
#define RT_LIST_NONE 0xffffu
#define RT_LIST_EMPTY 0xfffeu
#if RT_LIST_MAX == 32
#define RT_LIST_BITS 5
#elif RT_LIST_MAX == 64
#define RT_LIST_BITS 6
#else
#error "RT_LIST_MAX: 32 or 64"
#endif
/* list code = (offset in the tile's block / 8) << RT_LIST_BITS | (count - 1): the offset is below
   64 * RT_LIST_MAX, so a code stays below RT_LIST_EMPTY */
static_assert(((64u * RT_LIST_MAX / 8u - 1u) << RT_LIST_BITS | (RT_LIST_MAX - 1u)) < 0xfffeu, "list code range");

struct RtSphLaunch {
    float *out;
    uint32_t *seeds;
    const rt_sphere *spheres;
    uint32_t n_spheres;
    rt_camera cam;
    uint32_t W, H, Wpad, Hpad, Hl;
    uint32_t sample_rate, max_depth, progressive;
    uint32_t stripe, n_ranks, rank;
    const uint32_t *stripe_map; /* as RtTriLaunch::stripe_map */
    unsigned long long *counters;
};

/* All return a hipError_t as int (0 = success). */
/* traversal kinds (kernel template parameter) */
enum { RT_TRAV_LINEAR = 0, RT_TRAV_BVH4 = 2, RT_TRAV_BVH4Q = 4 };

int rt_launch_tris(const RtTriLaunch &a, int trav, bool count, int grid_blocks, void *stream);
/* a render's counters into the host's mapped pinned copy, then the counters and queue cursors
   zeroed for the next render (n_zero 64-bit words from dev) */
int rt_launch_counters_out(unsigned long long *dev, unsigned long long *host_mapped, unsigned long long *totals,
                           uint32_t n_cnt, uint32_t n_zero, void *stream);
/* Sample-split renders: the seed pass (grid a.split_seed_blocks, cursor a.split_counter reset
   first) and the in-order sums; rt_launch_tris runs the chunk tasks (a.split_chunks > 0). */
int rt_launch_split_seeds(const RtTriLaunch &a, void *stream);
int rt_launch_split_finish(const RtTriLaunch &a, void *stream);
int rt_launch_spheres(const RtSphLaunch &a, bool single_sample, void *stream);
int rt_launch_trace_rays(const float *nodes, const float *tris, uint32_t n_tris, const rt_ray *rays, uint32_t n,
                         int any_hit, int trav, int32_t *spill, uint32_t spill_cap, int32_t *out_idx, float *out_t,
                         unsigned long long *counters, void *stream); /* counters: NULL, or counting (queries, nodes, tests, leaves) */
/* Camera-ray candidate lists for the launch's pixels (writes a.pixel_lists and the list
   records in the triangle buffer at a.list_base); nodes4 = full-precision 4-wide tree,
   q4 = compressed nodes (their normal boxes; may be NULL). */
int rt_launch_pixel_lists(const RtTriLaunch &a, const float *nodes4, const uint32_t *q4, uint16_t *codes,
                          uint32_t *tile_base, void *stream);
/* Scheduling probe: per pixel the mesh hits of a grid of probe rays and the traversal steps of
   their queries (rt_kernels.hip). */
int rt_launch_probe_cost(const RtTriLaunch &a, int grid_blocks, uint32_t *out, void *stream);
/* Per stripe of stripe_rows rows of a W x H probe (rt_launch_probe_cost over the whole frame, pn2 rays
   per pixel): out[2 s] = pixels with a probe ray that missed the mesh, out[2 s + 1] = the probe steps
   of the others (rt_partition_stripes) */
int rt_launch_stripe_costs(const uint32_t *probe, uint32_t W, uint32_t H, uint32_t stripe_rows, uint32_t pn2,
                           unsigned long long *out, void *stream);
/* The pixel-queue schedule from the probe, on the device (rt_sched.hip): LPT tile order, box
   flags and their exclusive scan, pixel classes with the long chains' slots. */
struct RtSchedScratch {
    void *tmp = nullptr; /* hipCUB temporary storage */
    size_t tmp_bytes = 0;
    float *keys = nullptr, *keys_sorted = nullptr;
    uint32_t *idx = nullptr;
    uint32_t *box = nullptr, *scan = nullptr; /* npx + 1 entries: scan[npx] = box pixels */
    unsigned long long *sums = nullptr;       /* probe steps, probe hits */
    uint32_t cap_tiles = 0, cap_px = 0;
};
void rt_sched_free(RtSchedScratch &s);
int rt_sched_order(RtSchedScratch &s, const uint32_t *flags, uint32_t W, uint32_t hl, uint32_t pn2, uint32_t n_lights,
                   uint32_t max_depth, uint32_t *order, void *stream);
/* The LPT order again, from a rendered frame's measured costs instead of the probe: per pixel the
   wave iterations it was in flight (iters[p]: the iteration at its take, iters[npx + p]: at its
   finish; k_tris records them; nch > 1: per pixel nch chunk tasks, their iterations summed) */
int rt_sched_order_measured(RtSchedScratch &s, const uint32_t *iters, uint32_t W, uint32_t hl, uint32_t nch,
                            uint32_t *order, void *stream);
/* row > 0 (speculated mesh pixels): the tile's width; the neighbours of a pixel whose probe missed
   the mesh are flagged too */
int rt_sched_box_scan(RtSchedScratch &s, const uint32_t *flags, uint32_t npx, uint32_t pn2, uint32_t step_max,
                      uint32_t row, void *stream);
int rt_sched_classify(const RtSchedScratch &s, uint32_t npx, uint32_t slots, int32_t *cls, uint32_t *slot_pixel,
                      void *stream);
/* Seed-row halo: copy whole rows (both planes) of the seed layout to / from a packed
   buffer [plane][i][x] of 2 * n * wpad words (rows: device array of n row indices). */
int rt_launch_seed_rows(uint32_t *seeds, uint32_t wpad, uint32_t hpad, const uint32_t *rows, uint32_t n,
                        uint32_t *buf, bool unpack, void *stream);
/* Persistent-grid size for the triangle kernel on this device; form: RT_FORM_*. */
enum { RT_FORM_PLAIN = 0, RT_FORM_SPLIT = 1 };
int rt_tris_grid_blocks(int device, int trav, bool count, int form, int *blocks);

#endif /* RT_INTERNAL_H */
