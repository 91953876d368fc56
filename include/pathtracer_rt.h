/*
 * pathtracer_rt.h — C-ABI drop-in boundary of the MI355X path tracer
 * (librtmi.so, built from pathtracer.cl_amd/csrc).
 *
 * It replaces the OpenCL host RayTracerCL (clrt/RayTracerCL.{h,cpp}) and the
 * device-agnostic RayTracer API (clrt/RayTracer.{h,cpp}) for the per-pixel
 * path-tracing kernels of clrt/ocl/raytracer.cl.  Plain pointers and sizes,
 * int status codes, no exceptions and no HIP/torch types in any signature.
 * One context per GPU; a context is not thread-safe (the reference is driven
 * from one GLUT thread, clrt/GlutCLWindow.cpp:136-227).
 *
 * Each entry point names the reference interface it replaces.
 */
#ifndef PATHTRACER_RT_H
#define PATHTRACER_RT_H

#include <stddef.h>
#include <stdint.h>

#include "rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_ctx rt_ctx;

/* Status codes (the reference throws cl::Error, RayTracerCL.cpp:102-107, :297-303). */
enum {
    RT_OK = 0,
    RT_ERR_ARG = -1,      /* bad argument (null pointer, zero size, out of range) */
    RT_ERR_HIP = -2,      /* a HIP runtime call failed; see rt_last_error() */
    RT_ERR_NO_SCENE = -3, /* render requested with no spheres set */
    RT_ERR_NO_MESH = -4,  /* triangle kernel requested with no mesh set */
    RT_ERR_ALLOC = -5,    /* host or device allocation failed */
    RT_ERR_STATE = -6,    /* inconsistent state (e.g. seed layout smaller than the frame) */
    RT_ERR_LIMIT = -7     /* input exceeds a device limit (e.g. BVH deeper than the traversal stack) */
};

/* Kernels of clrt/ocl/raytracer.cl. */
enum {
    RT_KERNEL_SPHERES = 0,    /* raytrace      raytracer.cl:46-104  (row-shifted seeds, sampleRate^2 samples) */
    RT_KERNEL_SPHERES_SS = 1, /* raytrace_ss   raytracer.cl:120-166 (one sample, unshifted seeds) */
    RT_KERNEL_TRIS = 2        /* raytrace_tris raytracer.cl:184-243 (mesh lit by the emissive spheres) */
};

/* Triangle traversal: the reference's linear loop (rtcommon.h:39-68) or a BVH
   (identical results: closest hit = minimum t, ties to the highest index).
   RT_TRAVERSAL_BVH is the 4-wide tree with compressed (8-bit quantised) 64-B
   nodes traversed per lane; RT_TRAVERSAL_BVH4F the same tree with full-precision
   128-B nodes (also the automatic fallback for meshes whose extent the quantised
   grid cannot encode).  Values 2 and 3 (a binary-tree and a wave-coherent packet
   traversal, measured slower) are retired: rt_set_traversal refuses them. */
enum {
    RT_TRAVERSAL_BVH = 0,
    RT_TRAVERSAL_LINEAR = 1,
    RT_TRAVERSAL_BVH4F = 4
};

/* rt_render flags */
enum {
    RT_OUT_DEVICE = 1, /* `out` is a device pointer on the context's GPU (else host memory) */
    RT_SEEDS_HALO = 2  /* the caller keeps the seed rows this tile reads current (seed-row halo,
                          below): permits progressive sphere frames on a tile */
};

/* Row-stripe tile of the frame owned by one rank (multi-GPU sharding).
   The frame's rows are cut into ceil(H / stripe_rows) stripes; stripe s belongs to rank
   stripe_owner[s], or, with stripe_owner NULL, to rank s % n_ranks (interleaved).  A rank's
   rows are rendered compacted in increasing y into `out` (rt_tile_rows() rows of W pixels).
   Seeds are always indexed in the global padded frame (raytracer.cl:207-209), so any
   partition renders the same bits.  NULL tile = full frame.  rt_partition_stripes makes a
   cost-balanced owner map. */
typedef struct rt_tile {
    uint32_t stripe_rows;
    uint32_t n_ranks;
    uint32_t rank;
    const uint32_t *stripe_owner; /* NULL, or ceil(H / stripe_rows) owners, each < n_ranks */
} rt_tile;

/* Ray accounting: one closest-hit query or one any-hit (shadow) query = 1 ray. */
typedef struct rt_counters {
    uint64_t rays_closest;
    uint64_t rays_shadow;
    uint64_t nodes_visited; /* BVH inner nodes fetched (counting launches only) */
    uint64_t tris_tested;   /* ray/triangle tests (counting launches only) */
    uint64_t leaves_visited; /* BVH leaves entered (counting launches only) */
    uint64_t lane_slots;     /* lanes x traversal-step rounds of the resumable (BVH) queries: SIMD
                                efficiency = (nodes_visited + leaves_visited) / lane_slots */
    uint64_t clocks_traversal; /* shader clocks waves spent in traversal rounds, summed over waves */
    uint64_t clocks_total;     /* shader clocks of the waves' whole lifetimes, summed over waves */
    uint64_t pixel_clocks_max; /* the costliest pixel: shader clocks from its refill to its write */
    uint64_t pixel_rays_max;   /* the most queries any one pixel needed */
    uint64_t pixel_steps_max;  /* the most traversal steps any one pixel needed */
    uint64_t rays_skipped;     /* shadow rays (counted in rays_shadow) answered without a
                                  traversal because the answer cannot change the pixel:
                                  tmax <= tmin, or cos(wi) <= 0 (rtcommon.h:93-95) */
    uint64_t clocks_shade;     /* shader clocks waves spent advancing paths (counting launches) */
    uint64_t pixels_long;      /* sample-split render: long chains (box pixels) run on their own stream */
} rt_counters;

/* ---- lifetime: RayTracerCL::RayTracerCL / init / ~RayTracerCL (RayTracerCL.cpp:52-145) ---- */
int rt_create(int device, rt_ctx **out);
int rt_destroy(rt_ctx *ctx);
const char *rt_last_error(const rt_ctx *ctx);
const char *rt_status_string(int status);

/* ---- scene: RayTracer::addSphere / clearSpheres (RayTracer.cpp:50-63) and the
   scene upload of RayTracerCL::rayTrace (RayTracerCL.cpp:251-264) ---- */
int rt_set_spheres(rt_ctx *ctx, const rt_sphere *spheres, uint32_t n);

/* ---- mesh: the tri_verts / tri_vert_idx / n_tris kernel arguments of
   raytrace_tris (raytracer.cl:184-188); the context builds the BVH (the host build's cost area
   leans toward the emissive spheres of the last rt_set_spheres; a later rt_set_spheres keeps the
   tree: culling only, no result depends on it). ---- */
int rt_set_mesh(rt_ctx *ctx, const float *verts_xyz, uint32_t n_verts, const int32_t *idx, uint32_t n_tris);
/* BVH statistics of the current mesh. */
typedef struct rt_mesh_stats {
    uint32_t n_tris;
    uint32_t n_nodes2, depth2; /* binary tree */
    uint32_t n_nodes4, depth4; /* 4-wide tree */
    uint32_t stack4;           /* worst-case traversal stack of the 4-wide tree */
    double build_seconds;
    uint32_t builder; /* RT_BUILD_HOST or RT_BUILD_GPU */
    uint32_t n_tris_tree; /* triangles in the tree: the host build leaves out those no ray can
                             hit (|det| < 1e-4 for every unit direction, geometryFuncs.h:167) */
    uint32_t n_nodes4_shadow; /* the shadow queries' 4-wide tree (host build with lights: its cost
                                 area leans toward them); 0: they walk the closest-hit tree */
} rt_mesh_stats;
/* BVH builder used by the next rt_set_mesh: the host binned-SAH build (default: the best
   trees) or the GPU build (LBVH over Morton codes, collapsed on the device: seconds-to-
   milliseconds for large meshes, somewhat slower traversal).  Results are identical
   either way. */
enum { RT_BUILD_HOST = 0, RT_BUILD_GPU = 1 };
int rt_set_builder(rt_ctx *ctx, int builder);
int rt_mesh_info(const rt_ctx *ctx, rt_mesh_stats *out);

/* ---- camera: RayTracer::setCameraMatrix / setCameraSpherical / setFoVAngle
   (RayTracer.h:56-60, RayTracer.cpp:24-47); the Camera struct is derived per
   frame width exactly as RayTracerCL::updateCLCamera (RayTracerCL.cpp:178-215). ---- */
int rt_set_view_matrix(rt_ctx *ctx, const float m_colmajor[16]);
int rt_set_camera_spherical(rt_ctx *ctx, float tx, float ty, float tz, float elevation_deg, float azimuth_deg,
                            float distance);
int rt_set_fov(rt_ctx *ctx, float fov_deg);
/* Explicit Camera override (fixtures); cleared by the three calls above. */
int rt_set_camera(rt_ctx *ctx, const rt_camera *cam);
/* Host helper: the Camera the reference would upload for this setup and width. */
int rt_camera_spherical(float tx, float ty, float tz, float elevation_deg, float azimuth_deg, float distance,
                        float fov_deg, uint32_t width, rt_camera *out);

/* ---- settings: RayTracer::setSampleRate / setMaxPathDepth (RayTracer.h:62-66) ---- */
int rt_set_params(rt_ctx *ctx, uint32_t sample_rate, uint32_t max_depth);
int rt_set_traversal(rt_ctx *ctx, int traversal);

/* ---- RNG seeds: RayTracerCL::updateSeedBuffer (RayTracerCL.cpp:147-171).
   Work-group height ndY fixes the padded height (RayTracerCL.cpp:114-116,
   :229-232; 8 = a 256-item work-group on AMD GPUs, the default). ---- */
int rt_set_ndrange(rt_ctx *ctx, uint32_t nd_y);
/* Allocate a Wpad x Hpad layout filled from the context's glibc-rand() stream
   (glibc TYPE_3 random(), default seed 1 — no srand in the reference). */
int rt_set_seed_layout(rt_ctx *ctx, uint32_t wpad, uint32_t hpad);
/* Replace the seeds: count == 2 * Wpad * Hpad (x plane then y plane). */
int rt_set_seeds(rt_ctx *ctx, const uint32_t *seeds, size_t count);
int rt_get_seeds(const rt_ctx *ctx, uint32_t *out, size_t count);
int rt_seed_layout(const rt_ctx *ctx, uint32_t *wpad, uint32_t *hpad);
/* Seed-row halo for multi-GPU progressive sphere frames.  raytrace reads and writes
   seed row (y + progressive) % Hpad for pixel row y (get_seed / put_seed,
   raytracer.cl:20-30), so between frames one seed row per stripe boundary moves to
   the neighbouring rank.  These copy whole rows (both planes) of the context's seed
   layout to / from a packed buffer laid out [plane][i][x] (2 * n * Wpad words);
   `buf` is a device pointer with RT_OUT_DEVICE in flags, else host memory.  The
   rows to move are planned by pathtracer.cl_amd/dist.py (SeedHalo). */
int rt_pack_seed_rows(rt_ctx *ctx, const uint32_t *rows, uint32_t n, uint32_t *buf, int flags);
int rt_unpack_seed_rows(rt_ctx *ctx, const uint32_t *rows, uint32_t n, const uint32_t *buf, int flags);
/* glibc rand() stream restated (tests compare it with libc's own rand()). */
int rt_glibc_rand_fill(uint32_t seed, uint32_t *out, size_t count, uint32_t skip);

/* ---- render: RayTracerCL::rayTrace(cl_mem*, W, H, progression) (RayTracerCL.cpp:217-307).
   progression 0 overwrites; p > 0 mixes with weight 1/p (GlutCLWindow.cpp:144-158).
   Pads the frame, (re)creates seeds on a size change and refreshes the camera
   exactly as the reference does, then launches and waits (finish()). ---- */
int rt_render(rt_ctx *ctx, float *out_rgba, uint32_t width, uint32_t height, uint32_t progression, int kernel,
              const rt_tile *tile, int flags);
/* Same, enqueued on `hip_stream` (a hipStream_t, or NULL = the context stream), no wait. */
int rt_render_async(rt_ctx *ctx, float *out_rgba, uint32_t width, uint32_t height, uint32_t progression,
                    int kernel, const rt_tile *tile, int flags, void *hip_stream);
int rt_synchronize(rt_ctx *ctx);
/* Blocking readback of the last render's framebuffer (W x rows x 4 floats) into host
   memory: the non-sharing display path, enqueueReadBuffer(clPBOBuff, CL_TRUE, ...)
   into the mapped PBO (GlutCLWindow.cpp:214-225).  Valid while the buffer passed to
   that render (device framebuffers) is alive.  n_floats = capacity of `host`. */
int rt_read(rt_ctx *ctx, float *host, size_t n_floats);
/* Rows of `height` owned by `tile` (NULL: height). */
uint32_t rt_tile_rows(uint32_t height, const rt_tile *tile);
/* Cost-balanced partition of a W x H raytrace_tris frame's row stripes over n_ranks for the
   context's current camera, mesh and lights (the multi-GPU split; the reference renders on one
   device, RayTracerCL.cpp:217-307).  A probe of the whole frame — one camera ray per pixel
   through the compressed tree, and its shadow rays — counts per stripe the pixels whose camera
   ray misses the mesh (box pixels: the long serial chains of a tile) and the
   probe's traversal steps of the others; the stripes are dealt largest cost first to the least
   loaded rank (LPT; ties to the lower stripe and rank index).  Deterministic: every rank
   computes the same map from the same scene.  Cached per view (camera, mesh, lights, frame
   shape).  owner: ceil(H / stripe_rows) entries.  *recomputed (may be NULL) = 1 when the probe
   ran, 0 when the cached map was returned. */
int rt_partition_stripes(rt_ctx *ctx, uint32_t width, uint32_t height, uint32_t stripe_rows, uint32_t n_ranks,
                         uint32_t *owner, int *recomputed);

/* ---- instrumentation ---- */
int rt_get_counters(const rt_ctx *ctx, rt_counters *out); /* of the last completed render (or counting rt_trace_rays call) */
int rt_set_counting(rt_ctx *ctx, int enable);             /* count nodes/tris in the next renders */
/* Running totals over every render since the context was created or the totals were last reset
   (renders enqueued back to back with rt_render_async overwrite each other's rt_get_counters;
   their totals are kept on the device): waits for the context's renders, then sums of the summed
   counters, maxima of the per-pixel maxima (pixels_long: 0), *renders = renders counted.
   reset != 0 zeroes the totals after reading them.  RT_ERR_STATE if a sample-split defect guard
   fired in any of those renders (rt_synchronize reports only the last one's). */
int rt_counter_totals(rt_ctx *ctx, rt_counters *sum, uint64_t *renders, int reset);
/* Device time of the last render's kernel (HIP events on the launch stream), ms. */
int rt_last_kernel_ms(const rt_ctx *ctx, float *ms);
/* The same time split at the start of the main path kernel: the camera-ray candidate-list
   pre-pass of a triangle render (0 without one), then k_tris (+ a sample-split render's seed
   passes and in-order sums), ms. */
int rt_last_kernel_split_ms(const rt_ctx *ctx, float *prepass_ms, float *main_ms);

/* What the last render did beyond the reference's launch (the triangle kernel's own
   machinery; none of it changes a result bit). */
typedef struct rt_render_info {
    uint32_t kernel;           /* RT_KERNEL_* of the last render */
    uint32_t traversal;        /* internal traversal kind of a triangle render */
    uint32_t grid_blocks;      /* persistent grid of the main kernel */
    uint32_t lists;            /* 1: camera-ray candidate lists were built and used */
    uint64_t list_capacity;    /* list-area records (48 B each) reserved for the render */
    uint64_t list_records;     /* records the pixels' lists took (read on the first call) */
    uint32_t list_pixels_tree; /* pixels without a list (over RT_LIST_MAX candidates, a deep
                                  frustum stack, or the area full): their camera rays took the tree */
    uint32_t pixels_long;      /* sample-split render: long chains (box pixels) run on their own stream */
    uint32_t schedule_rebuilt; /* 1: the cost probe, LPT order and pixel classes were recomputed
                                  (camera, mesh, frame, tile or parameters changed) */
    uint32_t lists_rebuilt;    /* 1: the lists were built for this render (0: the previous render's,
                                  same camera, mesh, frame and tile, were reused) */
    double schedule_host_ms;   /* host time spent enqueueing / sizing the schedule this render */
    uint32_t split_chunks;     /* sample-split render (a tile with few pixels per lane): chunks per
                                  pixel, each an independent task seeded by the seed pass; 0: whole pixels */
    uint32_t split_coop;       /* lanes per query of the long chains' seed pass (4: coop_round; 0: one) */
    uint32_t split_guard;      /* read after completion: a defect guard of the long chains' seed pass
                                  fired (record index out of range, group stack overflow, query round
                                  bound); rt_synchronize then fails with RT_ERR_STATE */
    uint32_t split_spec;       /* 1: the mesh pixels' chunk seeds were jumped ahead from their frame
                                  seeds (no seed pass for them; pixels near a silhouette run as long chains) */
    uint32_t split_repaired;   /* read after completion: speculated pixels whose camera rays missed the
                                  mesh after all, re-rendered by the repair pass (seed pass + chunks) */
    uint32_t split_hit_depth;  /* 1: the long chains' chunk tasks answered their box segments' closest-hit
                                  queries from the seed pass's per-sample mesh-hit depths (no traversal) */
    uint32_t schedule_measured; /* 1: the queue's tiles were ordered by the view's previous frame's measured
                                   per-pixel costs (its traversal steps), not by the cost probe */
    uint32_t schedule_pilot;    /* 1: a view's first frame, ordered by the per-pixel costs of a pilot render of
                                   a few samples per pixel (scratch seeds and framebuffer), not by the probe */
} rt_render_info;
int rt_last_render_info(rt_ctx *ctx, rt_render_info *out);
/* The long chains of the last sample-split render (pixels_long of them: tile-local y * W + x, the
   order of their slots), the pixels whose seed pass ran on the second stream with split_coop lanes
   per query.  Copies min(cap, *n) entries; *n = pixels_long.  Diagnostics and parity tests. */
int rt_last_long_chains(rt_ctx *ctx, uint32_t *out, uint32_t cap, uint32_t *n);

/* ---- ray queries for hit-index parity (rtcommon.h:39-52 / :59-68 semantics).
   Host arrays; any_hit=0: out_idx = closest triangle (-1 none), out_t = its t;
   any_hit=1: out_idx = 1 if occluded in (tmin, tmax). ---- */
int rt_trace_rays(rt_ctx *ctx, const rt_ray *rays, uint32_t n, int any_hit, int32_t *out_idx, float *out_t);

/* ---- synthetic meshes (deterministic, host-independent: rt_math.h only) ----
   A displaced lat-long sphere truncated to exactly n_tris triangles, centred at
   (cx, cy, cz) with base radius r.  verts must hold rt_mesh_vertex_count(n_tris)
   xyz triples, idx 3*n_tris ints. */
uint32_t rt_mesh_vertex_count(uint32_t n_tris);
int rt_make_mesh(uint32_t n_tris, float cx, float cy, float cz, float r, float *verts_xyz, int32_t *idx);

/* ---- PLY meshes: PLYLoader (clrt/PLYLoader.cpp:4-90) over ply.c (ply.c:2457-2720).
   ascii / binary_little_endian / binary_big_endian; vertex x, y, z as float32, face
   `vertex_indices` lists (polygons fan-triangulated, < 3 vertices dropped, indices
   range-checked — the reference copies only 2-vertex faces, PLYLoader.cpp:74); other
   properties and elements skipped.  open decodes the file and reports the counts;
   read copies into caller buffers (3*n_verts floats, 3*n_tris ints). ---- */
typedef struct rt_ply rt_ply;
int rt_ply_open(const char *path, rt_ply **out, uint32_t *n_verts, uint32_t *n_tris);
int rt_ply_read(const rt_ply *ply, float *verts_xyz, int32_t *idx);
uint32_t rt_ply_dropped_faces(const rt_ply *ply);
int rt_ply_close(rt_ply *ply);
const char *rt_ply_last_error(void); /* message of the last failed rt_ply_open (this thread's process) */
/* Scale uniformly to `max_extent` on the longest axis, centre x and z on 0 and rest the
   lowest point on y = floor_y (extent 3 on the box floor y = -5). */
int rt_normalize_mesh(float *verts_xyz, uint32_t n_verts, float max_extent, float floor_y);

/* ---- multi-GPU from the native host: one process (or thread) per GPU, RCCL over
   xGMI.  The reference renders on one OpenCL device (RayTracerCL.cpp:52-145,
   :217-307); this is the sharded form of the same rayTrace call, with no data-path
   exchange (pixels are independent) besides the frame assembly, plus the seed-row
   halo of progressive sphere frames.  A communicator is created collectively:
   rank 0 makes the id, the caller hands the bytes to every rank by any channel
   (MPI, a file, a TCP store), each rank calls rt_comm_create with its own GPU. ---- */
typedef struct rt_comm rt_comm;
#define RT_COMM_ID_BYTES 128
/* ncclGetUniqueId (rccl.h:187). */
int rt_comm_get_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
/* ncclCommInitRank (rccl.h:215) on `device`; collective over n_ranks callers. */
int rt_comm_create(const uint8_t id[RT_COMM_ID_BYTES], int n_ranks, int rank, int device, rt_comm **out);
int rt_comm_destroy(rt_comm *comm);
const char *rt_comm_last_error(const rt_comm *comm);
/* ncclCommCount (rccl.h:378): ranks in the communicator as RCCL sees them. */
int rt_comm_count(const rt_comm *comm, int *n_ranks);
/* Frame assembly (collective): every rank passes its compact tile (device pointer,
   rt_tile_rows(H, {stripe, n_ranks, rank, stripe_owner}) rows of W RGBA32F pixels); `root`
   receives them with grouped ncclSend/ncclRecv (one point-to-point xGMI transfer per sender)
   and scatters the stripes into `frame_dev` (device, W*H*4 floats; others: ignored).
   stripe_owner: the partition the tiles were rendered with (NULL: interleaved). */
int rt_comm_gather_frame(rt_comm *comm, const float *tile_dev, float *frame_dev, uint32_t width, uint32_t height,
                         uint32_t stripe_rows, const uint32_t *stripe_owner, int root);
/* Device-side assembly on one GPU: n_ranks compact tiles (device pointers, rank
   order) scattered into frame_dev (the root's step of rt_comm_gather_frame). */
int rt_assemble_tiles(const float *const *tiles_dev, uint32_t n_ranks, uint32_t width, uint32_t height,
                      uint32_t stripe_rows, const uint32_t *stripe_owner, float *frame_dev, int device);
/* Seed-row halo plan (host only).  writer[Hpad]: last rank that wrote each seed row
   (-1: nobody, the initial seeds are identical on every rank).  Before a raytrace
   frame with row shift `progressive` under the partition (stripe_rows, n_ranks,
   stripe_owner: NULL = interleaved), lists the moves (src rank, dst rank, seed row) that
   bring every row a rank reads up to date — including rows whose stripe changed owner since
   it was written; then records the frame's writes in writer.  Capacity of the three output
   arrays: height entries. */
int rt_seed_halo_plan(int32_t *writer, uint32_t height, uint32_t hpad, uint32_t stripe_rows, uint32_t n_ranks,
                      const uint32_t *stripe_owner, uint32_t progressive, uint32_t *src, uint32_t *dst,
                      uint32_t *rows, uint32_t *n_moves);
/* One rank's side of a halo plan (host only): the rows `me` sends to each peer and receives
   from each peer, as one packed block per peer in peer order — send_rows holds the blocks to
   peers 0, 1, ... back to back (send_counts[p] rows to peer p), likewise recv_rows /
   recv_counts.  Row order within a block is the plan's, so peer p's send block to `me` and
   my receive block from p list the same rows in the same order (the packed buffers match
   word for word).  Capacity of send_rows / recv_rows: n_moves; of the counts: n_ranks. */
int rt_seed_halo_peer_blocks(const uint32_t *src, const uint32_t *dst, const uint32_t *rows, uint32_t n_moves,
                             uint32_t n_ranks, uint32_t me, uint32_t *send_rows, uint32_t *send_counts,
                             uint32_t *recv_rows, uint32_t *recv_counts);
/* One sharded rayTrace (collective): rank renders its stripes into a tile buffer the
   communicator keeps (progression mixes into it across frames), first brings the seed rows
   it reads up to date from their last writers (the seed-row halo: grouped ncclSend/ncclRecv
   of packed rows; raytrace shifts rows by the progression, the other kernels read row y,
   which after progressive sphere frames another rank may have written last), then
   gathers the frame to `root` (frame_dev: device, W*H*4 floats on root).  Bit-identical
   to rt_render of the whole frame on one GPU.  Call rt_comm_reset_halo after replacing
   a context's seeds (rt_set_seeds).  The stripes are dealt by the communicator's partition
   (rt_comm_set_partition). */
int rt_comm_render(rt_comm *comm, rt_ctx *ctx, float *frame_dev, uint32_t width, uint32_t height,
                   uint32_t progression, int kernel, uint32_t stripe_rows, int root);
int rt_comm_reset_halo(rt_comm *comm);
/* Partition of rt_comm_render's frames: RT_PARTITION_INTERLEAVED (stripe s to rank
   s % n_ranks) or RT_PARTITION_BALANCED (the default: raytrace_tris frames by
   rt_partition_stripes, computed by every rank for each new view, every rank then taking the
   root's map from one broadcast; sphere frames stay interleaved).  A change of owner moves the
   stripe's seed rows through the halo (rt_seed_halo_plan).  rt_comm_last_partition copies
   the last frame's owner map (cap entries; *n = its stripes). */
enum { RT_PARTITION_INTERLEAVED = 0, RT_PARTITION_BALANCED = 1 };
int rt_comm_set_partition(rt_comm *comm, int mode);
int rt_comm_last_partition(const rt_comm *comm, uint32_t *owner, uint32_t cap, uint32_t *n);

#ifdef __cplusplus
}
#endif

#endif /* PATHTRACER_RT_H */
