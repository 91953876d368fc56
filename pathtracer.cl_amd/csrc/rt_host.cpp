/*
 * rt_host.cpp — the C-ABI host runtime (librtmi.so), MI355X replacement of
 * the reference's OpenCL host RayTracerCL (clrt/RayTracerCL.cpp) and of the
 * device-agnostic RayTracer settings (clrt/RayTracer.cpp).
 *
 * Owns per context: the HIP stream and events, the scene (spheres, the
 * emissive subset for the triangle kernel), the mesh BVH, the seed planes, the
 * camera derivation and the launch of the kernels in rt_kernels.hip.  There is
 * no CPU fallback: every render runs the HIP kernels or returns an error.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "pathtracer_rt.h"
#include "rt_internal.h"
#include "rt_math.h"
#include "rt_quant.h"

namespace {

/* glibc random() TYPE_3 (the generator behind rand(), seeded with 1 when the
   program never calls srand — the reference never does).  Published algorithm:
   r[0] = seed; r[i] = 16807 r[i-1] mod (2^31-1) for i < 31; r[i] = r[i-31]
   for 31 <= i < 34; then r[i] = r[i-31] + r[i-3] (mod 2^32) and the outputs
   are r[i] >> 1 from i = 344 on. */
struct GlibcRand {
    uint32_t r[34];
    int k = 0;
    void seed(uint32_t s)
    {
        int32_t w[344 + 34];
        if (s == 0) s = 1;
        w[0] = (int32_t)s;
        for (int i = 1; i < 31; ++i) {
            const int64_t v = (16807LL * w[i - 1]) % 2147483647LL;
            w[i] = (int32_t)(v < 0 ? v + 2147483647LL : v);
        }
        for (int i = 31; i < 34; ++i) w[i] = w[i - 31];
        uint32_t u[344];
        for (int i = 0; i < 34; ++i) u[i] = (uint32_t)w[i];
        for (int i = 34; i < 344; ++i) u[i] = u[i - 31] + u[i - 3];
        for (int i = 0; i < 34; ++i) r[i] = u[310 + i]; /* last 34 values, oldest first */
        k = 0;
    }
    uint32_t next()
    {
        /* r holds the last 34 values in a ring starting at k (oldest) */
        const uint32_t v = r[(k + 34 - 31) % 34] + r[(k + 34 - 3) % 34];
        r[k] = v;
        k = (k + 1) % 34;
        return v >> 1;
    }
};

const char *hip_str(hipError_t e) { return hipGetErrorString(e); }

constexpr double kPi = 3.14159265358979323846; /* M_PI */

/* Scheduling constants of the triangle kernel, each swept on the dragon frame (DESIGN.md §5;
   results are independent of all of them):
     kProbeN    cost-probe rays per pixel, kProbeN x kProbeN;
     kFetchK    completed queries that end a wave's stepping round (12 / 16 / 20 / 24 / 32 / 40:
                166.8 / 163.9 / 163.0 / 162.3 / 163.9 / 168.2 ms); the same for waves holding
                box pixels (8 / 16 / 24 within 0.5 %);
     kFetchFrac the stepping round also ends at ceil(live lanes x kFetchFrac / 64) completed
                queries (r02 A/B: full frame 162.8 -> 160.6 ms, slowest 8-way tile 219 -> 107 ms). */
constexpr uint32_t kProbeN = 2;
/* a 1-spp frame traces fewer rays than a 2x2 probe would: one probe ray per pixel there (bunny
   class 1024^2 at 1 spp: a camera move cost 2.2 ms against a 1.0 ms frame with the 2x2 probe) */
uint32_t probe_n(uint32_t sample_rate) { return sample_rate >= 2 ? kProbeN : 1u; }
#ifndef RT_FETCH_K
#define RT_FETCH_K 24
#endif
constexpr size_t kCounterBytes = RT_COUNTER_WORDS * sizeof(unsigned long long);
/* the queue cursors after the counters: the main launch's RT_QHEADS heads RT_QSTRIDE words apart (mq_take),
   then the long chains' and the repairs' one-word cursors on lines of their own */
constexpr size_t kWorkWords = (size_t)RT_QSTRIDE * RT_QHEADS + 64;
constexpr uint32_t kWorkBox = RT_QSTRIDE * RT_QHEADS, kWorkRepair = RT_QSTRIDE * RT_QHEADS + 32;
#ifndef RT_LONG_FINE
#define RT_LONG_FINE 1 /* samples per stored seed (and per chunk task) of the subtree-parallel long chains */
#endif
#ifndef RT_REPAIR_WIDTH
#define RT_REPAIR_WIDTH 64u /* lanes per repaired chain: its hit samples in runs of 63 */
#endif
#ifndef RT_QUEUE_BATCH
#define RT_QUEUE_BATCH 64
#endif
#ifndef RT_REPAIR_SLOTS
#define RT_REPAIR_SLOTS 4096u /* repaired pixels with per-sample seeds by slot (8.4 MB at 256 spp) */
#endif
#ifndef RT_BOX_GRID_DIV
#define RT_BOX_GRID_DIV 4 /* the long chains' seed pass takes at most 1/RT_BOX_GRID_DIV of the persistent grid */
#endif
#ifndef RT_SEED_GRID_ITEMS
#define RT_SEED_GRID_ITEMS 1
#endif
constexpr uint32_t kFetchK = RT_FETCH_K;
constexpr uint64_t kShortFrameSamplesPerLane = 8; /* below: a short frame (fewer blocks per CU) */
constexpr int kShortFrameBlocksPerCU = 3;
/* the pilot render (pilot_order) only for frames of at least this many samples per pixel: its 4 spp
   are 1.6 % of a 256-spp frame, but a quarter of the Lucy class's 16-spp frame (133 against 506 ms,
   profiles/r06f), which keeps the probe's order */
constexpr uint32_t kPilotMinSpp = 64;
/* an unsigned environment knob (tuning sweeps), `def` when unset or unparsable */
uint32_t env_u32(const char *name, uint32_t def)
{
    const char *v = getenv(name);
    if (!v || !*v) return def;
    char *end = nullptr;
    const unsigned long x = strtoul(v, &end, 10);
    return (end && *end == 0) ? (uint32_t)x : def;
}
constexpr uint32_t kFetchFrac = 24;

} // namespace

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evm = nullptr; /* evm: the main kernel's start */
    std::string err;

    /* scene */
    std::vector<rt_sphere> spheres;
    std::vector<rt_sphere> lights;
    rt_sphere *d_spheres = nullptr;
    rt_sphere *d_lights = nullptr;

    /* mesh */
    RtBvh bvh;
    float *d_nodes4 = nullptr; /* 4-wide tree */
    uint32_t *d_nodes4q = nullptr; /* 4-wide tree, compressed nodes */
    float *d_tris = nullptr;
    size_t tris_cap = 0;       /* triangle records d_tris holds (mesh + camera-ray candidate lists) */
    size_t tree_recs = 0;      /* of them the trees' triangle records: n_tris, or 2 n_tris with the shadow tree */
    uint32_t shadow_root = 0;  /* the shadow queries' tree: its root node in d_nodes4q (0: the closest-hit tree) */
    uint32_t n_nodes4_shadow = 0, stack4_all = 0;
    uint16_t *d_list_code = nullptr;  /* per pixel: offset in its tile's block << 5 | count - 1 (k_pixel_lists) */
    uint32_t *d_list_tile = nullptr;  /* per 8x8 tile: first slot of its block of lists */
    uint32_t *d_list_alloc = nullptr; /* the list area's allocator */
    size_t list_px_cap = 0, list_tile_cap = 0;
    int pixel_lists = -1; /* RT_PIXEL_LISTS: 0 off, 1 on, unset: on for sampleRate >= 4 (the pre-pass
                             costs about a traversal per pixel: a 1-spp frame does not repay it) */
    size_t list_mb = 4096; /* RT_LIST_MB: device memory of the list area (pixels beyond it take the tree) */
    std::vector<uint32_t> list_key; /* what the lists in the list area were built for (empty: none) */
    uint64_t list_used_last = 0, list_cap_last = 0, list_npx_last = 0; /* the last list build: records taken /
                                                                          given, its pixels */
    std::vector<uint32_t> last_view; /* the previous triangle render's view (camera, mesh, frame, tile) */
    uint32_t n_tris = 0;
    int32_t *d_spill = nullptr; /* per-lane stack overflow for the 4-wide traversal */
    uint32_t *d_order = nullptr; /* pixel-queue tile order (expensive tiles first) */
    uint32_t order_cap = 0;
    uint32_t *d_flags = nullptr; /* cost probe per pixel (k_probe_cost) */
    RtSchedScratch sched;        /* the device-side schedule (rt_sched.hip) */
    int32_t *d_class = nullptr;  /* per pixel: -1 mesh, -2 box, >= 0 a long chain's slot (sample-split) */
    size_t class_bytes = 0;
    size_t split_mb = 16384; /* RT_SPLIT_MB: device memory cap of the sample-split buffers */
    /* sample-split tiles (k_split_seeds -> k_tris chunks -> k_split_finish) */
    int split = -1;                   /* RT_SPLIT: 1 on, 0 off, unset = auto (split_wanted) */
    /* the long chains' seed pass with 4 lanes per query (one lane per query: 8-way tile 24 -> 19 ms
       for the chains); 4 x 4 probe rays per pixel to find them */
    uint32_t seed_width = 0; /* lanes per long chain in the seed pass: 8-64 subtree-parallel (k_chain_seeds), 3 coop_round,
                                1 one lane, 0 by the launch (seed_width_auto) */
    uint32_t split_probe = 4;
    uint32_t split_nch = 16;   /* sample-split: chunk tasks per pixel, about (8 / 13 / 32 no faster, profiles/r05ba) */
    uint32_t *d_split_seed = nullptr; /* per pixel and chunk: the seed at the chunk's first sample */
    float *d_split_col = nullptr;     /* per sample and pixel: its radiance */
    uint32_t *d_split_counter = nullptr; /* [0]: the seed pass's cursor, [32]: the box pixels' (own line) */
    size_t split_seed_bytes = 0, split_col_bytes = 0;
    uint32_t *d_split_box = nullptr;  /* the box pixels (yl * W + x): their chains run on stream2 */
    uint32_t *d_long_seed = nullptr;  /* the long chains' seeds by slot, one per RT_LONG_FINE samples */
    size_t long_seed_bytes = 0;
    uint32_t *d_repair_seed = nullptr; /* the repaired pixels' seeds by slot (the first RT_REPAIR_SLOTS of them) */
    size_t repair_seed_bytes = 0;
    uint32_t repair_slots = RT_REPAIR_SLOTS; /* RT_REPAIR_SLOTS (env, test knob): repaired pixels with per-sample seeds */
    bool last_hit_depth = false; /* the last sample-split render used split_hit_depth */
    size_t split_box_cap = 0;
    uint32_t n_split_box = 0;
    int split_box_grid = 0;           /* the box pixels' seed-pass grid of the render being launched */
    hipStream_t stream2 = nullptr;    /* the box pixels' seed pass and chunks, beside the mesh pixels' */
    /* speculated mesh pixels (RT_SPLIT_SPEC, default on): their chunk seeds jumped ahead from the
       frame seeds; a per-pixel mark and the list of the pixels to repair */
    int split_spec = 1;
    uint32_t *d_split_dirty = nullptr, *d_split_repair = nullptr;
    size_t split_dirty_px = 0;
    uint32_t *d_spec_mul = nullptr;   /* per chunk: the two generators' jump multipliers */
    std::vector<uint32_t> h_spec_mul; /* their host copy (the upload's source; re-uploaded on change) */
    uint64_t spec_mul_key = ~0ull;
    hipEvent_t ev_split0 = nullptr, ev_box = nullptr, ev_mesh = nullptr, ev_fin3 = nullptr;
    hipStream_t stream3 = nullptr;    /* the clean mesh pixels' in-order sums, beside the repair pass */
    uint32_t *d_halo_rows = nullptr; /* seed-row halo: row indices */
    uint32_t *d_halo_buf = nullptr;  /* seed-row halo: staging for host buffers */
    size_t halo_rows_cap = 0, halo_buf_cap = 0;
    size_t flags_bytes = 0;
    std::vector<uint32_t> order_key; /* what the cached order was computed for */
    bool schedule = true;
    bool schedule_rebuilt = false; /* the last triangle render recomputed the schedule */
    /* measured-cost schedule (whole-pixel frames and sample-split tiles of >= 16 samples per pixel):
       a view's first frame records each pixel's traversal steps (pixel_iter; a split tile's mesh chunk
       tasks), its next frame re-sorts the tiles by them */
    uint32_t *d_pixel_iter = nullptr;
    size_t pixel_iter_px = 0;
    bool iter_recorded = false;  /* this view's costs are in d_pixel_iter */
    bool order_measured = false; /* d_order is sorted by them (once per view: re-sorting again from
                                    the re-sorted frame's costs measured slower, profiles/r05aa) */
    uint32_t iter_nch = 1;       /* chunk tasks per pixel of the recorded frame (1: whole pixels) */
    float mesh_lo[3] = {0, 0, 0}, mesh_hi[3] = {0, 0, 0}; /* the mesh's padded bounds (mesh_bounds) */
    bool mesh_bounds_ok = false;
    rt_render_info info = {};      /* rt_last_render_info */
    bool info_list_pending = false; /* info.list_records / list_pixels_tree still to be read */
    size_t info_list_px = 0;        /* pixels of the render the pending list counts belong to */
    int builder = RT_BUILD_HOST;      /* builder for the next rt_set_mesh */
    int mesh_builder = RT_BUILD_HOST; /* builder of the current mesh */
    uint64_t mesh_serial = 0;
    size_t spill_entries = 0;
    /* owner-map tiles (rt_tile.stripe_owner): the tile's frame stripes in order, on the device, and a
       serial that changes with them (in the view / schedule keys) */
    std::vector<uint32_t> stripe_map_h;
    uint32_t *d_stripe_map = nullptr;
    size_t stripe_map_cap = 0;
    uint32_t stripe_map_serial = 0;
    /* the pilot render of a view's first frame (pilot_order): its seeds, framebuffer and counters +
       queue cursors, apart from the frame's */
    int pilot_sr = 2; /* RT_PILOT (test knob): the pilot's sampleRate, 0 = no pilot (the probe's order) */
    uint32_t *d_pilot_seeds = nullptr;
    float *d_pilot_out = nullptr;
    unsigned long long *d_pilot_cnt = nullptr;
    size_t pilot_seed_words = 0, pilot_out_floats = 0;
    /* rt_partition_stripes: the last map and what it was computed for */
    std::vector<uint32_t> part_key, part_owner;
    uint32_t *d_part_probe = nullptr;
    unsigned long long *d_part_cost = nullptr;
    size_t part_probe_px = 0, part_cost_cap = 0;

    /* camera state (RayTracer.h:21-29) */
    float view[4][4]; /* viewMatrix, row-major; identity by default (gmtl) */
    float fov = 53.0f; /* RayTracer() default, RayTracer.cpp:18 */
    bool cam_override = false;
    rt_camera cam_explicit;
    bool cam_dirty = true;
    rt_camera cam;
    uint32_t width = 0, height = 0;

    /* settings: RayTracer() defaults (RayTracer.cpp:16-22) */
    uint32_t sample_rate = 8, max_depth = 4;
    int traversal = RT_TRAVERSAL_BVH;
    uint32_t nd_y = 8;
    bool counting = false;

    /* seeds */
    GlibcRand rng;
    uint32_t wpad = 0, hpad = 0;
    bool user_seeds = false;
    uint32_t *d_seeds = nullptr;

    /* scratch */
    uint32_t *d_work = nullptr;                 /* queue cursors: inside the d_counters allocation, after the counters */
    unsigned long long *d_counters = nullptr;   /* RT_COUNTER_WORDS counters + guard, then the kWorkWords cursor words */
    unsigned long long *h_counters = nullptr;   /* pinned: the counters (+ the list area's fill) copied back on the render's stream */
    unsigned long long *h_counters_dev = nullptr; /* its device address (mapped): k_counters_out writes it */
    bool counters_zeroed = false;                 /* the last render ended with k_counters_out: no fill needed */
    unsigned long long *d_totals = nullptr;     /* running totals over renders (k_counters_out; rt_counter_totals) */
    hipStream_t sync_stream = nullptr;          /* the stream of the last render (rt_synchronize waits on it) */
    hipEvent_t ev_done = nullptr;               /* the end of the last render's counter hand-back: a render on another
                                                   stream waits for it (the counters, the queue cursors).  Recorded at
                                                   the render's end on a caller's stream (which may be gone later), and
                                                   only when needed on the context's own (no per-frame record there) */
    float *d_stage = nullptr;
    size_t stage_bytes = 0;
    rt_counters last = {};
    uint32_t last_long = 0; /* long chains run apart by the last triangle launch (sample-split) */
    bool have_timing = false;
    const float *last_out = nullptr; /* device framebuffer of the last render (rt_read) */
    size_t last_bytes = 0;
    /* persistent-grid size per (traversal kind, counting, kernel form): index (trav * 2 + count) * 3 + form */
    int grid_cache[6 * (RT_TRAV_BVH4Q + 1)] = {};
};

namespace {

int fail(rt_ctx *c, int code, const std::string &msg)
{
    if (c) c->err = msg;
    return code;
}

int hip_fail(rt_ctx *c, hipError_t e, const char *what)
{
    return fail(c, RT_ERR_HIP, std::string(what) + ": " + hip_str(e));
}

#define HIPCHK(ctx, call)                                                                                              \
    do {                                                                                                               \
        hipError_t e_ = (call);                                                                                        \
        if (e_ != hipSuccess) return hip_fail((ctx), e_, #call);                                                       \
    } while (0)

void free_dev(void *p)
{
    if (p) (void)hipFree(p);
}

/* RayTracer::setCameraSpherical (RayTracer.cpp:33-47): gmtl EulerAngle<ZYX>
   (0, yaw, pitch) -> quaternion qz*qy*qx (Generate.h:214-260), normalised
   (QuatOps.h:337-351), position = q (0,0,d) q* (Xforms.h:40-60) + target, and
   the rotation matrix of q (Generate.h:1143-1176).  float arithmetic in gmtl's
   order; the two angle conversions are binary64 as in the D2R macro. */
void spherical_view(float tx, float ty, float tz, float el, float az, float dist, float m[4][4])
{
    const float yaw = (float)(-(az * kPi / 180.0f) + kPi);
    const float pitch = (float)(-(el * kPi / 180.0f));
    const float xr = pitch, yr = yaw, zr = 0.0f;
    const float x2 = xr * 0.5f, y2 = yr * 0.5f, z2 = zr * 0.5f;
    /* quaternions as (x, y, z, w) */
    const float qx[4] = {std::sin(x2), 0.0f, 0.0f, std::cos(x2)};
    const float qy[4] = {0.0f, std::sin(y2), 0.0f, std::cos(y2)};
    const float qz[4] = {0.0f, 0.0f, std::sin(z2), std::cos(z2)};
    auto qmul = [](const float *a, const float *b, float *r) {
        r[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
        r[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
        r[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
        r[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    };
    float t[4], q[4];
    qmul(qz, qy, t);
    qmul(t, qx, q);
    const float len = std::sqrt((((q[0] * q[0]) + (q[1] * q[1])) + (q[2] * q[2])) + (q[3] * q[3]));
    if (!(len < 0.0001f)) {
        const float li = 1.0f / len;
        for (int i = 0; i < 4; ++i) q[i] *= li;
    }
    /* position = q * (0,0,dist) * conj(q) */
    const float rc[4] = {-q[0], -q[1], -q[2], q[3]};
    const float pure[4] = {0.0f, 0.0f, dist, 0.0f};
    float tmp[4];
    tmp[0] = pure[3] * rc[0] + pure[0] * rc[3] + pure[1] * rc[2] - pure[2] * rc[1];
    tmp[1] = pure[3] * rc[1] + pure[1] * rc[3] + pure[2] * rc[0] - pure[0] * rc[2];
    tmp[2] = pure[3] * rc[2] + pure[2] * rc[3] + pure[0] * rc[1] - pure[1] * rc[0];
    tmp[3] = pure[3] * rc[3] - pure[0] * rc[0] - pure[1] * rc[1] - pure[2] * rc[2];
    const float px = q[3] * tmp[0] + q[0] * tmp[3] + q[1] * tmp[2] - q[2] * tmp[1];
    const float py = q[3] * tmp[1] + q[1] * tmp[3] + q[2] * tmp[0] - q[0] * tmp[2];
    const float pz = q[3] * tmp[2] + q[2] * tmp[3] + q[0] * tmp[1] - q[1] * tmp[0];
    /* rotation part (Watt & Watt) */
    const float xs = q[0] + q[0], ys = q[1] + q[1], zs = q[2] + q[2];
    const float xx = q[0] * xs, xy = q[0] * ys, xz = q[0] * zs;
    const float yy = q[1] * ys, yz = q[1] * zs, zz = q[2] * zs;
    const float wx = q[3] * xs, wy = q[3] * ys, wz = q[3] * zs;
    m[0][0] = 1.0f - (yy + zz);
    m[1][0] = xy + wz;
    m[2][0] = xz - wy;
    m[0][1] = xy - wz;
    m[1][1] = 1.0f - (xx + zz);
    m[2][1] = yz + wx;
    m[0][2] = xz + wy;
    m[1][2] = yz - wx;
    m[2][2] = 1.0f - (xx + yy);
    m[3][0] = m[3][1] = m[3][2] = 0.0f;
    m[3][3] = 1.0f;
    m[0][3] = px + tx;
    m[1][3] = py + ty;
    m[2][3] = pz + tz;
}

/* RayTracerCL::updateCLCamera (RayTracerCL.cpp:178-215). */
void camera_from_view(const float m[4][4], float fov_deg, uint32_t width, rt_camera *c)
{
    auto xform = [&](float v0, float v1, float v2, float *r) { /* gmtl Matrix44 * Vec3 (w = 0), Xforms.h:113-190 */
        float res[4];
        for (int i = 0; i < 4; ++i) {
            res[i] = 0.0f;
            res[i] += m[i][0] * v0;
            res[i] += m[i][1] * v1;
            res[i] += m[i][2] * v2;
            res[i] += m[i][3] * 0.0f;
        }
        if (!(std::fabs(res[3] - 0.0f) <= 0.0001f)) {
            const float wi = 1.0f / res[3];
            for (int i = 0; i < 3; ++i) r[i] = res[i] * wi;
        } else {
            for (int i = 0; i < 3; ++i) r[i] = res[i];
        }
    };
    float view[3], up[3], right[3];
    xform(0.0f, 0.0f, -1.0f, view);
    xform(0.0f, 1.0f, 0.0f, up);
    right[0] = (view[1] * up[2]) - (view[2] * up[1]);
    right[1] = (view[2] * up[0]) - (view[0] * up[2]);
    right[2] = (view[0] * up[1]) - (view[1] * up[0]);
    const float s = (float)((width / 2.0) / std::tan((fov_deg * kPi / 180.0f) / 2.0));
    for (int i = 0; i < 3; ++i) view[i] *= s;
    c->view = {view[0], view[1], view[2], 0.0f};
    c->up = {up[0], up[1], up[2], 0.0f};
    c->right = {right[0], right[1], right[2], 0.0f};
    c->position = {m[0][3], m[1][3], m[2][3], 0.0f};
}

int ensure_seeds(rt_ctx *c, uint32_t wpad, uint32_t hpad, const uint32_t *src)
{
    const size_t count = 2ull * wpad * hpad;
    if (wpad != c->wpad || hpad != c->hpad) {
        free_dev(c->d_seeds);
        c->d_seeds = nullptr;
        c->wpad = c->hpad = 0;
        if (count) HIPCHK(c, hipMalloc(&c->d_seeds, count * sizeof(uint32_t)));
        c->wpad = wpad;
        c->hpad = hpad;
    }
    std::vector<uint32_t> host;
    if (!src) { /* RayTracerCL::updateSeedBuffer: rand(), values < 2 raised to 2 */
        host.resize(count);
        for (size_t i = 0; i < count; ++i) {
            uint32_t v = c->rng.next();
            host[i] = v < 2 ? 2 : v;
        }
        src = host.data();
    }
    if (count) HIPCHK(c, hipMemcpy(c->d_seeds, src, count * sizeof(uint32_t), hipMemcpyHostToDevice));
    return RT_OK;
}

int trav_kind(const rt_ctx *c)
{
    if (c->traversal == RT_TRAVERSAL_LINEAR) return RT_TRAV_LINEAR;
    if (c->traversal == RT_TRAVERSAL_BVH4F || !c->d_nodes4q) return RT_TRAV_BVH4;
    return RT_TRAV_BVH4Q;
}

uint32_t spill_cap(const rt_ctx *c)
{
    /* worst-case stack: the 4-wide tree's stack4 */
    const int k = trav_kind(c);
    const uint32_t need = (k == RT_TRAV_BVH4 || k == RT_TRAV_BVH4Q) ? std::max(c->bvh.stack4, c->stack4_all) : 0u;
    return need > RT_STACK_DEPTH ? need - RT_STACK_DEPTH : 0;
}

const float *trav_nodes(const rt_ctx *c)
{
    const int k = trav_kind(c);
    if (k == RT_TRAV_BVH4Q) return reinterpret_cast<const float *>(c->d_nodes4q);
    return k == RT_TRAV_BVH4 ? c->d_nodes4 : nullptr;
}

/* Grow the triangle buffer to `records` 48-B records, keeping the first `keep` (the mesh's). */
int ensure_tris_capacity(rt_ctx *c, size_t records, size_t keep, hipStream_t st, bool shrink = false)
{
    /* grows to `records`; with `shrink`, also gives back an area more than twice the need */
    if (records <= c->tris_cap && !(shrink && c->tris_cap > keep + 2 * (records - keep) + (1u << 20))) return RT_OK;
    float *nt = nullptr;
    HIPCHK(c, hipMalloc(&nt, records * 48));
    hipError_t e = hipMemcpyAsync(nt, c->d_tris, keep * 48, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipFree(nt);
        return hip_fail(c, e, "triangle buffer copy");
    }
    free_dev(c->d_tris);
    c->d_tris = nt;
    c->tris_cap = records;
    c->list_key.clear(); /* only the mesh's records were carried over */
    return RT_OK;
}

int ensure_spill(rt_ctx *c, size_t entries)
{
    if (entries <= c->spill_entries) return RT_OK;
    free_dev(c->d_spill);
    c->d_spill = nullptr;
    c->spill_entries = 0;
    HIPCHK(c, hipMalloc(&c->d_spill, entries * sizeof(int32_t)));
    c->spill_entries = entries;
    return RT_OK;
}

int grid_blocks(rt_ctx *c, int trav, bool count, int form, int *out)
{
    const int key = (trav * 2 + (count ? 1 : 0)) * 3 + form;
    if (key < 0 || key >= (int)(sizeof(c->grid_cache) / sizeof(c->grid_cache[0])))
        return fail(c, RT_ERR_ARG, "unknown traversal kind");
    if (!c->grid_cache[key]) {
        int b = 0;
        const int e = rt_tris_grid_blocks(c->device, trav, count, form, &b);
        if (e) return hip_fail(c, (hipError_t)e, "occupancy query");
        c->grid_cache[key] = b;
    }
    *out = c->grid_cache[key];
    return RT_OK;
}

/* Sample-split tiles (RT_SPLIT): when a launch has fewer pixels than about two
   per resident lane — a multi-GPU tile of a many-sample frame — every lane holds one pixel
   from the start and the launch lasts as long as its slowest pixel's serial sample chain.
   Splitting each pixel's samples into chunks (seeded by a closest-hit-only pass) turns it back
   into a queue of many short tasks.  Automatic below two pixels per lane at sampleRate >= 4
   (dragon class, 1920x1080 at 256 spp, one rank's row-stripe tile: 4-way 42.1 -> 35.6 ms, 8-way
   29.2 -> 24.8 ms; 2-way 59.3 -> 68.3 and the whole frame 96.5 -> 127.4 ms would lose:
   profiles/r03v). */
bool split_wanted(const rt_ctx *c, uint64_t npx, uint64_t lanes)
{
    if (c->sample_rate < 2) return false;
    return c->split == 1 || (c->split < 0 && npx < 2 * lanes && c->sample_rate >= 4);
}

/* The long chains' seed-pass form for a sample-split launch: below 1.2 pixels per resident lane
   (the 8-way tile of the 1920x1080 frame: 0.8) the chains are the tile's critical path and take
   8 subtree-parallel lanes each (k_chain_seeds: 8-way tile 18.5 -> 16.4 ms); above it (the 4-way
   tile: 1.6) the chunks' throughput is, and the 4-lane cooperative pass, lighter on the chip,
   wins (4-way tile 32.5 -> 30.1 ms; profiles/r04t). */
uint32_t seed_width_auto(uint64_t npx, uint64_t lanes) { return npx * 5 < lanes * 6 ? 8u : (uint32_t)RT_SEED_COOP4; }

/* Sample-split buffers: per pixel (nch + 1) seed pairs, per sample and pixel an RGB radiance. */
int ensure_split(rt_ctx *c, size_t seed_bytes, size_t col_bytes)
{
    if (c->split_seed_bytes < seed_bytes) {
        free_dev(c->d_split_seed);
        c->d_split_seed = nullptr;
        c->split_seed_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_split_seed, seed_bytes));
        c->split_seed_bytes = seed_bytes;
    }
    if (c->split_col_bytes < col_bytes) {
        free_dev(c->d_split_col);
        c->d_split_col = nullptr;
        c->split_col_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_split_col, col_bytes));
        c->split_col_bytes = col_bytes;
    }
    if (!c->d_split_counter) HIPCHK(c, hipMalloc(&c->d_split_counter, 64 * sizeof(uint32_t)));
    if (!c->stream2) HIPCHK(c, hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    if (!c->ev_split0) HIPCHK(c, hipEventCreateWithFlags(&c->ev_split0, hipEventDisableTiming));
    if (!c->ev_box) HIPCHK(c, hipEventCreateWithFlags(&c->ev_box, hipEventDisableTiming));
    if (!c->stream3) HIPCHK(c, hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking));
    if (!c->ev_mesh) HIPCHK(c, hipEventCreateWithFlags(&c->ev_mesh, hipEventDisableTiming));
    if (!c->ev_fin3) HIPCHK(c, hipEventCreateWithFlags(&c->ev_fin3, hipEventDisableTiming));
    return RT_OK;
}

/* The long chains' seed-pass grid: one chain per group of `width` lanes, at most a quarter of
   the full grid (further chains queue behind the first) — subtree-parallel chains at most three
   quarters, so the mesh pixels' chunk launch beside it keeps a quarter of the grid (a tile with
   tens of thousands of chains left it one block: RT_SEED_WIDTH=8 on the 2-way tile ran for
   seconds, profiles/r05bc; 77 ms with the cap, r05bf); full_grid 0: unbounded. */
int split_box_blocks(const rt_ctx *c, uint32_t width, int full_grid)
{
    const uint32_t per_wave = 64u / std::max(1u, width == RT_SEED_COOP4 ? 4u : width);
    int n = (int)((c->n_split_box + per_wave * 4u - 1u) / (per_wave * 4u));
    /* subtree-parallel chains (width >= 8) all run at once where they fit: each is the critical path */
    if (full_grid > 0) n = std::min(n, std::max(1, width >= 8 ? full_grid * 3 / 4 : full_grid / RT_BOX_GRID_DIV));
    return n;
}

/* Speculated mesh pixels: every mesh pixel's sample draws 2 + 2 x lights random
   numbers, so chunk c starts c x chunk x D draws after the frame seed; per chunk the jump
   multipliers A^(c chunk D) mod A 2^16 - 1 of the two MWC generators (rng.h:9-47), computed here
   and uploaded when they change; the per-pixel marks are cleared for the render. */
uint32_t powmod(uint64_t a, uint64_t e, uint64_t m)
{
    uint64_t r = 1 % m;
    a %= m;
    while (e) {
        if (e & 1u) r = r * a % m;
        a = a * a % m;
        e >>= 1;
    }
    return (uint32_t)r;
}

int spec_setup(rt_ctx *c, RtTriLaunch &a, size_t npx, hipStream_t st)
{
    const uint32_t draws = 2u + 2u * (uint32_t)c->lights.size();
    const uint64_t key = (uint64_t)a.split_chunks << 40 | (uint64_t)a.split_chunk << 20 | draws;
    if (!c->d_spec_mul) HIPCHK(c, hipMalloc(&c->d_spec_mul, 4 * 64 * sizeof(uint32_t)));
    if (a.split_chunks > 64) return fail(c, RT_ERR_ARG, "speculated split: more than 64 chunks");
    if (key != c->spec_mul_key) {
        c->h_spec_mul.assign(4 * 64, 1u);
        for (uint32_t ch = 0; ch < a.split_chunks; ++ch) {
            const uint64_t k = (uint64_t)ch * a.split_chunk * draws;
            c->h_spec_mul[2 * ch] = powmod(36969u, k, 36969ull * 65536u - 1u);
            c->h_spec_mul[2 * ch + 1] = powmod(18000u, k, 18000ull * 65536u - 1u);
        }
        for (uint32_t j = 0; j < 64; ++j) { /* the repair's runs: lane j's sample is j x D draws on */
            c->h_spec_mul[128 + 2 * j] = powmod(36969u, (uint64_t)j * draws, 36969ull * 65536u - 1u);
            c->h_spec_mul[128 + 2 * j + 1] = powmod(18000u, (uint64_t)j * draws, 18000ull * 65536u - 1u);
        }
        /* on the render stream, after the previous frame's chunk tasks and repair pass (which read
           the multipliers: split_render ends with the render stream waiting on the other two); the
           wait keeps the host copy alive until the upload is done (a rare event: the key changes
           with the chunking or the light count) */
        HIPCHK(c, hipMemcpyAsync(c->d_spec_mul, c->h_spec_mul.data(), 4 * 64 * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        HIPCHK(c, hipStreamSynchronize(st));
        c->spec_mul_key = key;
    }
    if (c->split_dirty_px < npx) {
        free_dev(c->d_split_dirty);
        free_dev(c->d_split_repair);
        c->d_split_dirty = c->d_split_repair = nullptr;
        c->split_dirty_px = 0;
        HIPCHK(c, hipMalloc(&c->d_split_dirty, npx * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc(&c->d_split_repair, npx * sizeof(uint32_t)));
        c->split_dirty_px = npx;
    }
    HIPCHK(c, hipMemsetAsync(c->d_split_dirty, 0xff, npx * sizeof(uint32_t), st));
    a.split_spec = 1;
    a.split_spec_draws = draws;
    a.split_spec_mul = c->d_spec_mul;
    a.split_run_mul = c->d_spec_mul + 128;
    a.split_dirty = c->d_split_dirty;
    a.split_repair = c->d_split_repair;
    return RT_OK;
}

/* The long chains' mesh-hit depths (split_hit_depth): their subtree-parallel seed pass answers, for
   every segment of every sample, whether its closest-hit query accepts a triangle — the same answer
   the chunk task's traversal would give (the seeds depend on it) — and stores the depth of the one
   that does (a path ends at its mesh hit, rtcommon.h:411-421); a chunk task then answers the box
   segments above it without a traversal.  One sample per task (the depth is read at the take), and
   depths in a byte.  Not for the repair pass: its chains are mesh pixels, whose paths meet the mesh
   at the camera ray. */
bool hit_depth_on(const rt_ctx *c, const RtTriLaunch &t)
{
    (void)c;
    return (t.split_coop >= 8 || t.split_coop == RT_SEED_COOP4) && !t.split_restart && t.split_chunk == 1u && t.max_depth < 255u;
}

/* A sample-split render: the box pixels' seed pass, their chunks and their in-order sums on
   stream2, beside the mesh pixels' seed pass (none when speculated) and chunks on the render
   stream (the box pixels' chains are the long ones: they overlap the rest of the frame instead
   of preceding it); the clean mesh pixels' sums on stream3 beside the repair pass, then the
   repaired pixels' sums.  Each stream has its own queue cursors and its own part of the spill area. */
int split_render(rt_ctx *c, const RtTriLaunch &a, int blocks, hipStream_t st)
{
    const uint32_t n_box = a.split_which == RT_SPLIT_MESH ? a.split_n_box : 0u;
    if (n_box) {
        RtTriLaunch b = a;
        b.split_which = RT_SPLIT_BOX;
        b.pixel_iter = nullptr; /* the measured costs: the mesh pixels' chunk tasks only */
        b.split_counter = a.split_counter + 32;
        b.work_counter = a.work_counter + kWorkBox;
        b.spill = a.spill + (size_t)std::max<int>(blocks, (int)a.split_seed_blocks) * RT_BLOCK * a.spill_cap;
        b.split_gpw = 0;
        b.split_seed_blocks = (uint32_t)std::max(1, c->split_box_grid);
        b.split_chunk = a.split_fine; /* the long chains' chunks: one stored seed each */
        b.split_chunks = (a.sample_rate * a.sample_rate + b.split_chunk - 1u) / b.split_chunk;
        HIPCHK(c, hipEventRecord(c->ev_split0, st));
        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_split0, 0));
        if (a.split_coop >= 8 || a.split_coop == RT_SEED_COOP4) {
            /* the long chains' pass (subtree-parallel or cooperative) stores a chain's seed every
               RT_LONG_FINE samples into a buffer of its own, by slot, and each sample's mesh-hit
               depth: their chunk tasks are that short, so the long chains' last chunks (box paths,
               the costliest samples) do not trail the tile */
            const uint32_t spp = a.sample_rate * a.sample_rate;
            b.split_fine = RT_LONG_FINE;
            b.split_chunk = RT_LONG_FINE;
            b.split_chunks = (spp + RT_LONG_FINE - 1u) / RT_LONG_FINE;
            b.split_nseed = b.split_chunks + 1u;
            const size_t seed_bytes = (size_t)n_box * b.split_nseed * 8u;
            const bool hd = hit_depth_on(c, b);
            const size_t bytes = seed_bytes + (hd ? (size_t)n_box * spp : 0u);
            if (c->long_seed_bytes < bytes) {
                free_dev(c->d_long_seed);
                c->d_long_seed = nullptr;
                c->long_seed_bytes = 0;
                HIPCHK(c, hipMalloc(&c->d_long_seed, bytes));
                c->long_seed_bytes = bytes;
            }
            b.split_seed = c->d_long_seed;
            b.split_seed_slot = 1;
            b.split_hit_depth = hd ? reinterpret_cast<uint8_t *>(c->d_long_seed) + seed_bytes : nullptr;
            c->last_hit_depth = hd;
        }
        const int chunk_grid = (int)std::min<uint64_t>((uint64_t)blocks, ((uint64_t)n_box * b.split_chunks + RT_BLOCK - 1) / RT_BLOCK);
        int e = rt_launch_split_seeds(b, c->stream2);
        if (!e) e = rt_launch_tris(b, RT_TRAV_BVH4Q, c->counting, std::max(1, chunk_grid), c->stream2);
        RtTriLaunch f = b; /* the long chains' in-order sums, as soon as their chunks are done */
        f.finish_part = RT_FIN_LIST;
        if (!e) e = rt_launch_split_finish(f, c->stream2);
        if (e) return hip_fail(c, (hipError_t)e, "box-pixel split launches");
        HIPCHK(c, hipEventRecord(c->ev_box, c->stream2));
    }
    RtTriLaunch m = a; /* the mesh pixels' seed pass: short chains, one lane each */
    m.split_coop = 0;
    int e = a.split_spec ? 0 : rt_launch_split_seeds(m, st); /* speculated: no seed pass */
    if (!e) e = rt_launch_tris(m, RT_TRAV_BVH4Q, c->counting, blocks, st);
    if (e) return e;
    if (n_box) { /* the mesh pixels no chunk of which missed: summed on stream3, beside the repair pass */
        HIPCHK(c, hipEventRecord(c->ev_mesh, st));
        HIPCHK(c, hipStreamWaitEvent(c->stream3, c->ev_mesh, 0));
        RtTriLaunch f = a;
        f.finish_part = RT_FIN_MESH;
        e = rt_launch_split_finish(f, c->stream3);
        if (e) return hip_fail(c, (hipError_t)e, "mesh-pixel sums");
        HIPCHK(c, hipEventRecord(c->ev_fin3, c->stream3));
    }
    if (!n_box) return rt_launch_split_finish(a, st);
    if (a.split_spec) {
        /* the repair pass: the speculated pixels a camera ray of which missed the mesh, as long
           chains from their first missed chunk (seed pass, chunks, sums), their count read on
           the device (usually none: the grids find no item and end).  With the subtree-parallel
           pass the first RT_REPAIR_SLOTS of them store a seed per sample by slot, so their chunk
           tasks are single samples; any beyond take the per-pixel seeds */
        RtTriLaunch r = a;
        r.split_spec = 0;
        r.pixel_iter = nullptr;
        r.split_which = RT_SPLIT_BOX;
        r.split_box = a.split_repair;
        r.split_n_box = 0;
        r.split_n_dev = reinterpret_cast<const uint32_t *>(a.counters + RT_CNT_REPAIR);
        r.split_counter = a.split_counter + 48;
        r.work_counter = a.work_counter + kWorkRepair;
        r.split_gpw = 0;
        r.split_seed_blocks = 16u * RT_REPAIR_WIDTH / 16u; /* RT_REPAIR_WIDTH blocks of 4 waves, one chain per wave
                                                                at width 64: up to 256 chains at once */
        r.split_chunk = a.split_fine;
        r.split_chunks = (a.sample_rate * a.sample_rate + r.split_chunk - 1u) / r.split_chunk;
        r.split_restart = a.split_dirty; /* each chain from its first missed chunk on */
        r.split_restart_chunk = a.split_chunk;
        r.finish_part = RT_FIN_LIST;
        /* the runs form also where the long chains take the cooperative pass (the 4-way tile: the
           repair 2.7 -> 2.1 ms at the end of the mesh pixels' stream, the tile 28.83 -> 28.39 ms, profiles/r05bg, r05bh) */
        {
            const uint32_t spp = a.sample_rate * a.sample_rate;
            r.split_coop = RT_REPAIR_WIDTH; /* runs of width - 1 hit samples (k_chain_seeds<width, true>) */
            RtTriLaunch s = r;
            s.split_fine = RT_LONG_FINE;
            s.split_chunk = RT_LONG_FINE;
            s.split_chunks = (spp + RT_LONG_FINE - 1u) / RT_LONG_FINE;
            s.split_nseed = s.split_chunks + 1u;
            s.split_item_cap = c->repair_slots;
            const size_t bytes = (size_t)c->repair_slots * s.split_nseed * 8u;
            if (c->repair_seed_bytes < bytes) {
                free_dev(c->d_repair_seed);
                c->d_repair_seed = nullptr;
                c->repair_seed_bytes = 0;
                HIPCHK(c, hipMalloc(&c->d_repair_seed, bytes));
                c->repair_seed_bytes = bytes;
            }
            s.split_seed = c->d_repair_seed;
            s.split_seed_slot = 1;
            e = rt_launch_split_seeds(s, st);
            if (!e) e = rt_launch_tris(s, RT_TRAV_BVH4Q, c->counting, 128, st);
            if (!e) e = rt_launch_split_finish(s, st);
            if (e) return hip_fail(c, (hipError_t)e, "repair launches");
            r.split_item_base = c->repair_slots; /* the rest, if any */
        }
        e = rt_launch_split_seeds(r, st);
        if (!e) e = rt_launch_tris(r, RT_TRAV_BVH4Q, c->counting, 64, st);
        if (!e) e = rt_launch_split_finish(r, st);
        if (e) return hip_fail(c, (hipError_t)e, "repair launches");
    }
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_box, 0));
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_fin3, 0));
    return RT_OK;
}

/* LPT scheduling of the pixel queue.  The reference's per-pixel cost is set by its paths: a
   camera ray that hits the mesh ends after one shadow query per light (rtcommon.h:411-421),
   one that misses bounces off the box up to maxDepth+1 times with shadow queries at each
   (rtcommon.h:425-461), and each query costs its traversal steps.  A probe (k_probe_cost)
   traces a grid of camera rays per pixel (2x2; 4x4 for a sample-split render) and, on mesh
   hits, their shadow rays toward the light centres with the real traversal, counting steps.
   From it the device computes the tile costs, the LPT order (most expensive 8x8 tiles first,
   so the launch does not end on a tail of long pixels) and the pixel classes (rt_sched.hip).
   A sample-split render (split_wanted) also takes its long chains from it — the box pixels
   (some probe ray missed the mesh) and the mesh pixels whose probe took more than 96 steps per
   ray — at the price of one 4-byte read (their count, to size the slot list).  Scheduling
   only: every pixel's result is independent of when and where it is rendered.  Cached until
   camera, mesh, traversal, frame, tile or path parameters change. */
int tile_order(rt_ctx *c, const RtTriLaunch &a, int blocks, hipStream_t st)
{
    const uint32_t W = a.W, hl = a.Hl;
    /* everything the order and the pixel classes depend on — including the traversal (only
       the compressed tree is probed: a key without it would hand a BVH4F / linear launch stale
       classes) */
    const uintptr_t np = reinterpret_cast<uintptr_t>(a.nodes);
    std::vector<uint32_t> key = {a.W, a.H, hl, a.stripe, a.n_ranks, a.rank, a.map_key, c->max_depth, (uint32_t)c->lights.size(),
                                 (uint32_t)c->mesh_serial, (uint32_t)(c->mesh_serial >> 32), (uint32_t)blocks,
                                 c->sample_rate, (uint32_t)(c->split + 1) | (uint32_t)c->split_spec << 8,
                                 (uint32_t)trav_kind(c), (uint32_t)np,
                                 (uint32_t)((uint64_t)np >> 32)};
    const uint32_t *cb = reinterpret_cast<const uint32_t *>(&c->cam);
    key.insert(key.end(), cb, cb + sizeof(rt_camera) / 4);
    const uint32_t n_t = ((W + 7) / 8) * ((hl + 7) / 8);
    c->schedule_rebuilt = false;
    if (key == c->order_key) {
        if (c->iter_recorded && !c->order_measured && c->d_order) {
            /* the view's second frame: its tiles by the first frame's measured costs (the probe's
               few rays miss where the samples' shadow rays are long: dragon frame) */
            const int e = rt_sched_order_measured(c->sched, c->d_pixel_iter, W, hl, c->iter_nch, c->d_order, st);
            if (e) return hip_fail(c, (hipError_t)e, "measured tile order");
            c->order_measured = true;
        }
        return RT_OK;
    }
    c->order_key.clear();
    c->iter_recorded = false;
    c->order_measured = false;
    c->n_split_box = 0;
    if (trav_kind(c) != RT_TRAV_BVH4Q || a.nodes != reinterpret_cast<const float *>(c->d_nodes4q)) {
        /* the probe walks the compressed tree with its spill layout: other traversal kinds
           (measurement variants) keep the row-major queue and no classes */
        free_dev(c->d_order);
        c->d_order = nullptr;
        c->order_cap = 0;
        c->order_key = key;
        return RT_OK;
    }
    const size_t npx = (size_t)W * hl;
    if (c->flags_bytes < npx * 4) {
        free_dev(c->d_flags);
        c->d_flags = nullptr;
        c->flags_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_flags, npx * 4));
        c->flags_bytes = npx * 4;
    }
    if (c->class_bytes < npx * 4) {
        free_dev(c->d_class);
        c->d_class = nullptr;
        c->class_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_class, npx * 4));
        c->class_bytes = npx * 4;
    }
    if (c->order_cap < n_t) {
        free_dev(c->d_order);
        c->d_order = nullptr;
        c->order_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_order, n_t * sizeof(uint32_t)));
        c->order_cap = n_t;
    }
    const bool split = split_wanted(c, npx, (uint64_t)blocks * RT_BLOCK);
    RtTriLaunch pa = a;
    pa.probe_n = split && c->sample_rate >= 4 ? c->split_probe : probe_n(c->sample_rate);
    /* a whole-pixel frame that a pilot render will order (pilot_order): the probe only classes the
       pixels (box pixels: the issue priority), one ray each */
    const bool pilot_next = !split && c->pilot_sr > 0 && c->sample_rate * c->sample_rate >= kPilotMinSpp && !c->counting;
    if (pilot_next) pa.probe_n = 1;
    const uint32_t pn2 = pa.probe_n * pa.probe_n;
    int e = rt_launch_probe_cost(pa, blocks, c->d_flags, st);
    if (e) return hip_fail(c, (hipError_t)e, "probe launch");
    /* (the probe's order even then: the frame falls back to it should the pilot not run) */
    e = rt_sched_order(c->sched, c->d_flags, W, hl, pn2, (uint32_t)c->lights.size(), c->max_depth, c->d_order, st);
    if (e) return hip_fail(c, (hipError_t)e, "tile order");
    /* speculated mesh pixels: the silhouettes' neighbours run as long chains (RT_SPLIT_SPEC=2: every
       probe-hit pixel speculated — a test knob that makes repairs happen) */
    const uint32_t spec_row = split && c->split_spec == 1 ? W : 0u;
    /* the probe steps per ray above which a mesh pixel runs as a long chain (none / 200 measured slower,
       profiles/r05ak) */
    const uint32_t long_steps = 96;
    e = rt_sched_box_scan(c->sched, c->d_flags, (uint32_t)npx, pn2, split ? long_steps * pn2 : 0u, spec_row, st);
    if (e) return hip_fail(c, (hipError_t)e, "box-pixel scan");
    uint32_t n_box = 0;
    if (split) { /* every long chain gets a slot: their seed pass and chunks run on a stream of their own */
        HIPCHK(c, hipMemcpyAsync(&n_box, c->sched.scan + npx, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (c->split_box_cap < n_box) {
            free_dev(c->d_split_box);
            c->d_split_box = nullptr;
            c->split_box_cap = 0;
            HIPCHK(c, hipMalloc(&c->d_split_box, (size_t)n_box * 4));
            c->split_box_cap = n_box;
        }
    }
    e = rt_sched_classify(c->sched, (uint32_t)npx, n_box, c->d_class, c->d_split_box, st);
    if (e) return hip_fail(c, (hipError_t)e, "pixel classes");
    c->n_split_box = n_box;
    c->order_key = key;
    c->schedule_rebuilt = true;
    return RT_OK;
}

/* The first frame of a view, whole pixels of many samples: its queue order from a pilot render
   instead of the cost probe.  The probe's few rays per pixel aim their shadow rays at the light
   centres and miss where the samples' rays graze the mesh; the view's next frames are ordered by
   the measured per-pixel costs of the frame before, and the first frame had only
   the probe.  The pilot is the same kernel on the same pixels at pilot_sr^2 samples per pixel,
   with candidate lists built, from a copy of the seeds into a scratch framebuffer and its own
   counters and queue cursors, recording each pixel's traversal steps; the tiles are then sorted
   by them exactly as a measured frame's (rt_sched_order_measured).  Scheduling only: the frame's
   seeds, output and counters are not touched. */
int pilot_order(rt_ctx *c, const RtTriLaunch &a, int trav, int blocks, hipStream_t st)
{
    const size_t seed_words = 2ull * c->wpad * c->hpad, out_floats = (size_t)a.W * a.Hl * 4;
    if (c->pilot_seed_words < seed_words) {
        free_dev(c->d_pilot_seeds);
        c->d_pilot_seeds = nullptr;
        c->pilot_seed_words = 0;
        HIPCHK(c, hipMalloc(&c->d_pilot_seeds, seed_words * sizeof(uint32_t)));
        c->pilot_seed_words = seed_words;
    }
    if (c->pilot_out_floats < out_floats) {
        free_dev(c->d_pilot_out);
        c->d_pilot_out = nullptr;
        c->pilot_out_floats = 0;
        HIPCHK(c, hipMalloc(&c->d_pilot_out, out_floats * sizeof(float)));
        c->pilot_out_floats = out_floats;
    }
    if (!c->d_pilot_cnt) HIPCHK(c, hipMalloc(&c->d_pilot_cnt, kCounterBytes + kWorkWords * sizeof(uint32_t)));
    HIPCHK(c, hipMemcpyAsync(c->d_pilot_seeds, c->d_seeds, seed_words * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemsetAsync(c->d_pilot_cnt, 0, kCounterBytes + kWorkWords * sizeof(uint32_t), st));
    RtTriLaunch p = a;
    p.seeds = c->d_pilot_seeds;
    p.out = c->d_pilot_out;
    p.progressive = 0;
    p.sample_rate = (uint32_t)c->pilot_sr;
    p.counters = c->d_pilot_cnt;
    p.work_counter = reinterpret_cast<uint32_t *>(c->d_pilot_cnt + RT_COUNTER_WORDS);
    p.take_exact = 0; /* a short-task launch: batched takes from the multi-head queue */
    p.queue_batch = RT_QUEUE_BATCH;
    p.pixel_stats = nullptr;
    p.pixel_iter = c->d_pixel_iter;
    int e = rt_launch_tris(p, trav, false, blocks, st);
    if (!e) e = rt_sched_order_measured(c->sched, c->d_pixel_iter, a.W, a.Hl, 1u, c->d_order, st);
    if (e) return hip_fail(c, (hipError_t)e, "pilot render");
    return RT_OK;
}

} // namespace

int rt_exception_status(std::string *err) noexcept
{
    int code = RT_ERR_STATE;
    const char *what = "unknown exception";
    try {
        throw;
    } catch (const std::bad_alloc &e) {
        code = RT_ERR_ALLOC;
        what = e.what();
    } catch (const std::length_error &e) {
        code = RT_ERR_ALLOC;
        what = e.what();
    } catch (const std::exception &e) {
        code = RT_ERR_ARG;
        what = e.what();
    } catch (...) {
    }
    if (err) {
        try {
            *err = std::string("host exception: ") + what;
        } catch (...) {
        }
    }
    return code;
}

extern "C" {

const char *rt_status_string(int s)
{
    switch (s) {
    case RT_OK: return "ok";
    case RT_ERR_ARG: return "invalid argument";
    case RT_ERR_HIP: return "HIP runtime error";
    case RT_ERR_NO_SCENE: return "no spheres set";
    case RT_ERR_NO_MESH: return "no mesh set";
    case RT_ERR_ALLOC: return "allocation failed";
    case RT_ERR_STATE: return "invalid state";
    case RT_ERR_LIMIT: return "device limit exceeded";
    default: return "unknown status";
    }
}

int rt_create(int device, rt_ctx **out)
try {
    if (!out) return RT_ERR_ARG;
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return RT_ERR_HIP;
    if (device < 0 || device >= n) return RT_ERR_ARG;
    rt_ctx *c = new (std::nothrow) rt_ctx();
    if (!c) return RT_ERR_ALLOC;
    c->device = device;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) c->view[i][j] = (i == j) ? 1.0f : 0.0f;
    c->rng.seed(1);
    /* A/B and capacity knobs (none changes a result bit) */
    if (const char *sch = getenv("RT_SCHEDULE")) c->schedule = std::string(sch) != "0";
    if (const char *v = getenv("RT_SPLIT_MB")) c->split_mb = (size_t)std::max(0L, atol(v));
    if (const char *v = getenv("RT_SPLIT")) c->split = atoi(v) != 0 ? 1 : 0;
    if (const char *v = getenv("RT_SPLIT_SPEC")) c->split_spec = atoi(v);
    if (const char *v = getenv("RT_SEED_WIDTH")) { /* test knob: 0 automatic, 1 one lane, 3 cooperative, 8-64 (a power of two) */
        const int w = atoi(v);
        if (w == 0 || w == 1 || w == 3 || (w >= 8 && w <= 64 && (w & (w - 1)) == 0)) c->seed_width = (uint32_t)w;
        else fprintf(stderr, "[rtmi] RT_SEED_WIDTH=%s ignored (0, 1, 3 or a power of two from 8 to 64)\n", v);
    }
    if (const char *v = getenv("RT_PIXEL_LISTS")) c->pixel_lists = atoi(v) != 0 ? 1 : 0;
    if (const char *v = getenv("RT_PILOT")) c->pilot_sr = std::max(0, std::min(8, atoi(v))); /* test knob */
    c->repair_slots = std::max(1u, env_u32("RT_REPAIR_SLOTS", RT_REPAIR_SLOTS)); /* test knob: the path beyond them */
    if (const char *v = getenv("RT_LIST_MB")) c->list_mb = (size_t)std::max(0L, atol(v));
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->evm) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&c->d_totals, (RT_COUNTER_WORDS + 1) * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_totals, 0, (RT_COUNTER_WORDS + 1) * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_counters, kCounterBytes + kWorkWords * sizeof(uint32_t)) != hipSuccess ||
        hipHostMalloc(&c->h_counters, kCounterBytes + sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        rt_destroy(c);
        return RT_ERR_HIP;
    }
    memset(c->h_counters, 0, kCounterBytes + sizeof(unsigned long long)); /* no stale guard before any render */
    c->d_work = reinterpret_cast<uint32_t *>(c->d_counters + RT_COUNTER_WORDS);
    /* the pinned copy's device address: a render hands its counters back with k_counters_out (a copy-engine
       transfer where the mapping is unavailable) */
    void *hd = nullptr;
    if (hipHostGetDevicePointer(&hd, c->h_counters, 0) == hipSuccess)
        c->h_counters_dev = static_cast<unsigned long long *>(hd);
    *out = c;
    return RT_OK;
} RT_CATCH(nullptr)

int rt_destroy(rt_ctx *c)
try {
    if (!c) return RT_ERR_ARG;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_dev(c->d_spheres);
    free_dev(c->d_lights);
    free_dev(c->d_nodes4);
    free_dev(c->d_nodes4q);
    free_dev(c->d_spill);
    free_dev(c->d_order);
    free_dev(c->d_flags);
    free_dev(c->d_class);
    free_dev(c->d_split_seed);
    free_dev(c->d_pixel_iter);
    free_dev(c->d_long_seed);
    free_dev(c->d_repair_seed);
    free_dev(c->d_split_col);
    free_dev(c->d_split_counter);
    free_dev(c->d_split_dirty);
    free_dev(c->d_split_repair);
    free_dev(c->d_spec_mul);
    free_dev(c->d_split_box);
    if (c->ev_split0) (void)hipEventDestroy(c->ev_split0);
    if (c->ev_box) (void)hipEventDestroy(c->ev_box);
    if (c->ev_mesh) (void)hipEventDestroy(c->ev_mesh);
    if (c->ev_fin3) (void)hipEventDestroy(c->ev_fin3);
    if (c->stream3) (void)hipStreamDestroy(c->stream3);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    free_dev(c->d_halo_rows);
    free_dev(c->d_halo_buf);
    free_dev(c->d_tris);
    free_dev(c->d_list_code);
    free_dev(c->d_list_tile);
    free_dev(c->d_list_alloc);
    rt_sched_free(c->sched);
    free_dev(c->d_seeds);
    free_dev(c->d_counters); /* d_work lives in it */
    free_dev(c->d_totals);
    free_dev(c->d_stripe_map);
    free_dev(c->d_pilot_seeds);
    free_dev(c->d_pilot_out);
    free_dev(c->d_pilot_cnt);
    free_dev(c->d_part_probe);
    free_dev(c->d_part_cost);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->h_counters) (void)hipHostFree(c->h_counters);
    free_dev(c->d_stage);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->evm) (void)hipEventDestroy(c->evm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

const char *rt_last_error(const rt_ctx *c) { return c ? c->err.c_str() : "null context"; }

int rt_set_spheres(rt_ctx *c, const rt_sphere *s, uint32_t n)
try {
    if (!c || (n && !s)) return RT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    c->spheres.assign(s, s + n);
    c->lights.clear();
    for (uint32_t i = 0; i < n; ++i)
        if (s[i].mat.emission_power != 0) c->lights.push_back(s[i]); /* rtcommon.h:90 */
    free_dev(c->d_spheres);
    free_dev(c->d_lights);
    c->d_spheres = c->d_lights = nullptr;
    if (n) {
        HIPCHK(c, hipMalloc(&c->d_spheres, n * sizeof(rt_sphere)));
        HIPCHK(c, hipMemcpy(c->d_spheres, s, n * sizeof(rt_sphere), hipMemcpyHostToDevice));
    }
    if (!c->lights.empty()) {
        HIPCHK(c, hipMalloc(&c->d_lights, c->lights.size() * sizeof(rt_sphere)));
        HIPCHK(c, hipMemcpy(c->d_lights, c->lights.data(), c->lights.size() * sizeof(rt_sphere),
                            hipMemcpyHostToDevice));
    }
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

/* The mesh's bounds, padded: the box of the vertices the triangles use, grown by 1e-3 of its
   extent + 1e-4 — every point of every triangle (and every point the kernel's triangle test can
   accept: its error is orders of magnitude below the pad) lies at least the pad inside, so a ray
   segment that misses the padded box meets no triangle (k_tris answers such box-path queries
   without a traversal). False when the vertices are not finite (validation reports it). */
static bool mesh_bounds(const float *verts, const int32_t *idx, uint32_t n_tris, float lo[3], float hi[3])
{
    for (int k = 0; k < 3; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
    }
    for (uint64_t i = 0; i < 3ull * n_tris; ++i) {
        const float *v = verts + 3ull * (uint32_t)idx[i];
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], v[k]);
            hi[k] = std::max(hi[k], v[k]);
        }
    }
    float ext = 0.0f;
    for (int k = 0; k < 3; ++k) {
        if (!std::isfinite(lo[k]) || !std::isfinite(hi[k])) return false;
        ext = std::max(ext, hi[k] - lo[k]);
    }
    const float pad = 1e-3f * ext + 1e-4f;
    for (int k = 0; k < 3; ++k) {
        lo[k] -= pad;
        hi[k] += pad;
    }
    return true;
}

int rt_set_mesh(rt_ctx *c, const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris)
try {
    if (!c || !verts || !idx || !n_verts || !n_tris) return fail(c, RT_ERR_ARG, "empty mesh");
    HIPCHK(c, hipSetDevice(c->device));
    std::string err;
    c->mesh_bounds_ok = false;
    if (c->builder == RT_BUILD_GPU) {
        if (!rt_validate_mesh(verts, n_verts, idx, n_tris, err)) return fail(c, RT_ERR_ARG, err);
        free_dev(c->d_nodes4);
        free_dev(c->d_nodes4q);
        free_dev(c->d_tris);
        c->d_nodes4 = c->d_tris = nullptr;
        c->d_nodes4q = nullptr;
        c->n_tris = 0;
        RtGpuBvh g;
        bool det_cull = true;
        if (const char *v = getenv("RT_DET_CULL")) det_cull = atoi(v) != 0; /* A/B knob */
        const int e = rt_build_bvh_gpu(verts, n_verts, idx, n_tris, g, err, c->stream, det_cull);
        c->d_nodes4 = g.nodes4;
        c->d_nodes4q = g.nodes4q;
        c->d_tris = g.tris;
        c->tris_cap = n_tris;
        if (e) return fail(c, RT_ERR_HIP, "GPU BVH build: " + err);
        c->n_tris = n_tris;
        c->mesh_serial++;
        c->bvh.n_nodes = 0; /* no binary layout */
        c->bvh.n_leaves = 0;
        c->bvh.depth = 0;
        c->bvh.n_nodes4 = g.n_nodes4;
        c->bvh.depth4 = g.depth4;
        c->bvh.stack4 = g.stack4;
        c->bvh.build_seconds = g.build_seconds;
        c->bvh.n_hit = n_tris; /* the GPU build keeps every triangle */
        c->tree_recs = n_tris; /* one tree for every query */
        c->shadow_root = 0;
        c->n_nodes4_shadow = 0;
        c->stack4_all = g.stack4;
        c->mesh_builder = RT_BUILD_GPU;
        c->mesh_bounds_ok = mesh_bounds(verts, idx, n_tris, c->mesh_lo, c->mesh_hi);
        return RT_OK;
    }
    /* Two host trees over the same triangles: the closest-hit queries (camera rays, bounces, the
       seed passes) walk one split by surface area, the shadow queries one whose cost area leans
       toward the scene's lights (rt_bvh.cpp Builder::area) — three quarters of the dragon frame's
       steps are shadow rays from mesh hits, and the lights' tree cuts them 10 %, while the long
       chains' subtree-parallel seed pass (closest hits of box paths over a cut of the tree's top
       levels) ran 1.3 ms slower on it (profiles/r06za).  Built side by side on two host threads;
       the shadow tree's nodes and triangle records follow the first tree's in d_nodes4q / d_tris
       (links offset), so a shadow query only starts at another root.  Culling only: any tree gives
       the same hits. */
    RtBvh b;
    if (const char *v = getenv("RT_CULL_UNHITTABLE")) b.cull_unhittable = atoi(v) != 0; /* A/B knob */
    if (const char *v = getenv("RT_DET_CULL")) b.det_cull = atoi(v) != 0; /* A/B knob */
    RtBvh sb;
    sb.cull_unhittable = b.cull_unhittable;
    sb.det_cull = b.det_cull;
    for (const rt_sphere &L : c->lights) {
        sb.light_centres.push_back(L.center.x);
        sb.light_centres.push_back(L.center.y);
        sb.light_centres.push_back(L.center.z);
    }
    if (const char *v = getenv("RT_BVH_LIGHT_W")) sb.light_cost_weight = (float)atof(v); /* A/B knob (0: one tree) */
    b.light_cost_weight = 0.0f;
    bool two = !sb.light_centres.empty() && sb.light_cost_weight > 0.0f && 2ull * n_tris < (1ull << 28);
    bool ok2 = false;
    std::string err2;
    std::thread th;
    if (two)
        th = std::thread([&]() {
            try {
                ok2 = rt_build_bvh(verts, n_verts, idx, n_tris, sb, err2);
            } catch (...) {
                ok2 = false;
            }
        });
    bool ok = false;
    try {
        ok = rt_build_bvh(verts, n_verts, idx, n_tris, b, err);
    } catch (...) {
        if (th.joinable()) th.join();
        throw;
    }
    if (th.joinable()) th.join();
    if (!ok)
        return fail(c, err.find("deeper") != std::string::npos ? RT_ERR_LIMIT : RT_ERR_ARG, err);
    two = two && ok2 && !b.nodes4q.empty() && !sb.nodes4q.empty();
    std::vector<uint32_t> q4 = std::move(b.nodes4q);
    std::vector<float> tr = std::move(b.tris);
    const uint32_t n_a = b.n_nodes4;
    if (two) {
        q4.insert(q4.end(), sb.nodes4q.begin(), sb.nodes4q.end());
        for (size_t i = n_a; i < (size_t)n_a + sb.n_nodes4; ++i)
            for (int k = 0; k < 4; ++k) {
                uint32_t &w = q4[i * RT_QNODE_DWORDS + 12 + k]; /* the explicit child links (rt_quant.h) */
                int32_t code = (int32_t)w;
                if (code == RT_EMPTY_CHILD) continue;
                if (code >= 0) {
                    code += (int32_t)n_a;
                } else {
                    const uint32_t enc = (uint32_t)(~code);
                    code = ~(int32_t)((((enc >> 3) + n_tris) << 3) | (enc & 7u));
                }
                w = (uint32_t)code;
            }
        tr.insert(tr.end(), sb.tris.begin(), sb.tris.end());
    }
    c->mesh_builder = RT_BUILD_HOST;
    free_dev(c->d_nodes4);
    free_dev(c->d_nodes4q);
    free_dev(c->d_tris);
    c->d_nodes4 = c->d_tris = nullptr;
    c->d_nodes4q = nullptr;
    c->n_tris = 0;
    HIPCHK(c, hipMalloc(&c->d_nodes4, b.nodes4.size() * sizeof(float)));
    if (!q4.empty()) HIPCHK(c, hipMalloc(&c->d_nodes4q, q4.size() * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_tris, tr.size() * sizeof(float)));
    c->tris_cap = tr.size() / 12;
    HIPCHK(c, hipMemcpy(c->d_nodes4, b.nodes4.data(), b.nodes4.size() * sizeof(float), hipMemcpyHostToDevice));
    if (!q4.empty())
        HIPCHK(c, hipMemcpy(c->d_nodes4q, q4.data(), q4.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_tris, tr.data(), tr.size() * sizeof(float), hipMemcpyHostToDevice));
    c->tree_recs = tr.size() / 12;
    c->shadow_root = two ? n_a : 0u;
    c->n_nodes4_shadow = two ? sb.n_nodes4 : 0u;
    c->stack4_all = two ? std::max(b.stack4, sb.stack4) : b.stack4;
    c->n_tris = n_tris;
    c->mesh_serial++;
    c->bvh.n_nodes = b.n_nodes;
    c->bvh.n_leaves = b.n_leaves;
    c->bvh.depth = b.depth;
    c->bvh.n_nodes4 = b.n_nodes4;
    c->bvh.depth4 = b.depth4;
    c->bvh.stack4 = b.stack4;
    c->bvh.build_seconds = b.build_seconds;
    c->bvh.n_hit = b.n_hit;
    c->mesh_bounds_ok = mesh_bounds(verts, idx, n_tris, c->mesh_lo, c->mesh_hi);
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_mesh_info(const rt_ctx *c, rt_mesh_stats *out)
try {
    if (!c || !out) return RT_ERR_ARG;
    if (!c->n_tris) return RT_ERR_NO_MESH;
    out->n_tris = c->n_tris;
    out->n_nodes2 = c->bvh.n_nodes;
    out->depth2 = c->bvh.depth;
    out->n_nodes4_shadow = c->n_nodes4_shadow;
    out->n_nodes4 = c->bvh.n_nodes4;
    out->depth4 = c->bvh.depth4;
    out->stack4 = c->bvh.stack4;
    out->builder = (uint32_t)c->mesh_builder;
    out->build_seconds = c->bvh.build_seconds;
    out->n_tris_tree = c->bvh.n_hit;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_view_matrix(rt_ctx *c, const float m[16])
try {
    if (!c || !m) return RT_ERR_ARG;
    for (int col = 0; col < 4; ++col)
        for (int row = 0; row < 4; ++row) c->view[row][col] = m[col * 4 + row];
    c->cam_override = false;
    c->cam_dirty = true;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_camera_spherical(rt_ctx *c, float tx, float ty, float tz, float el, float az, float dist)
try {
    if (!c) return RT_ERR_ARG;
    spherical_view(tx, ty, tz, el, az, dist, c->view);
    c->cam_override = false;
    c->cam_dirty = true;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_fov(rt_ctx *c, float fov)
try {
    if (!c) return RT_ERR_ARG;
    c->fov = fov;
    c->cam_override = false;
    c->cam_dirty = true;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_camera(rt_ctx *c, const rt_camera *cam)
try {
    if (!c || !cam) return RT_ERR_ARG;
    c->cam_explicit = *cam;
    c->cam_override = true;
    c->cam_dirty = true;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_camera_spherical(float tx, float ty, float tz, float el, float az, float dist, float fov, uint32_t width,
                        rt_camera *out)
try {
    if (!out) return RT_ERR_ARG;
    float m[4][4];
    spherical_view(tx, ty, tz, el, az, dist, m);
    camera_from_view(m, fov, width, out);
    return RT_OK;
} RT_CATCH(nullptr)

int rt_set_params(rt_ctx *c, uint32_t sample_rate, uint32_t max_depth)
try {
    if (!c) return RT_ERR_ARG;
    if (sample_rate > 4096) return fail(c, RT_ERR_ARG, "sample rate too large");
    c->sample_rate = sample_rate;
    c->max_depth = max_depth;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_builder(rt_ctx *c, int builder)
try {
    if (!c || (builder != RT_BUILD_HOST && builder != RT_BUILD_GPU)) return RT_ERR_ARG;
    c->builder = builder;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_traversal(rt_ctx *c, int t)
try {
    if (!c || !(t == RT_TRAVERSAL_BVH || t == RT_TRAVERSAL_LINEAR || t == RT_TRAVERSAL_BVH4F)) return RT_ERR_ARG;
    c->traversal = t;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_ndrange(rt_ctx *c, uint32_t nd_y)
try {
    if (!c || nd_y == 0 || nd_y > 1024) return RT_ERR_ARG;
    c->nd_y = nd_y;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_seed_layout(rt_ctx *c, uint32_t wpad, uint32_t hpad)
try {
    if (!c || !wpad || !hpad) return RT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int r = ensure_seeds(c, wpad, hpad, nullptr);
    if (r == RT_OK) c->user_seeds = true;
    return r;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_seeds(rt_ctx *c, const uint32_t *seeds, size_t count)
try {
    if (!c || !seeds) return RT_ERR_ARG;
    if (!c->wpad || count != 2ull * c->wpad * c->hpad) return fail(c, RT_ERR_STATE, "seed count != 2*Wpad*Hpad");
    HIPCHK(c, hipSetDevice(c->device));
    const int r = ensure_seeds(c, c->wpad, c->hpad, seeds);
    if (r == RT_OK) c->user_seeds = true;
    return r;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_get_seeds(const rt_ctx *c, uint32_t *out, size_t count)
try {
    if (!c || !out) return RT_ERR_ARG;
    if (!c->wpad || count != 2ull * c->wpad * c->hpad) return RT_ERR_STATE;
    if (hipSetDevice(c->device) != hipSuccess) return RT_ERR_HIP;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return RT_ERR_HIP;
    if (hipMemcpy(out, c->d_seeds, count * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) return RT_ERR_HIP;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_seed_layout(const rt_ctx *c, uint32_t *wpad, uint32_t *hpad)
try {
    if (!c) return RT_ERR_ARG;
    if (wpad) *wpad = c->wpad;
    if (hpad) *hpad = c->hpad;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_glibc_rand_fill(uint32_t seed, uint32_t *out, size_t count, uint32_t skip)
try {
    if (!out && count) return RT_ERR_ARG;
    GlibcRand g;
    g.seed(seed);
    for (uint32_t i = 0; i < skip; ++i) (void)g.next();
    for (size_t i = 0; i < count; ++i) out[i] = g.next();
    return RT_OK;
} RT_CATCH(nullptr)

uint32_t rt_tile_rows(uint32_t height, const rt_tile *t)
{
    if (!t || t->n_ranks <= 1) return height;
    if (t->stripe_rows == 0 || t->rank >= t->n_ranks) return 0;
    if (t->stripe_owner) { /* an owner map: the rank's stripes (only the frame's last can be short) */
        uint32_t rows = 0;
        for (uint32_t s = 0, y = 0; y < height; ++s, y += t->stripe_rows)
            if (t->stripe_owner[s] == t->rank) rows += std::min(t->stripe_rows, height - y);
        return rows;
    }
    const uint32_t period = t->stripe_rows * t->n_ranks;
    const uint32_t full = height / period;
    uint32_t rows = full * t->stripe_rows;
    const uint32_t rem = height - full * period;
    const uint32_t start = t->rank * t->stripe_rows;
    if (rem > start) rows += std::min(rem - start, t->stripe_rows);
    return rows;
}

/* A box pixel's serial chain against a mesh pixel of the frame's mean probe steps, in the stripes'
   cost (rt_partition_stripes).  From the 8-way dragon tiles (profiles/r06b/partition8.npz: rank
   time against the rank's long chains and traversal steps, least squares): a long chain adds
   3.5e-4 ms, a whole mesh pixel of the mean steps 6.2e-6 ms — about 55 of them. */
static constexpr uint64_t kPartitionBoxWeight = 55;

int rt_partition_stripes(rt_ctx *c, uint32_t W, uint32_t H, uint32_t stripe, uint32_t n, uint32_t *owner,
                         int *recomputed)
try {
    if (!c || !owner || stripe == 0 || n == 0) return RT_ERR_ARG;
    if (recomputed) *recomputed = 0;
    const uint32_t ns = (H + stripe - 1) / stripe;
    if (ns == 0) return RT_OK;
    const int trav = trav_kind(c);
    if (c->n_tris == 0 || trav != RT_TRAV_BVH4Q || n == 1) { /* nothing to probe (or one rank): interleaved */
        for (uint32_t s = 0; s < ns; ++s) owner[s] = s % n;
        return RT_OK;
    }
    rt_camera cam;
    if (c->cam_override) cam = c->cam_explicit;
    else camera_from_view(c->view, c->fov, W, &cam);
    std::vector<uint32_t> key = {W, H, stripe, n, (uint32_t)c->mesh_serial, (uint32_t)(c->mesh_serial >> 32),
                                 (uint32_t)c->lights.size()};
    {
        const uint32_t *cb = reinterpret_cast<const uint32_t *>(&cam);
        key.insert(key.end(), cb, cb + sizeof(rt_camera) / 4);
        for (const rt_sphere &L : c->lights) {
            const uint32_t *lb = reinterpret_cast<const uint32_t *>(&L);
            key.insert(key.end(), lb, lb + sizeof(rt_sphere) / 4);
        }
    }
    if (key == c->part_key && c->part_owner.size() == ns) {
        std::copy(c->part_owner.begin(), c->part_owner.end(), owner);
        return RT_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    if (c->sync_stream && c->sync_stream != st) {
        if (c->sync_stream == c->stream) HIPCHK(c, hipEventRecord(c->ev_done, c->stream));
        HIPCHK(c, hipStreamWaitEvent(st, c->ev_done, 0));
    }
    const size_t npx = (size_t)W * H;
    if (c->part_probe_px < npx) {
        HIPCHK(c, hipStreamSynchronize(st));
        free_dev(c->d_part_probe);
        c->d_part_probe = nullptr;
        c->part_probe_px = 0;
        HIPCHK(c, hipMalloc(&c->d_part_probe, npx * sizeof(uint32_t)));
        c->part_probe_px = npx;
    }
    if (c->part_cost_cap < ns) {
        HIPCHK(c, hipStreamSynchronize(st));
        free_dev(c->d_part_cost);
        c->d_part_cost = nullptr;
        c->part_cost_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_part_cost, (size_t)ns * 2 * sizeof(unsigned long long)));
        c->part_cost_cap = ns;
    }
    /* the probe of the whole frame: one camera ray per pixel (its centre) and its shadow rays */
    RtTriLaunch a{};
    a.nodes = trav_nodes(c);
    a.tris = c->d_tris;
    a.n_tris = c->n_tris;
    a.lights = c->d_lights;
    a.n_lights = (uint32_t)c->lights.size();
    a.cam = cam;
    a.W = W;
    a.H = H;
    a.Hl = H;
    a.stripe = 1;
    a.n_ranks = 1;
    a.rank = 0;
    a.stripe_map = nullptr;
    a.probe_n = 1;
    int blocks = 0;
    if (const int r = grid_blocks(c, trav, false, RT_FORM_PLAIN, &blocks)) return r;
    a.spill_cap = spill_cap(c);
    if (a.spill_cap) {
        HIPCHK(c, hipStreamSynchronize(st)); /* (a render in flight may use the spill area) */
        if (const int r = ensure_spill(c, (size_t)blocks * 2 * RT_BLOCK * a.spill_cap)) return r;
    }
    a.spill = c->d_spill;
    int e = rt_launch_probe_cost(a, blocks, c->d_part_probe, st);
    if (!e) e = rt_launch_stripe_costs(c->d_part_probe, W, H, stripe, 1u, c->d_part_cost, st);
    if (e) return hip_fail(c, (hipError_t)e, "partition probe");
    std::vector<unsigned long long> h((size_t)ns * 2);
    HIPCHK(c, hipMemcpyAsync(h.data(), c->d_part_cost, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    /* a stripe's cost in probe steps: its mesh pixels' steps + its box pixels at kPartitionBoxWeight
       mesh pixels of the frame's mean steps each (integers: every rank gets the same map) */
    uint64_t mesh_px = 0, mesh_steps = 0;
    for (uint32_t s = 0; s < ns; ++s) {
        const uint64_t px = (uint64_t)W * std::min(stripe, H - s * stripe);
        mesh_px += px - h[2 * s];
        mesh_steps += h[2 * s + 1];
    }
    const uint64_t box_cost = kPartitionBoxWeight * (mesh_px ? (mesh_steps + mesh_px / 2) / mesh_px : 1u);
    std::vector<uint64_t> cost(ns);
    for (uint32_t s = 0; s < ns; ++s) cost[s] = h[2 * s] * box_cost + h[2 * s + 1] + 1u;
    /* LPT: costliest stripe first (ties: lower index), to the least loaded rank (ties: lower rank) */
    std::vector<uint32_t> order(ns);
    for (uint32_t s = 0; s < ns; ++s) order[s] = s;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return cost[x] > cost[y]; });
    std::vector<uint64_t> load(n, 0);
    for (uint32_t s : order) {
        uint32_t best = 0;
        for (uint32_t r = 1; r < n; ++r)
            if (load[r] < load[best]) best = r;
        owner[s] = best;
        load[best] += cost[s];
    }
    c->part_key = key;
    c->part_owner.assign(owner, owner + ns);
    if (recomputed) *recomputed = 1;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

/* An owner-map tile's frame stripes, in tile order, on the device (RtTriLaunch::stripe_map);
   re-uploaded (after the stream's earlier renders) only when they change. */
static int upload_stripe_map(rt_ctx *c, uint32_t H, const rt_tile *t, hipStream_t st)
{
    const uint32_t ns = (H + t->stripe_rows - 1) / t->stripe_rows;
    std::vector<uint32_t> mine;
    for (uint32_t s = 0; s < ns; ++s) {
        if (t->stripe_owner[s] >= t->n_ranks) return fail(c, RT_ERR_ARG, "stripe owner out of range");
        if (t->stripe_owner[s] == t->rank) mine.push_back(s);
    }
    if (mine == c->stripe_map_h && c->d_stripe_map) return RT_OK;
    HIPCHK(c, hipStreamSynchronize(st)); /* earlier renders on this stream read the old map */
    if (c->sync_stream && c->sync_stream != st) HIPCHK(c, hipStreamSynchronize(c->sync_stream));
    if (c->stripe_map_cap < std::max<size_t>(mine.size(), 1)) {
        free_dev(c->d_stripe_map);
        c->d_stripe_map = nullptr;
        c->stripe_map_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_stripe_map, std::max<size_t>(mine.size(), 1) * sizeof(uint32_t)));
        c->stripe_map_cap = std::max<size_t>(mine.size(), 1);
    }
    if (!mine.empty())
        HIPCHK(c, hipMemcpy(c->d_stripe_map, mine.data(), mine.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    c->stripe_map_h = std::move(mine);
    ++c->stripe_map_serial;
    return RT_OK;
}

int rt_render_async(rt_ctx *c, float *out, uint32_t W, uint32_t H, uint32_t prog, int kernel, const rt_tile *tile,
                    int flags, void *stream)
try {
    if (!c) return RT_ERR_ARG;
    if (W == 0 || H == 0) return RT_OK; /* RayTracerCL.cpp:219-220 */
    if (!out) return fail(c, RT_ERR_ARG, "null output buffer");
    if (kernel < RT_KERNEL_SPHERES || kernel > RT_KERNEL_TRIS) return fail(c, RT_ERR_ARG, "unknown kernel");
    if (tile && tile->n_ranks > 1 && (tile->stripe_rows == 0 || tile->rank >= tile->n_ranks))
        return fail(c, RT_ERR_ARG, "bad tile");
    if (tile && tile->n_ranks > 1 && kernel == RT_KERNEL_SPHERES && prog > 0 && !(flags & RT_SEEDS_HALO))
        return fail(c, RT_ERR_ARG,
                    "row-shifted seeds (raytracer.cl:20-30) cross stripe boundaries: progressive sphere frames on "
                    "a tile need the seed-row halo (rt_pack_seed_rows / rt_unpack_seed_rows, flag RT_SEEDS_HALO)");
    if (kernel == RT_KERNEL_TRIS && c->n_tris == 0) return fail(c, RT_ERR_NO_MESH, "no mesh set");
    if (kernel != RT_KERNEL_TRIS && c->spheres.empty()) return fail(c, RT_ERR_NO_SCENE, "no spheres set");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;

    /* RayTracerCL.cpp:229-249: NDRange padding, camera/seed refresh */
    const uint32_t wpad = ((W & 0x1F) == 0) ? W : ((W & 0xFFFFFFE0u) + 0x20u);
    const uint32_t hpad = (uint32_t)std::ceil(H / (float)c->nd_y) * c->nd_y;
    if (W != c->width || H != c->height) {
        c->cam_dirty = false;
        c->width = W;
        c->height = H;
        if (c->cam_override) c->cam = c->cam_explicit;
        else camera_from_view(c->view, c->fov, W, &c->cam);
        if (c->user_seeds && c->wpad == wpad && c->hpad == hpad) {
            c->user_seeds = false; /* caller-provided seeds for this layout */
        } else {
            const int r = ensure_seeds(c, wpad, hpad, nullptr);
            if (r != RT_OK) return r;
            c->user_seeds = false;
        }
    } else if (c->cam_dirty) {
        c->cam_dirty = false;
        if (c->cam_override) c->cam = c->cam_explicit;
        else camera_from_view(c->view, c->fov, W, &c->cam);
    }
    if (c->wpad < W || c->hpad < H) return fail(c, RT_ERR_STATE, "seed layout smaller than the frame");

    const uint32_t hl = rt_tile_rows(H, tile);
    if (hl == 0) { /* a rank with no rows: nothing rendered, and nothing of an earlier render reported */
        if (c->sync_stream) HIPCHK(c, hipStreamSynchronize(c->sync_stream)); /* its counter copy has landed */
        memset(c->h_counters, 0, kCounterBytes + sizeof(unsigned long long));
        c->info = rt_render_info{};
        c->info.kernel = (uint32_t)kernel;
        c->info_list_pending = false;
        c->last_long = 0;
        c->sync_stream = nullptr;
        return RT_OK;
    }
    const size_t out_bytes = (size_t)W * hl * 4 * sizeof(float);
    float *dout = out;
    if (!(flags & RT_OUT_DEVICE)) {
        if (c->stage_bytes < out_bytes) {
            free_dev(c->d_stage);
            c->d_stage = nullptr;
            c->stage_bytes = 0;
            HIPCHK(c, hipMalloc(&c->d_stage, out_bytes));
            c->stage_bytes = out_bytes;
        }
        dout = c->d_stage;
        if (prog > 0) HIPCHK(c, hipMemcpyAsync(dout, out, out_bytes, hipMemcpyHostToDevice, st));
    }
    /* a render on another stream than the last one's: ordered after that render's counter hand-back
       (which reads and zeroes the counters and queue cursors this render uses) */
    if (c->sync_stream && st != c->sync_stream) {
        if (c->sync_stream == c->stream) HIPCHK(c, hipEventRecord(c->ev_done, c->stream));
        HIPCHK(c, hipStreamWaitEvent(st, c->ev_done, 0));
    }
    /* the counters, the guard word and the queue cursors: one memset (none when the last render's
       k_counters_out left them zeroed) */
    if (!c->counters_zeroed)
        HIPCHK(c, hipMemsetAsync(c->d_counters, 0, kCounterBytes + kWorkWords * sizeof(uint32_t), st));
    c->counters_zeroed = false;
    const uint32_t stripe = tile ? tile->stripe_rows : 1u, nr = tile ? std::max(tile->n_ranks, 1u) : 1u,
                   rk = tile ? tile->rank : 0u;
    /* an owner-map tile: its stripes' frame indices on the device (the view and schedule keys
       carry the map's serial) */
    const uint32_t *smap = nullptr;
    if (tile && nr > 1 && tile->stripe_owner) {
        const int r = upload_stripe_map(c, H, tile, st);
        if (r != RT_OK) return r;
        smap = c->d_stripe_map;
    }
    const uint32_t map_key = smap ? c->stripe_map_serial : 0u;
    int e = 0;
    if (kernel == RT_KERNEL_TRIS) {
        RtTriLaunch a{};
        a.out = dout;
        a.seeds = c->d_seeds;
        a.nodes = trav_nodes(c);
        a.shadow_root = trav_kind(c) == RT_TRAV_BVH4Q ? c->shadow_root : 0u; /* the shadow tree: compressed nodes only */
        a.tris = c->d_tris;
        a.n_tris = c->n_tris;
        a.lights = c->d_lights;
        a.n_lights = (uint32_t)c->lights.size();
        if (a.n_lights > 16) return fail(c, RT_ERR_LIMIT, "more than 16 emissive spheres");
        a.cam = c->cam;
        a.W = W;
        a.H = H;
        a.Wpad = c->wpad;
        a.Hpad = c->hpad;
        a.Hl = hl;
        a.sample_rate = c->sample_rate;
        a.max_depth = c->max_depth;
        a.progressive = prog;
        a.stripe = stripe;
        a.n_ranks = nr;
        a.rank = rk;
        a.stripe_map = smap;
        a.map_key = map_key;
        a.work_counter = c->d_work;
        a.counters = c->d_counters;
        const int trav = trav_kind(c);
        const uint64_t items = (uint64_t)((W + 7) / 8) * ((hl + 7) / 8) * 64;
        const uint64_t item_blocks = (items + RT_BLOCK - 1) / RT_BLOCK;
        /* persistent grids: the plain form's and the sample-split form's own occupancy, the
           plain one at most one block per RT_BLOCK queue items */
        int blocks = 0, blocks_split = 0;
        int r = grid_blocks(c, trav, c->counting, RT_FORM_PLAIN, &blocks);
        if (r != RT_OK) return r;
        blocks = std::max(1, (int)std::min<uint64_t>((uint64_t)blocks, item_blocks));
        /* a short frame — a few samples per resident lane (bunny class at 1 spp: 3.2) — runs on
           3 of the 5 blocks per CU: its time is then its costliest pixels' serial paths, which step
           faster on less crowded SIMDs (bunny class 0.54 -> 0.46 ms at 768 of 1280 blocks; the
           dragon frame at 1024 blocks 96.7 -> 101.2 ms: profiles/r04l, r04m) */
        const bool short_frame =
            (uint64_t)W * hl * c->sample_rate * c->sample_rate < kShortFrameSamplesPerLane * (uint64_t)blocks * RT_BLOCK;
        if (short_frame) blocks = std::max(1, blocks * (int)kShortFrameBlocksPerCU / RT_TRIS_WAVES);
        /* scheduling knobs (read every render; test_stepping_knobs_change_no_bits): a smaller grid, the
           stepping round's exit rule */
        if (const uint32_t gb = env_u32("RTMI_GRID_BLOCKS", 0)) blocks = std::min(blocks, (int)gb);
        if (trav == RT_TRAV_BVH4Q) {
            r = grid_blocks(c, trav, c->counting, RT_FORM_SPLIT, &blocks_split);
            if (r != RT_OK) return r;
        }
        /* the spill area is indexed by blockIdx: sized for twice the larger grid any kernel of
           this render may run with (a sample-split render runs two streams side by side, each on
           its own part of the area) */
        a.spill_cap = spill_cap(c);
        if (a.spill_cap) {
            const int rs = ensure_spill(c, (size_t)std::max<uint64_t>(std::max(blocks, blocks_split), item_blocks) * 2 *
                                               RT_BLOCK * a.spill_cap);
            if (rs != RT_OK) return rs;
        }
        a.spill = c->d_spill;
        a.fetch_k = env_u32("RTMI_FETCH_K", kFetchK);
        a.fetch_frac = env_u32("RTMI_FETCH_FRAC", kFetchFrac);
        a.probe_n = probe_n(c->sample_rate);
        a.diag_pixel = 0xffffffffu;
#if RT_DIAG_ONE_PIXEL
        a.diag_k = 1;
        if (const char *v = getenv("RT_DIAG_PIXEL")) { /* diagnostics build only: "x,y[,k]" */
            unsigned dx = 0, dy = 0, dk = 1;
            const int n = sscanf(v, "%u,%u,%u", &dx, &dy, &dk);
            if (n >= 2) a.diag_pixel = dy * W + dx;
            if (n == 3) a.diag_k = dk;
        }
#endif
        a.tile_order = nullptr;
        a.pixel_flags = nullptr;
        a.pixel_class = nullptr;
        const auto h0 = std::chrono::steady_clock::now();
        c->schedule_rebuilt = false;
        if (c->schedule) {
            const int ro = tile_order(c, a, blocks, st);
            if (ro != RT_OK) return ro;
            a.tile_order = c->d_order;
            a.pixel_flags = a.tile_order ? c->d_flags : nullptr;
            a.pixel_class = a.tile_order ? c->d_class : nullptr;
        }
        /* sample-split tiles: chunks of about spp / 16 samples; the buffers within RT_SPLIT_MB */
        a.split_chunks = 0;
        if (a.tile_order && trav == RT_TRAV_BVH4Q &&
            split_wanted(c, (uint64_t)W * hl, (uint64_t)blocks * RT_BLOCK)) {
            /* chunks of about spp / 16 samples; seeds stored every quarter chunk, so that the long
               chains' chunks (run after their seed pass, on a nearly idle chip) are 4x shorter:
               8-way tile 22.6 -> 20.x ms */
            const uint32_t spp = c->sample_rate * c->sample_rate;
            const uint32_t fine = std::max(1u, (spp + 63u) / 64u), csz = fine * std::max(1u, ((spp + c->split_nch - 1u) / c->split_nch) / fine);
            const uint32_t nch = (spp + csz - 1u) / csz, nseed = (spp + fine - 1u) / fine + 1u;
            const size_t npx_s = (size_t)W * hl;
            const size_t seed_bytes = npx_s * nseed * 8u, col_bytes = npx_s * spp * 12u;
            if (seed_bytes + col_bytes <= (c->split_mb << 20)) {
                const int rs = ensure_split(c, seed_bytes, col_bytes);
                if (rs != RT_OK) return rs;
                a.split_chunks = nch;
                a.split_chunk = csz;
                a.split_fine = fine;
                a.split_nseed = nseed;
                a.split_seed = c->d_split_seed;
                a.split_col = c->d_split_col;
                a.split_counter = c->d_split_counter;
                a.split_which = c->n_split_box ? RT_SPLIT_MESH : RT_SPLIT_ALL;
                a.split_box = c->d_split_box;
                a.split_n_box = c->n_split_box;
                a.n_nodes4 = c->bvh.n_nodes4;
                /* lanes per long chain: seed_width (a power of two, 8-64) subtree-parallel lanes
                   (k_chain_seeds); RT_SEED_COOP4 (3): 4 cooperative lanes (coop_round) where the
                   group's LDS stack holds the tree's worst depth-first stack (+ a candidate list's
                   blocks); else one */
                const uint32_t sw = c->seed_width ? c->seed_width : seed_width_auto((uint64_t)W * hl, (uint64_t)blocks * RT_BLOCK);
                a.split_coop = sw >= 4 ? std::min(64u, std::max(8u, 1u << (31 - __builtin_clz(sw))))
                             : sw == RT_SEED_COOP4 && c->bvh.stack4 + 4 <= RT_COOP_STACK ? RT_SEED_COOP4 : 0u;
                /* a round of 4 nodes adds at most 12 entries and a one-item depth-first walk at
                   most the tree's worst stack: rounds take 4 items up to this depth (coop_round) */
                a.coop_multi_sp = std::max(0, (int)RT_COOP_STACK - 12 - (int)c->bvh.stack4);
                if (c->split_spec && a.split_which == RT_SPLIT_MESH) {
                    const int rs = spec_setup(c, a, npx_s, st);
                    if (rs != RT_OK) return rs;
                }
                /* the box pixels' seed pass (one lane per pixel) keeps its blocks resident beside
                   the mesh pixels' kernels, whose grids leave room for it */
                const int box_blocks = c->n_split_box ? split_box_blocks(c, std::max(1u, a.split_coop), blocks) : 0;
                c->split_box_grid = box_blocks;
                /* the mesh pixels' seed pass: at least one lane per queue item (RT_SEED_GRID_ITEMS), so no lane
                   walks two pixels' chains in turn (the blocks beyond residency start as others end) */
                a.split_seed_blocks = (uint32_t)std::max(1, blocks - box_blocks);
                if (RT_SEED_GRID_ITEMS) a.split_seed_blocks = (uint32_t)std::max<uint64_t>(a.split_seed_blocks, item_blocks);
                blocks = std::max(1, std::min((int)std::min<uint64_t>((uint64_t)blocks_split, item_blocks * nch),
                                              blocks_split - box_blocks));
            }
        }
        /* whole pixels of many samples (long tasks, a few dequeues per microsecond): queue takes of
           exactly the items the idle lanes need, so no wave holds the queue's last tiles back */
        a.take_exact = !a.split_chunks && c->sample_rate * c->sample_rate >= 16u ? 1u : 0u;
        /* short frames: box-path queries whose segment misses the mesh's padded bounds are answered
           without a traversal (bunny class 0.469 -> 0.457 ms; the dragon frame measured 87.1 -> 88.4
           ms with it, profiles/r05ah; the 2-way tile within noise, r05bj: off there) */
        a.mesh_bounds = c->mesh_bounds_ok && short_frame ? 1u : 0u;
        for (int k = 0; k < 3; ++k) {
            a.mesh_lo[k] = c->mesh_lo[k];
            a.mesh_hi[k] = c->mesh_hi[k];
        }
        /* short whole-pixel frames take from the multi-head queue (mq_take) in batches of
           RT_QUEUE_BATCH items (0: one head; bunny class 0.519 -> 0.473 ms, profiles/r05ac) */
        a.queue_batch = a.take_exact || a.split_chunks ? 0u : RT_QUEUE_BATCH;
        /* long tasks take exactly from the multi-head queue too: each head's tiles go to the waves
           of one XCD's blocks, so a tile's pixels share that XCD's L2 (dragon frame 87.4 -> 86.5 ms,
           profiles/r05ar) */
        if (a.take_exact) a.queue_batch = 64u;
        /* a split tile's mesh chunk tasks from the heads too, in batches of 64, a tile's chunk layers on
           one head (8-way tile 15.95 -> 15.71 ms, profiles/r05au) */
        if (a.split_chunks) a.queue_batch = 64u;
        /* a frame under the probe's order records its pixels' costs for the next frame (a sample-split
           frame: its mesh pixels' chunk tasks; the long chains' entries stay 0) */
        a.pixel_iter = nullptr;
        bool record_iter = false;
        /* (frames of >= 16 samples per pixel: a 1-spp pixel's cost is one random path, and the bunny
           class measured 0.436 -> 0.459 ms re-sorted by it, profiles/r05aj) */
        if (a.tile_order && !c->order_measured && c->sample_rate * c->sample_rate >= 16u) {
            const uint32_t nch = a.split_chunks ? a.split_chunks : 1u;
            const size_t n_i = (size_t)W * hl * nch;
            if (c->pixel_iter_px < n_i) {
                free_dev(c->d_pixel_iter);
                c->d_pixel_iter = nullptr;
                c->pixel_iter_px = 0;
                HIPCHK(c, hipMalloc(&c->d_pixel_iter, 2 * n_i * sizeof(uint32_t)));
                c->pixel_iter_px = n_i;
            }
            if (a.split_chunks) HIPCHK(c, hipMemsetAsync(c->d_pixel_iter, 0, 2 * n_i * sizeof(uint32_t), st));
            a.pixel_iter = c->d_pixel_iter;
            c->iter_nch = nch;
            record_iter = true;
        }
        const double sched_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
        if (getenv("RT_DEBUG_LAUNCH")) /* diagnostics: the launch shape */
            fprintf(stderr,
                    "[rtmi %p] k_tris trav %d count %d grid %d x %d, spill_cap %u, order %p, split %u x %u, long %u\n",
                    (void *)c, trav, (int)c->counting, blocks, RT_BLOCK, a.spill_cap, (const void *)a.tile_order,
                    a.split_chunks, a.split_chunk, a.split_n_box);
        /* diagnostics: per-pixel start/finish clocks (+ queries, steps and the wall clocks
           by phase in a counting launch: 8 x u32 per pixel), dumped raw to $RT_PIXEL_STATS */
        const char *stats_path = getenv("RT_PIXEL_STATS");
        uint32_t *d_stats = nullptr;
        a.pixel_stats = nullptr;
        if (stats_path) {
            HIPCHK(c, hipMalloc(&d_stats, (size_t)W * hl * 32));
            HIPCHK(c, hipMemsetAsync(d_stats, 0, (size_t)W * hl * 32, st));
            a.pixel_stats = d_stats;
        }
        /* camera-ray candidate lists (k_pixel_lists, rebuilt every frame): a compacted list area
           after the mesh's triangle records in the same buffer (a list block is a leaf code like
           any other), a count and a first slot per pixel.  Leaf codes address slots below 2^28;
           pixels whose list does not fit the area (RT_LIST_MB) take the tree, and a list area
           that cannot be allocated turns the lists off for the render — same bits either way. */
        a.list_code = nullptr;
        a.list_tile = nullptr;
        const bool bvh4 = c->d_nodes4 && (trav == RT_TRAV_BVH4Q || trav == RT_TRAV_BVH4);
        const uint64_t kept = (c->tree_recs + 7ull) & ~7ull; /* the list area starts on a 128-B line, after the trees' records */
        const uint64_t npx = (uint64_t)W * hl;
        uint64_t list_cap = std::min<uint64_t>(npx * RT_LIST_MAX, ((uint64_t)c->list_mb << 20) / 48);
        list_cap = std::min<uint64_t>(list_cap, kept < (1ull << 28) ? (1ull << 28) - 8 - kept : 0);
        /* the view the lists (and the schedule) are a function of */
        const uintptr_t np4 = reinterpret_cast<uintptr_t>(c->d_nodes4);
        std::vector<uint32_t> view = {W, H, hl, stripe, nr, rk, map_key, (uint32_t)trav, (uint32_t)c->mesh_serial,
                                      (uint32_t)(c->mesh_serial >> 32), (uint32_t)np4, (uint32_t)((uint64_t)np4 >> 32)};
        {
            const uint32_t *cb = reinterpret_cast<const uint32_t *>(&c->cam);
            view.insert(view.end(), cb, cb + sizeof(rt_camera) / 4);
        }
        const bool same_view = view == c->last_view;
        c->last_view = view;
        /* The list area: after a build that did not fill its area, a new view's build gets twice
           what the last one took per pixel plus 8 records per pixel (dragon 1080p: 24.9M records
           used of the 89.5M the RT_LIST_MB cap allows), and the buffer gives back the rest; a build
           that filled its area gets the whole cap again (pixels whose list does not fit take the
           tree: the same bits).  The same view keeps the area its lists were built in. */
        bool list_shrink = false;
        if (c->list_cap_last && c->list_used_last < c->list_cap_last && c->list_npx_last) {
            if (same_view) {
                list_cap = std::min<uint64_t>(list_cap, c->list_cap_last);
            } else {
                const uint64_t est = (2 * c->list_used_last * npx + c->list_npx_last - 1) / c->list_npx_last + 8 * npx;
                list_cap = std::min<uint64_t>(list_cap, est);
                list_shrink = true;
            }
        }
        /* Lists pay for their pre-pass (about one traversal per pixel) within one frame from
           sampleRate 4 on; below, from the second frame of a view on, since they are then reused
           (bunny class 1024^2 at 1 spp: a 2.4-ms pre-pass against a 1.0-ms frame) */
        bool lists = (c->pixel_lists == 1 || (c->pixel_lists < 0 && (c->sample_rate >= 4 || same_view))) && bvh4 &&
                     list_cap > 0;
        if (lists && ensure_tris_capacity(c, (size_t)(kept + list_cap), c->tree_recs, st, list_shrink) != RT_OK) {
            (void)hipGetLastError(); /* out of device memory: no lists this render */
            lists = false;
        }
        const uint64_t n_tiles = (uint64_t)((W + 7) / 8) * ((hl + 7) / 8);
        if (lists && (c->list_px_cap < npx || c->list_tile_cap < n_tiles)) {
            free_dev(c->d_list_code);
            free_dev(c->d_list_tile);
            c->d_list_code = nullptr;
            c->d_list_tile = nullptr;
            c->list_px_cap = c->list_tile_cap = 0;
            c->list_key.clear();
            HIPCHK(c, hipMalloc(&c->d_list_code, npx * sizeof(uint16_t)));
            HIPCHK(c, hipMalloc(&c->d_list_tile, n_tiles * sizeof(uint32_t)));
            c->list_px_cap = npx;
            c->list_tile_cap = n_tiles;
        }
        if (lists && !c->d_list_alloc) HIPCHK(c, hipMalloc(&c->d_list_alloc, sizeof(uint32_t)));
        if (lists) {
            a.list_code = c->d_list_code;
            a.list_tile = c->d_list_tile;
            a.list_base = (uint32_t)kept;
            a.list_cap = (uint32_t)list_cap;
            a.list_alloc = c->d_list_alloc;
        }
        a.tris = c->d_tris;
        /* The lists depend only on the camera, the mesh and tree, the frame shape and the tile —
           like the BVH and the schedule, they are rebuilt when one of those changes and reused
           by the frames in between (GlutCLWindow refines one view over many frames,
           GlutCLWindow.cpp:151-158; a camera move rebuilds them: bench.py cold_frame_ms). */
        bool build_lists = false;
        if (lists) {
            const uintptr_t tp = reinterpret_cast<uintptr_t>(c->d_tris);
            std::vector<uint32_t> key = view;
            key.insert(key.end(), {(uint32_t)list_cap, (uint32_t)tp, (uint32_t)((uint64_t)tp >> 32)});
            build_lists = key != c->list_key;
            c->list_key = key;
        }
        HIPCHK(c, hipEventRecord(c->ev0, st));
        /* a view's first frame of whole pixels: its order from a pilot render (pilot_order) */
        const bool pilot = record_iter && !a.split_chunks && c->schedule_rebuilt && c->pilot_sr > 0 && !c->counting &&
                           c->sample_rate * c->sample_rate >= kPilotMinSpp;
        e = build_lists ? rt_launch_pixel_lists(a, c->d_nodes4, trav == RT_TRAV_BVH4Q ? c->d_nodes4q : nullptr,
                                                c->d_list_code, c->d_list_tile, st)
                        : 0;
        if (e) c->list_key.clear();
        /* (after the lists: the pilot's camera rays take them, as the frame's do; beside the list
           pre-pass on a second stream, through the tree, it ordered the frame worse: 94.96 against
           98.89 ms, profiles/r06m) */
        if (pilot && !e) {
            const int rp = pilot_order(c, a, trav, blocks, st);
            if (rp != RT_OK) return rp;
        }
        HIPCHK(c, hipEventRecord(c->evm, st));
        if (!e && lists && getenv("RT_LIST_STATS")) { /* diagnostics: candidate list lengths */
            std::vector<uint16_t> h((size_t)npx);
            HIPCHK(c, hipMemcpyAsync(h.data(), c->d_list_code, h.size() * 2, hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipStreamSynchronize(st));
            uint64_t b[7] = {}, sum = 0, nl = 0;
            for (uint16_t code : h) {
                const uint32_t v = code == RT_LIST_NONE ? 255u : code == RT_LIST_EMPTY ? 0u : (code & (RT_LIST_MAX - 1u)) + 1u;
                b[v == 0 ? 0 : v <= 8 ? 1 : v <= 16 ? 2 : v <= 24 ? 3 : v <= 32 ? 4 : v <= 64 ? 5 : 6]++;
                if (v <= RT_LIST_MAX) sum += v, nl++;
            }
            fprintf(stderr, "lists: 0:%llu 1-8:%llu 9-16:%llu 17-24:%llu 25-32:%llu 33-64:%llu none:%llu mean %.2f\n",
                    (unsigned long long)b[0], (unsigned long long)b[1], (unsigned long long)b[2],
                    (unsigned long long)b[3], (unsigned long long)b[4], (unsigned long long)b[5],
                    (unsigned long long)b[6], nl ? (double)sum / (double)nl : 0.0);
        }
        if (!e && a.split_chunks) {
            a.n_recs = (uint32_t)std::min<size_t>(c->tris_cap, 0xffffffffu); /* the list area included */
            c->last_hit_depth = false;
            e = split_render(c, a, blocks, st);
        }
        else if (!e) e = rt_launch_tris(a, trav, c->counting, blocks, st);
        if (!e && record_iter) c->iter_recorded = true;
        c->last_long = a.split_chunks ? a.split_n_box : 0u;
        HIPCHK(c, hipEventRecord(c->ev1, st));
        c->info = rt_render_info{};
        c->info.kernel = RT_KERNEL_TRIS;
        c->info.traversal = (uint32_t)trav;
        c->info.grid_blocks = (uint32_t)blocks;
        c->info.lists = lists ? 1u : 0u;
        c->info.lists_rebuilt = build_lists ? 1u : 0u;
        c->info.list_capacity = lists ? list_cap : 0;
        c->info_list_px = lists ? (size_t)npx : 0u;
        c->info.pixels_long = c->last_long;
        c->info.split_chunks = a.split_chunks;
        c->info.split_coop = a.split_chunks && a.split_n_box ? a.split_coop : 0u;
        c->info.split_spec = a.split_chunks ? a.split_spec : 0u;
        c->info.split_hit_depth = a.split_chunks && c->last_hit_depth ? 1u : 0u;
        c->info.schedule_measured = a.tile_order && c->order_measured ? 1u : 0u;
        c->info.schedule_rebuilt = c->schedule_rebuilt ? 1u : 0u;
        c->info.schedule_host_ms = sched_ms;
        c->info.schedule_pilot = pilot ? 1u : 0u;
        c->info_list_pending = lists;
        if (d_stats) {
            std::vector<uint32_t> h((size_t)W * hl * 8);
            HIPCHK(c, hipMemcpyAsync(h.data(), d_stats, h.size() * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipStreamSynchronize(st));
            (void)hipFree(d_stats);
            if (FILE *f = fopen(stats_path, "wb")) {
                fwrite(h.data(), 4, h.size(), f);
                fclose(f);
            }
        }
    } else {
        RtSphLaunch a;
        a.out = dout;
        a.seeds = c->d_seeds;
        a.spheres = c->d_spheres;
        a.n_spheres = (uint32_t)c->spheres.size();
        a.cam = c->cam;
        a.W = W;
        a.H = H;
        a.Wpad = c->wpad;
        a.Hpad = c->hpad;
        a.Hl = hl;
        a.sample_rate = c->sample_rate;
        a.max_depth = c->max_depth;
        a.progressive = prog;
        a.stripe = stripe;
        a.n_ranks = nr;
        a.rank = rk;
        a.stripe_map = smap;
        a.counters = c->d_counters;
        HIPCHK(c, hipEventRecord(c->ev0, st));
        HIPCHK(c, hipEventRecord(c->evm, st));
        e = rt_launch_spheres(a, kernel == RT_KERNEL_SPHERES_SS, st);
        HIPCHK(c, hipEventRecord(c->ev1, st));
        c->info = rt_render_info{};
        c->info.kernel = (uint32_t)kernel;
        c->info_list_pending = false;
    }
    if (e) return hip_fail(c, (hipError_t)e, "kernel launch");
    /* the counters (and a new list build's fill) come back on the render's stream, so that
       rt_synchronize is one stream wait (no blocking copy after it) */
    if (c->h_counters_dev && !c->info.lists_rebuilt) {
        /* counters to the host, added to the running totals and zeroed for the next render, in one kernel */
        const int ek = rt_launch_counters_out(c->d_counters, c->h_counters_dev, c->d_totals, (uint32_t)RT_COUNTER_WORDS,
                                              (uint32_t)((kCounterBytes + kWorkWords * sizeof(uint32_t)) / 8u), st);
        if (ek) return hip_fail(c, (hipError_t)ek, "counter hand-back");
        c->counters_zeroed = true;
    } else {
        const int ek = rt_launch_counters_out(c->d_counters, nullptr, c->d_totals, (uint32_t)RT_COUNTER_WORDS, 0u, st);
        if (ek) return hip_fail(c, (hipError_t)ek, "counter totals");
        HIPCHK(c, hipMemcpyAsync(c->h_counters, c->d_counters, kCounterBytes, hipMemcpyDeviceToHost, st));
    }
    if (c->info.lists_rebuilt)
        HIPCHK(c, hipMemcpyAsync(c->h_counters + RT_COUNTER_WORDS, c->d_list_alloc, sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, st));
    if (st != c->stream) HIPCHK(c, hipEventRecord(c->ev_done, st));
    c->sync_stream = st;
    c->have_timing = true;
    c->last_out = dout;
    c->last_bytes = out_bytes;
    if (!(flags & RT_OUT_DEVICE)) HIPCHK(c, hipMemcpyAsync(out, dout, out_bytes, hipMemcpyDeviceToHost, st));
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_synchronize(rt_ctx *c)
try {
    if (!c) return RT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->sync_stream && c->sync_stream != c->stream) HIPCHK(c, hipStreamSynchronize(c->sync_stream));
    const unsigned long long *h = c->h_counters;
    if (c->info.lists_rebuilt) { /* the list area the new lists took: sizes the next build's area */
        const uint32_t used = (uint32_t)(h[RT_COUNTER_WORDS] & 0xffffffffu);
        c->list_used_last = used;
        c->list_cap_last = c->info.list_capacity;
        c->list_npx_last = c->info_list_px;
    }
    c->last.rays_closest = h[0];
    c->last.rays_shadow = h[1];
    c->last.nodes_visited = h[2];
    c->last.tris_tested = h[3];
    c->last.leaves_visited = h[4];
    c->last.lane_slots = h[5];
    c->last.clocks_traversal = h[6] / 64; /* summed over every lane of a wave */
    c->last.clocks_total = h[7] / 64;
    c->last.rays_skipped = h[RT_CNT_SKIPPED];
    c->last.clocks_shade = h[RT_CNT_SHADE] / 64;
    c->last.pixel_clocks_max = h[10];
    c->last.pixel_rays_max = h[11];
    c->last.pixel_steps_max = h[12];
    c->last.pixels_long = c->last_long;
    c->info.split_repaired = (uint32_t)h[RT_CNT_REPAIR];
    if (h[RT_CNT_GUARD]) { /* a defect guard of the long chains' seed pass: the frame is not the reference's */
        c->info.split_guard = (uint32_t)h[RT_CNT_GUARD];
        char msg[160];
        snprintf(msg, sizeof(msg),
                 "sample-split seed pass: a defect guard fired (flags 0x%x: 1 record index, 2 group stack, 4 round "
                 "bound); the frame is invalid (RT_SPLIT=0 renders whole pixels)",
                 (unsigned)h[RT_CNT_GUARD]);
        return fail(c, RT_ERR_STATE, msg);
    }
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_counter_totals(rt_ctx *c, rt_counters *sum, uint64_t *renders, int reset)
try {
    if (!c || !sum) return RT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->sync_stream && c->sync_stream != c->stream) HIPCHK(c, hipStreamSynchronize(c->sync_stream));
    unsigned long long h[RT_COUNTER_WORDS + 1];
    HIPCHK(c, hipMemcpy(h, c->d_totals, sizeof(h), hipMemcpyDeviceToHost));
    if (reset) HIPCHK(c, hipMemset(c->d_totals, 0, sizeof(h)));
    *sum = rt_counters{};
    sum->rays_closest = h[0];
    sum->rays_shadow = h[1];
    sum->nodes_visited = h[2];
    sum->tris_tested = h[3];
    sum->leaves_visited = h[4];
    sum->lane_slots = h[5];
    sum->clocks_traversal = h[6] / 64;
    sum->clocks_total = h[7] / 64;
    sum->rays_skipped = h[RT_CNT_SKIPPED];
    sum->clocks_shade = h[RT_CNT_SHADE] / 64;
    sum->pixel_clocks_max = h[10];
    sum->pixel_rays_max = h[11];
    sum->pixel_steps_max = h[12];
    if (renders) *renders = h[RT_COUNTER_WORDS];
    if (h[RT_CNT_GUARD]) {
        char msg[160];
        snprintf(msg, sizeof(msg),
                 "rt_counter_totals: a sample-split seed pass defect guard fired in one of the renders (flags 0x%x); "
                 "those frames are invalid",
                 (unsigned)h[RT_CNT_GUARD]);
        return fail(c, RT_ERR_STATE, msg);
    }
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_render(rt_ctx *c, float *out, uint32_t W, uint32_t H, uint32_t prog, int kernel, const rt_tile *tile,
              int flags)
try {
    const int r = rt_render_async(c, out, W, H, prog, kernel, tile, flags, nullptr);
    if (r != RT_OK) return r;
    return rt_synchronize(c); /* cmdQueue.finish(), RayTracerCL.cpp:292 */
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

static int seed_rows_io(rt_ctx *c, const uint32_t *rows, uint32_t n, uint32_t *buf, int flags, bool unpack)
{
    if (!c || (n && (!rows || !buf))) return RT_ERR_ARG;
    if (!c->wpad) return fail(c, RT_ERR_STATE, "no seed layout");
    for (uint32_t i = 0; i < n; ++i)
        if (rows[i] >= c->hpad) return fail(c, RT_ERR_ARG, "seed row out of range");
    if (!n) return RT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t words = 2ull * n * c->wpad;
    if (c->halo_rows_cap < n) {
        free_dev(c->d_halo_rows);
        c->d_halo_rows = nullptr;
        c->halo_rows_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_halo_rows, n * sizeof(uint32_t)));
        c->halo_rows_cap = n;
    }
    uint32_t *dbuf = buf;
    const bool on_device = (flags & RT_OUT_DEVICE) != 0;
    if (!on_device) {
        if (c->halo_buf_cap < words) {
            free_dev(c->d_halo_buf);
            c->d_halo_buf = nullptr;
            c->halo_buf_cap = 0;
            HIPCHK(c, hipMalloc(&c->d_halo_buf, words * sizeof(uint32_t)));
            c->halo_buf_cap = words;
        }
        dbuf = c->d_halo_buf;
        if (unpack) HIPCHK(c, hipMemcpyAsync(dbuf, buf, words * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipMemcpyAsync(c->d_halo_rows, rows, n * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    const int e = rt_launch_seed_rows(c->d_seeds, c->wpad, c->hpad, c->d_halo_rows, n, dbuf, unpack, c->stream);
    if (e) return hip_fail(c, (hipError_t)e, "seed-row kernel");
    if (!on_device && !unpack)
        HIPCHK(c, hipMemcpyAsync(buf, dbuf, words * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_pack_seed_rows(rt_ctx *c, const uint32_t *rows, uint32_t n, uint32_t *buf, int flags)
try {
    return seed_rows_io(c, rows, n, buf, flags, false);
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_unpack_seed_rows(rt_ctx *c, const uint32_t *rows, uint32_t n, const uint32_t *buf, int flags)
try {
    return seed_rows_io(c, rows, n, const_cast<uint32_t *>(buf), flags, true);
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_read(rt_ctx *c, float *host, size_t n_floats)
try {
    if (!c || !host) return RT_ERR_ARG;
    if (!c->last_out) return fail(c, RT_ERR_STATE, "rt_read before any render");
    if (n_floats * sizeof(float) < c->last_bytes) return fail(c, RT_ERR_ARG, "rt_read: host buffer too small");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(host, c->last_out, c->last_bytes, hipMemcpyDeviceToHost));
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_last_render_info(rt_ctx *c, rt_render_info *out)
try {
    if (!c || !out) return RT_ERR_ARG;
    if (c->info_list_pending) { /* how much of the list area the render's lists took */
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        uint32_t used = 0;
        HIPCHK(c, hipMemcpy(&used, c->d_list_alloc, sizeof(used), hipMemcpyDeviceToHost));
        c->info.list_records = std::min<uint64_t>(used, c->info.list_capacity);
        const size_t npx = c->info_list_px;
        std::vector<uint16_t> h(npx);
        if (npx) HIPCHK(c, hipMemcpy(h.data(), c->d_list_code, npx * 2, hipMemcpyDeviceToHost));
        uint32_t tree = 0;
        for (uint16_t v : h) tree += v == RT_LIST_NONE ? 1u : 0u;
        c->info.list_pixels_tree = tree;
        c->info_list_pending = false;
    }
    *out = c->info;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_last_long_chains(rt_ctx *c, uint32_t *out, uint32_t cap, uint32_t *n)
try {
    if (!c || !n || (cap && !out)) return RT_ERR_ARG;
    *n = c->last_long;
    const uint32_t k = std::min(cap, c->last_long);
    if (!k) return RT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, c->d_split_box, (size_t)k * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_get_counters(const rt_ctx *c, rt_counters *out)
try {
    if (!c || !out) return RT_ERR_ARG;
    *out = c->last;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_set_counting(rt_ctx *c, int enable)
try {
    if (!c) return RT_ERR_ARG;
    c->counting = enable != 0;
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_last_kernel_split_ms(const rt_ctx *c, float *prepass_ms, float *main_ms)
try {
    if (!c || !prepass_ms || !main_ms) return RT_ERR_ARG;
    if (!c->have_timing) return RT_ERR_STATE;
    if (hipEventSynchronize(c->ev1) != hipSuccess) return RT_ERR_HIP;
    if (hipEventElapsedTime(prepass_ms, c->ev0, c->evm) != hipSuccess) return RT_ERR_HIP;
    return hipEventElapsedTime(main_ms, c->evm, c->ev1) == hipSuccess ? RT_OK : RT_ERR_HIP;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_last_kernel_ms(const rt_ctx *c, float *ms)
try {
    if (!c || !ms) return RT_ERR_ARG;
    if (!c->have_timing) return RT_ERR_STATE;
    if (hipEventSynchronize(c->ev1) != hipSuccess) return RT_ERR_HIP;
    return hipEventElapsedTime(ms, c->ev0, c->ev1) == hipSuccess ? RT_OK : RT_ERR_HIP;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

int rt_trace_rays(rt_ctx *c, const rt_ray *rays, uint32_t n, int any_hit, int32_t *out_idx, float *out_t)
try {
    if (!c || !rays || !out_idx) return RT_ERR_ARG;
    if (!c->n_tris) return fail(c, RT_ERR_NO_MESH, "no mesh set");
    if (n == 0) return RT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    rt_ray *d_rays = nullptr;
    int32_t *d_idx = nullptr;
    float *d_t = nullptr;
    auto cleanup = [&]() {
        free_dev(d_rays);
        free_dev(d_idx);
        free_dev(d_t);
    };
    hipError_t e = hipMalloc(&d_rays, n * sizeof(rt_ray));
    if (e == hipSuccess) e = hipMalloc(&d_idx, n * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&d_t, n * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(d_rays, rays, n * sizeof(rt_ray), hipMemcpyHostToDevice);
    const uint32_t cap = spill_cap(c);
    if (e == hipSuccess && cap) {
        const int rs = ensure_spill(c, (size_t)n * cap);
        if (rs != RT_OK) {
            cleanup();
            return rs;
        }
    }
    if (e == hipSuccess) e = hipEventRecord(c->ev0, c->stream);
    if (e == hipSuccess) e = hipEventRecord(c->evm, c->stream);
    if (e == hipSuccess) {
        /* The tree leaves out triangles no UNIT-length ray can hit (rt_bvh.cpp never_hit); the
           kernels only trace unit directions, but a caller's rays may be longer: then the
           linear loop over every triangle answers (same semantics, all triangles). */
        int kind = trav_kind(c);
        if (c->bvh.n_hit < c->n_tris)
            for (uint32_t i = 0; i < n; ++i) {
                const rt_vec3 &d = rays[i].d;
                if (!((double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z <= 1.002)) { /* |d| <= 1.001 */
                    kind = RT_TRAV_LINEAR;
                    break;
                }
            }
        c->counters_zeroed = false; /* this trace leaves its counts there */
        if (c->sync_stream && c->sync_stream != c->stream) {
            e = hipStreamWaitEvent(c->stream, c->ev_done, 0); /* (recorded on the caller's stream) */
        }
        if (e == hipSuccess && c->counting) e = hipMemsetAsync(c->d_counters, 0, RT_COUNTER_WORDS * sizeof(unsigned long long), c->stream);
        if (e == hipSuccess) {
            const int le = rt_launch_trace_rays(trav_nodes(c), c->d_tris, c->n_tris, d_rays, n, any_hit, kind, c->d_spill,
                                                cap, d_idx, d_t, c->counting ? c->d_counters : nullptr, c->stream);
            e = (hipError_t)le;
        }
    }
    if (e == hipSuccess) e = hipEventRecord(c->ev1, c->stream);
    if (e == hipSuccess) c->have_timing = true;
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out_idx, d_idx, n * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && out_t) e = hipMemcpy(out_t, d_t, n * sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess && c->counting) { /* rt_get_counters: queries and records of these rays */
        unsigned long long h[RT_N_COUNTERS];
        e = hipMemcpy(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost);
        c->last = rt_counters{};
        c->last.rays_closest = h[0];
        c->last.rays_shadow = h[1];
        c->last.nodes_visited = h[2];
        c->last.tris_tested = h[3];
        c->last.leaves_visited = h[4];
    }
    cleanup();
    if (e != hipSuccess) return hip_fail(c, e, "rt_trace_rays");
    return RT_OK;
} RT_CATCH(c ? &const_cast<rt_ctx *>(c)->err : nullptr)

/* ---- synthetic meshes ---------------------------------------------------- */

static void mesh_grid(uint32_t n_tris, uint32_t *nt, uint32_t *np)
{
    uint32_t t = 2;
    while (4ull * t * (t - 1) < n_tris) ++t;
    *nt = t;     /* latitude bands */
    *np = 2 * t; /* longitude segments */
}

uint32_t rt_mesh_vertex_count(uint32_t n_tris)
{
    uint32_t nt, np;
    mesh_grid(n_tris, &nt, &np);
    return 2 + (nt - 1) * np;
}

int rt_make_mesh(uint32_t n_tris, float cx, float cy, float cz, float r, float *verts, int32_t *idx)
try {
    if (!n_tris || !verts || !idx) return RT_ERR_ARG;
    uint32_t nt, np;
    mesh_grid(n_tris, &nt, &np);
    const float pi = RT_M_PI_F;
    auto put = [&](uint32_t v, float th, float ph) {
        /* displaced sphere: two bump frequencies, deterministic (rt_math.h only) */
        const float bump = 0.08f * rt_sinf(9.0f * th) * rt_sinf(8.0f * ph) +
                           0.04f * rt_sinf(23.0f * th + 3.0f * ph) * rt_cosf(19.0f * ph - 2.0f * th);
        const float rr = r * (1.0f + bump);
        const float st = rt_sinf(th), ct = rt_cosf(th);
        verts[3ull * v + 0] = cx + rr * st * rt_cosf(ph);
        verts[3ull * v + 1] = cy + rr * ct;
        verts[3ull * v + 2] = cz + rr * st * rt_sinf(ph);
    };
    const uint32_t top = 0, bottom = 1 + (nt - 1) * np;
    put(top, 0.0f, 0.0f);
    put(bottom, pi, 0.0f);
    for (uint32_t i = 1; i < nt; ++i) {
        const float th = pi * (float)i / (float)nt;
        for (uint32_t j = 0; j < np; ++j) put(1 + (i - 1) * np + j, th, 2.0f * pi * (float)j / (float)np);
    }
    auto ring = [&](uint32_t i, uint32_t j) -> int32_t { return (int32_t)(1 + (i - 1) * np + (j % np)); };
    /* winding chosen so that cross(e2, e1) (the reference's normal,
       rtcommon.h:389) points outward */
    uint64_t k = 0;
    auto tri = [&](int32_t a, int32_t b, int32_t c) {
        if (k >= n_tris) return;
        idx[3 * k + 0] = a;
        idx[3 * k + 1] = b;
        idx[3 * k + 2] = c;
        ++k;
    };
    for (uint32_t j = 0; j < np; ++j) tri((int32_t)top, ring(1, j), ring(1, j + 1));
    for (uint32_t i = 1; i + 1 < nt; ++i)
        for (uint32_t j = 0; j < np; ++j) {
            tri(ring(i, j), ring(i + 1, j), ring(i + 1, j + 1));
            tri(ring(i, j), ring(i + 1, j + 1), ring(i, j + 1));
        }
    for (uint32_t j = 0; j < np; ++j) tri(ring(nt - 1, j), (int32_t)bottom, ring(nt - 1, j + 1));
    return k == n_tris ? RT_OK : RT_ERR_STATE;
} RT_CATCH(nullptr)

} /* extern "C" */
