/*
 * rt_comm.hip — multi-GPU from the native host: RCCL communicator, frame assembly
 * and the seed-row halo behind the C-ABI (include/pathtracer_rt.h, "multi-GPU").
 *
 * The reference drives one OpenCL device from GlutCLWindow (RayTracerCL.cpp:52-145,
 * :217-307).  Sharded, every pixel of a frame stays independent (own seed slot, own
 * read-modify-write of its output pixel, raytracer.cl:20-30, :207-242), so a rank
 * renders its row stripes (rt_tile: interleaved, or dealt by a cost-balanced owner map,
 * rt_partition_stripes) with a full scene/BVH replica and the
 * only data-path exchange is the frame assembly on the root: grouped ncclSend /
 * ncclRecv, one point-to-point xGMI transfer per sender, into a staging buffer that one
 * kernel scatters into the frame.  raytrace's row-shifted seeds (get_seed/put_seed,
 * raytracer.cl:20-30) add the seed-row halo: before a progressive frame with shift s,
 * the rows a rank reads are fetched from their last writer (rt_seed_halo_plan), packed
 * and moved with the same grouped point-to-point calls.
 *
 * Same protocol as pathtracer.cl_amd/dist.py (the torch.distributed form), so a C++
 * host without Python shards the same way.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "pathtracer_rt.h"
#include "rt_internal.h"

#define RT_COMM_MAX_RANKS 64

struct rt_comm {
    ncclComm_t nccl = nullptr;
    int n_ranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    float *stage = nullptr; /* root: the other ranks' tiles, rank order */
    size_t stage_bytes = 0;
    float *tile = nullptr; /* rt_comm_render: this rank's compact tile (persists: progression mixes into it) */
    size_t tile_bytes = 0;
    uint32_t *halo_send = nullptr, *halo_recv = nullptr;
    size_t halo_send_bytes = 0, halo_recv_bytes = 0;
    /* seed-row halo state: last writer of every seed row, valid for this frame shape */
    std::vector<int32_t> writer;
    uint32_t key_w = 0, key_h = 0, key_stripe = 0, hpad = 0, wpad = 0;
    const rt_ctx *key_ctx = nullptr;
    /* rt_comm_render's partition and the last frame's owner map (empty: interleaved) */
    int partition = RT_PARTITION_BALANCED;
    std::vector<uint32_t> owner;
    uint32_t *d_bcast = nullptr; /* the root's map, broadcast to the ranks when a view's map is made */
    size_t bcast_bytes = 0;
    /* k_assemble's per-stripe (owner << 24 | the stripe's index in its owner's tile), and its host copy */
    uint32_t *d_info = nullptr;
    size_t info_bytes = 0;
    std::vector<uint32_t> info_h;
};

namespace {

int fail(rt_comm *m, int code, const std::string &what)
{
    if (m) m->err = what;
    return code;
}

int hip_fail(rt_comm *m, hipError_t e, const char *what)
{
    return fail(m, RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int nccl_fail(rt_comm *m, ncclResult_t r, const char *what)
{
    return fail(m, RT_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

#define HIPC(m, call)                                                 \
    do {                                                              \
        hipError_t e_ = (call);                                       \
        if (e_ != hipSuccess) return hip_fail((m), e_, #call);        \
    } while (0)
#define NCCLC(m, call)                                                \
    do {                                                              \
        ncclResult_t r_ = (call);                                     \
        if (r_ != ncclSuccess) return nccl_fail((m), r_, #call);      \
    } while (0)

template <class T>
int grow(rt_comm *m, T **p, size_t *cap_bytes, size_t bytes)
{
    if (*cap_bytes >= bytes) return RT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap_bytes = 0;
    HIPC(m, hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(bytes, 256)));
    *cap_bytes = bytes;
    return RT_OK;
}

/* Owner of global row y (rt_tile: the owner map, or interleaved stripes). */
inline uint32_t row_rank(uint32_t y, uint32_t stripe, uint32_t n, const uint32_t *owner)
{
    return owner ? owner[y / stripe] : (y / stripe) % n;
}

struct TilePtrs {
    const float4 *p[RT_COMM_MAX_RANKS];
};

/* One thread per output pixel: gather the pixel from its owner's compact tile (info[stripe] =
   owner << 24 | the stripe's index among its owner's).  Reads and writes are row-contiguous
   float4 (16 B per lane, coalesced). */
__global__ void __launch_bounds__(256) k_assemble(TilePtrs tiles, const uint32_t *__restrict__ info, uint32_t W,
                                                  uint32_t H, uint32_t stripe, float4 *frame)
{
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t y = blockIdx.y;
    if (x >= W || y >= H) return;
    const uint32_t v = info[y / stripe];
    const size_t local = (size_t)(v & 0xffffffu) * stripe + y % stripe;
    frame[(size_t)y * W + x] = tiles.p[v >> 24][local * W + x];
}

/* The assembly's stripe table for a partition, uploaded when it changes (the gathers end with a
   stream synchronisation, so no assembly is reading the old one). */
int stripe_info(rt_comm *m, uint32_t H, uint32_t stripe, uint32_t n, const uint32_t *owner)
{
    const uint32_t ns = (H + stripe - 1) / stripe;
    std::vector<uint32_t> info(ns), next(n, 0);
    for (uint32_t s = 0; s < ns; ++s) {
        const uint32_t r = owner ? owner[s] : s % n;
        if (r >= n) return fail(m, RT_ERR_ARG, "stripe owner out of range");
        info[s] = r << 24 | next[r]++;
    }
    if (info == m->info_h && m->d_info) return RT_OK;
    if (int e = grow(m, &m->d_info, &m->info_bytes, ns * sizeof(uint32_t))) return e;
    HIPC(m, hipMemcpy(m->d_info, info.data(), ns * sizeof(uint32_t), hipMemcpyHostToDevice));
    m->info_h = std::move(info);
    return RT_OK;
}

int assemble(rt_comm *m, const float *const *tiles, uint32_t n, uint32_t W, uint32_t H, uint32_t stripe,
             const uint32_t *owner, float *frame, hipStream_t st)
{
    if (int e = stripe_info(m, H, stripe, n, owner)) return e;
    TilePtrs tp{};
    for (uint32_t r = 0; r < n; ++r) tp.p[r] = reinterpret_cast<const float4 *>(tiles[r]);
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(k_assemble, grid, dim3(256), 0, st, tp, m->d_info, W, H, stripe,
                       reinterpret_cast<float4 *>(frame));
    HIPC(m, hipGetLastError());
    return RT_OK;
}

uint32_t tile_rows(uint32_t H, uint32_t stripe, uint32_t n, uint32_t r, const uint32_t *owner)
{
    const rt_tile t{stripe, n, r, owner};
    return rt_tile_rows(H, &t);
}

} // namespace

extern "C" {

int rt_comm_get_unique_id(uint8_t id[RT_COMM_ID_BYTES])
try {
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES != NCCL_UNIQUE_ID_BYTES");
    if (!id) return RT_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return RT_ERR_HIP;
    std::memcpy(id, &u, sizeof(u));
    return RT_OK;
} RT_CATCH(nullptr)

int rt_comm_create(const uint8_t id[RT_COMM_ID_BYTES], int n_ranks, int rank, int device, rt_comm **out)
try {
    if (!out) return RT_ERR_ARG;
    *out = nullptr;
    if (!id || n_ranks < 1 || n_ranks > RT_COMM_MAX_RANKS || rank < 0 || rank >= n_ranks) return RT_ERR_ARG;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return RT_ERR_HIP;
    if (device < 0 || device >= nd) return RT_ERR_ARG;
    rt_comm *m = new (std::nothrow) rt_comm();
    if (!m) return RT_ERR_ALLOC;
    m->n_ranks = n_ranks;
    m->rank = rank;
    m->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
        ncclCommInitRank(&m->nccl, n_ranks, u, rank) != ncclSuccess) {
        rt_comm_destroy(m);
        return RT_ERR_HIP;
    }
    *out = m;
    return RT_OK;
} RT_CATCH(nullptr)

int rt_comm_destroy(rt_comm *m)
try {
    if (!m) return RT_ERR_ARG;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->nccl) (void)ncclCommDestroy(m->nccl);
    for (void *p : {(void *)m->stage, (void *)m->tile, (void *)m->halo_send, (void *)m->halo_recv, (void *)m->d_bcast,
                    (void *)m->d_info})
        if (p) (void)hipFree(p);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
    return RT_OK;
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

const char *rt_comm_last_error(const rt_comm *m) { return m ? m->err.c_str() : "null communicator"; }

int rt_comm_count(const rt_comm *m, int *n)
try {
    if (!m || !n) return RT_ERR_ARG;
    return ncclCommCount(m->nccl, n) == ncclSuccess ? RT_OK : RT_ERR_HIP;
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

int rt_assemble_tiles(const float *const *tiles, uint32_t n, uint32_t W, uint32_t H, uint32_t stripe,
                      const uint32_t *owner, float *frame, int device)
try {
    if (!tiles || !frame || n < 1 || n > RT_COMM_MAX_RANKS || stripe == 0) return RT_ERR_ARG;
    if (owner)
        for (uint32_t s = 0; s < (H + stripe - 1) / stripe; ++s)
            if (owner[s] >= n) return RT_ERR_ARG;
    for (uint32_t r = 0; r < n; ++r)
        if (!tiles[r] && tile_rows(H, stripe, n, r, owner) > 0) return RT_ERR_ARG;
    if (W == 0 || H == 0) return RT_OK;
    if (hipSetDevice(device) != hipSuccess) return RT_ERR_HIP;
    rt_comm tmp;
    int st = assemble(&tmp, tiles, n, W, H, stripe, owner, frame, nullptr);
    if (st == RT_OK && hipStreamSynchronize(nullptr) != hipSuccess) st = RT_ERR_HIP;
    if (tmp.d_info) (void)hipFree(tmp.d_info);
    return st == RT_OK ? RT_OK : RT_ERR_HIP;
} RT_CATCH(nullptr)

int rt_comm_gather_frame(rt_comm *m, const float *tile, float *frame, uint32_t W, uint32_t H, uint32_t stripe,
                         const uint32_t *owner, int root)
try {
    if (!m) return RT_ERR_ARG;
    const uint32_t n = (uint32_t)m->n_ranks, me = (uint32_t)m->rank;
    if (stripe == 0 || root < 0 || root >= m->n_ranks) return fail(m, RT_ERR_ARG, "bad stripe or root");
    if (W == 0 || H == 0) return RT_OK;
    const size_t row_floats = (size_t)W * 4;
    const uint32_t mine = tile_rows(H, stripe, n, me, owner);
    if (mine && !tile) return fail(m, RT_ERR_ARG, "null tile");
    if (me == (uint32_t)root && !frame) return fail(m, RT_ERR_ARG, "null frame on root");
    HIPC(m, hipSetDevice(m->device));
    std::vector<const float *> ptrs(n, nullptr);
    if (me == (uint32_t)root) {
        size_t total = 0;
        for (uint32_t r = 0; r < n; ++r)
            if (r != me) total += tile_rows(H, stripe, n, r, owner) * row_floats;
        if (int e = grow(m, &m->stage, &m->stage_bytes, total * sizeof(float))) return e;
        size_t off = 0;
        NCCLC(m, ncclGroupStart());
        for (uint32_t r = 0; r < n; ++r) {
            const size_t cnt = tile_rows(H, stripe, n, r, owner) * row_floats;
            if (r == me) {
                ptrs[r] = tile;
                continue;
            }
            ptrs[r] = m->stage + off;
            if (cnt) NCCLC(m, ncclRecv(m->stage + off, cnt, ncclFloat32, (int)r, m->nccl, m->stream));
            off += cnt;
        }
        NCCLC(m, ncclGroupEnd());
        if (int e = assemble(m, ptrs.data(), n, W, H, stripe, owner, frame, m->stream)) return e;
    } else if (mine) {
        NCCLC(m, ncclSend(tile, mine * row_floats, ncclFloat32, root, m->nccl, m->stream));
    }
    HIPC(m, hipStreamSynchronize(m->stream));
    return RT_OK;
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

int rt_seed_halo_plan(int32_t *writer, uint32_t H, uint32_t hpad, uint32_t stripe, uint32_t n, const uint32_t *owner,
                      uint32_t shift, uint32_t *src, uint32_t *dst, uint32_t *rows, uint32_t *n_moves)
try {
    if (!writer || !n_moves || stripe == 0 || n == 0 || hpad < H) return RT_ERR_ARG;
    if (owner)
        for (uint32_t s = 0; s < (H + stripe - 1) / stripe; ++s)
            if (owner[s] >= n) return RT_ERR_ARG;
    /* moves grouped by (src, dst) pair in pair order, rows in pixel-row order within a
       pair (the order dist.SeedHalo.plan produces) */
    std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> moves;
    for (uint32_t y = 0; y < H; ++y) {
        const uint32_t r = (uint32_t)(((uint64_t)y + shift) % hpad);
        const int32_t w = writer[r];
        const uint32_t d = row_rank(y, stripe, n, owner);
        if (w >= 0 && (uint32_t)w != d) moves[{(uint32_t)w, d}].push_back(r);
    }
    uint32_t k = 0;
    for (auto &kv : moves)
        for (uint32_t r : kv.second) {
            if (!src || !dst || !rows) return RT_ERR_ARG;
            src[k] = kv.first.first;
            dst[k] = kv.first.second;
            rows[k] = r;
            ++k;
        }
    *n_moves = k;
    for (uint32_t y = 0; y < H; ++y) writer[((uint64_t)y + shift) % hpad] = (int32_t)row_rank(y, stripe, n, owner);
    return RT_OK;
} RT_CATCH(nullptr)

int rt_seed_halo_peer_blocks(const uint32_t *src, const uint32_t *dst, const uint32_t *rows, uint32_t k, uint32_t n,
                             uint32_t me, uint32_t *send_rows, uint32_t *send_counts, uint32_t *recv_rows,
                             uint32_t *recv_counts)
try {
    if (n == 0 || me >= n || !send_counts || !recv_counts || (k && (!src || !dst || !rows || !send_rows || !recv_rows)))
        return RT_ERR_ARG;
    std::vector<std::vector<uint32_t>> to(n), from(n);
    for (uint32_t i = 0; i < k; ++i) {
        if (src[i] >= n || dst[i] >= n) return RT_ERR_ARG;
        if (src[i] == me) to[dst[i]].push_back(rows[i]);
        if (dst[i] == me) from[src[i]].push_back(rows[i]);
    }
    size_t so = 0, ro = 0;
    for (uint32_t p = 0; p < n; ++p) {
        send_counts[p] = (uint32_t)to[p].size();
        recv_counts[p] = (uint32_t)from[p].size();
        for (uint32_t r : to[p]) send_rows[so++] = r;
        for (uint32_t r : from[p]) recv_rows[ro++] = r;
    }
    return RT_OK;
} RT_CATCH(nullptr)

int rt_comm_reset_halo(rt_comm *m)
try {
    if (!m) return RT_ERR_ARG;
    m->writer.clear();
    m->key_ctx = nullptr;
    return RT_OK;
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

int rt_comm_render(rt_comm *m, rt_ctx *c, float *frame, uint32_t W, uint32_t H, uint32_t prog, int kernel,
                   uint32_t stripe, int root)
try {
    if (!m || !c) return RT_ERR_ARG;
    if (stripe == 0 || root < 0 || root >= m->n_ranks) return fail(m, RT_ERR_ARG, "bad stripe or root");
    if (W == 0 || H == 0) return RT_OK;
    const uint32_t n = (uint32_t)m->n_ranks, me = (uint32_t)m->rank;
    HIPC(m, hipSetDevice(m->device));
    /* the partition: triangle frames dealt by cost (rt_partition_stripes, per view; every rank takes
       the root's map, broadcast whenever a view's map is made), sphere frames interleaved */
    const uint32_t ns = (H + stripe - 1) / stripe;
    if (m->partition == RT_PARTITION_BALANCED && kernel == RT_KERNEL_TRIS && n > 1) {
        std::vector<uint32_t> own(ns);
        int made = 0;
        const int pe = rt_partition_stripes(c, W, H, stripe, n, own.data(), &made);
        if (pe) return fail(m, pe, std::string("rt_partition_stripes: ") + rt_last_error(c));
        if (made) { /* (every rank makes it for the same frames: the same view changes reach them all) */
            if (int e = grow(m, &m->d_bcast, &m->bcast_bytes, ns * sizeof(uint32_t))) return e;
            HIPC(m, hipMemcpy(m->d_bcast, own.data(), ns * sizeof(uint32_t), hipMemcpyHostToDevice));
            NCCLC(m, ncclBroadcast(m->d_bcast, m->d_bcast, ns, ncclUint32, root, m->nccl, m->stream));
            HIPC(m, hipStreamSynchronize(m->stream));
            HIPC(m, hipMemcpy(own.data(), m->d_bcast, ns * sizeof(uint32_t), hipMemcpyDeviceToHost));
            m->owner = std::move(own);
        } else if (own != m->owner) {
            m->owner = std::move(own); /* (a cached map this communicator has not used: the same on every rank) */
        }
    } else {
        m->owner.clear();
    }
    const uint32_t *owner = m->owner.empty() ? nullptr : m->owner.data();
    const rt_tile tile{stripe, n, me, owner};
    const uint32_t mine = rt_tile_rows(H, &tile);
    if (int e = grow(m, &m->tile, &m->tile_bytes, (size_t)std::max(mine, 1u) * W * 4 * sizeof(float))) return e;

    /* halo state belongs to one frame shape on one context: a new shape regenerates the
       seeds identically on every rank (rt_render), so nothing is stale */
    const bool fresh = m->writer.empty() || m->key_ctx != c || m->key_w != W || m->key_h != H ||
                       m->key_stripe != stripe;
    /* the rows this frame reads: raytrace shifts them by the progression, the other kernels read
       row y (raytracer.cl:20-30, :142-144, :207-209) */
    const uint32_t shift = kernel == RT_KERNEL_SPHERES ? prog : 0u;
    int flags = RT_OUT_DEVICE;
    if (n > 1) flags |= RT_SEEDS_HALO;
    if (n > 1 && !fresh) {
        std::vector<uint32_t> src(H), dst(H), rows(H);
        std::vector<int32_t> w = m->writer; /* committed after the render */
        uint32_t k = 0;
        if (rt_seed_halo_plan(w.data(), H, m->hpad, stripe, n, owner, shift, src.data(), dst.data(), rows.data(), &k))
            return fail(m, RT_ERR_STATE, "halo plan");
        /* my sends and receives, one contiguous packed block per peer */
        std::vector<uint32_t> to_rows(k), to_cnt(n), from_rows(k), from_cnt(n);
        if (rt_seed_halo_peer_blocks(src.data(), dst.data(), rows.data(), k, n, me, to_rows.data(), to_cnt.data(),
                                     from_rows.data(), from_cnt.data()))
            return fail(m, RT_ERR_STATE, "halo peer blocks");
        size_t ns = 0, nr = 0;
        for (uint32_t p = 0; p < n; ++p) {
            ns += to_cnt[p];
            nr += from_cnt[p];
        }
        const size_t row_words = 2ull * m->wpad;
        if (ns + nr) {
            if (int e = grow(m, &m->halo_send, &m->halo_send_bytes, ns * row_words * 4)) return e;
            if (int e = grow(m, &m->halo_recv, &m->halo_recv_bytes, nr * row_words * 4)) return e;
            /* one packed block ([plane][row][x], rt_pack_seed_rows) per peer, back to back */
            for (uint32_t p = 0, so = 0; p < n; so += to_cnt[p], ++p)
                if (to_cnt[p]) {
                    const int e = rt_pack_seed_rows(c, to_rows.data() + so, to_cnt[p], m->halo_send + so * row_words,
                                                    RT_OUT_DEVICE);
                    if (e) return fail(m, e, std::string("rt_pack_seed_rows: ") + rt_last_error(c));
                }
            NCCLC(m, ncclGroupStart());
            size_t so = 0, ro = 0;
            for (uint32_t p = 0; p < n; ++p) {
                if (to_cnt[p]) {
                    NCCLC(m, ncclSend(m->halo_send + so * row_words, to_cnt[p] * row_words, ncclUint32, (int)p,
                                      m->nccl, m->stream));
                    so += to_cnt[p];
                }
                if (from_cnt[p]) {
                    NCCLC(m, ncclRecv(m->halo_recv + ro * row_words, from_cnt[p] * row_words, ncclUint32, (int)p,
                                      m->nccl, m->stream));
                    ro += from_cnt[p];
                }
            }
            NCCLC(m, ncclGroupEnd());
            HIPC(m, hipStreamSynchronize(m->stream));
            for (uint32_t p = 0, ro2 = 0; p < n; ro2 += from_cnt[p], ++p)
                if (from_cnt[p]) {
                    const int e = rt_unpack_seed_rows(c, from_rows.data() + ro2, from_cnt[p],
                                                      m->halo_recv + ro2 * row_words, RT_OUT_DEVICE);
                    if (e) return fail(m, e, std::string("rt_unpack_seed_rows: ") + rt_last_error(c));
                }
        }
    }
    const int e = rt_render(c, m->tile, W, H, prog, kernel, &tile, flags);
    if (e) return fail(m, e, std::string("rt_render: ") + rt_last_error(c));
    if (fresh) {
        if (rt_seed_layout(c, &m->wpad, &m->hpad) != RT_OK) return fail(m, RT_ERR_STATE, "no seed layout");
        m->writer.assign(m->hpad, -1);
        m->key_ctx = c;
        m->key_w = W;
        m->key_h = H;
        m->key_stripe = stripe;
    }
    /* record this frame's seed writes: raytrace writes row (y + prog) % Hpad, the other
       kernels row y */
    for (uint32_t y = 0; y < H; ++y)
        m->writer[((uint64_t)y + shift) % m->hpad] = (int32_t)row_rank(y, stripe, n, owner);
    return rt_comm_gather_frame(m, m->tile, frame, W, H, stripe, owner, root);
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

int rt_comm_set_partition(rt_comm *m, int mode)
try {
    if (!m || (mode != RT_PARTITION_INTERLEAVED && mode != RT_PARTITION_BALANCED)) return RT_ERR_ARG;
    m->partition = mode;
    return RT_OK;
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

int rt_comm_last_partition(const rt_comm *m, uint32_t *owner, uint32_t cap, uint32_t *n)
try {
    if (!m || !n || (cap && !owner)) return RT_ERR_ARG;
    *n = (uint32_t)m->owner.size();
    std::copy(m->owner.begin(), m->owner.begin() + std::min<size_t>(cap, m->owner.size()), owner);
    return RT_OK;
} RT_CATCH(m ? &const_cast<rt_comm *>(m)->err : nullptr)

} /* extern "C" */
