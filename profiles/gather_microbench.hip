/*
 * gather_microbench.hip — how should a wave fetch 64 lanes' divergent 64-B records?
 *
 * The traversal step of k_tris fetches, per lane, one 64-B record (a compressed
 * 4-wide node) whose index depends on the previous record (a dependent chain),
 * as 4 global_load_dwordx4 per lane: every instruction touches up to 64 different
 * cache lines with 16 B each.  This measures that against a transposed fetch in
 * which the 4 lanes of a quad load the 4 quarters of ONE lane's record per
 * instruction (LDS-DMA, global_load_lds_dwordx4), so that each instruction touches
 * at most 16 lines with 64 contiguous bytes each, and every lane then reads its
 * own record back from LDS (4 ds_read_b128).
 *
 *   hipcc --offload-arch=gfx950 -O3 -o gather_microbench gather_microbench.hip
 *   ./gather_microbench [table_MB] [steps] [distinct_records_per_wave]
 *
 * Records per wave-step are drawn from G distinct records (G = 64: every lane its
 * own; smaller G: lanes share records, as coherent rays do near the root).
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                                 \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int kBlock = 256;

template <int CTRL> __device__ __forceinline__ uint32_t dpp(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
/* quad_perm rotating quad-mates by M */
template <int M> constexpr int rot_ctrl()
{
    return ((4 - M) & 3) | (((5 - M) & 3) << 2) | (((6 - M) & 3) << 4) | (((7 - M) & 3) << 6);
}
template <int M> __device__ __forceinline__ uint32_t round_m(const uint4 (&v)[4], uint32_t q)
{
    const uint32_t idx = (q + 4 - M) & 3;
    const uint32_t x = idx == 0 ? v[0].x : idx == 1 ? v[1].x : idx == 2 ? v[2].x : v[3].x;
    const uint32_t y = idx == 0 ? v[0].y : idx == 1 ? v[1].y : idx == 2 ? v[2].y : v[3].y;
    const uint32_t z = idx == 0 ? v[0].z : idx == 1 ? v[1].z : idx == 2 ? v[2].z : v[3].z;
    const uint32_t w = idx == 0 ? v[0].w : idx == 1 ? v[1].w : idx == 2 ? v[2].w : v[3].w;
    uint32_t h = dpp<rot_ctrl<M>()>(x);
    h += dpp<rot_ctrl<M>()>(y);
    h ^= dpp<rot_ctrl<M>()>(z);
    h += dpp<rot_ctrl<M>()>(w);
    return h;
}

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

/* the lane's next record: a function of the data it just read (dependent chain),
   shared by the lanes with equal (lane % G) */
__device__ __forceinline__ uint32_t next_rec(uint32_t prev, uint32_t lane, uint32_t G, uint32_t n)
{
    return mix(prev * 0x9e3779b9U + (lane % G)) % n;
}

/* A: every lane loads its own record with 4 dwordx4 */
__global__ __launch_bounds__(kBlock, 5) void k_direct(const uint4 *__restrict__ tab, uint32_t n, int steps, uint32_t G,
                                                     uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63;
    uint32_t wave_seed = mix(blockIdx.x * 4 + (threadIdx.x >> 6));
    uint32_t r = next_rec(wave_seed, lane, G, n);
    uint32_t acc = 0;
    for (int s = 0; s < steps; ++s) {
        const uint4 *p = tab + 4 * (size_t)r;
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        const uint32_t h = a.x ^ b.y ^ c.z ^ d.w;
        acc += h;
        r = next_rec(__builtin_amdgcn_readfirstlane(h) + (uint32_t)s, lane, G, n);
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

/* B: transposed through LDS: instruction k, lane 4j+m loads quarter m of the record
   of lane 4j+k (one 64-B run per quad); lane 4j+k reads its record from region k. */
__global__ __launch_bounds__(kBlock, 5) void k_quad_lds(const uint4 *__restrict__ tab, uint32_t n, int steps, uint32_t G,
                                                       uint32_t *out)
{
    __shared__ uint4 stage[kBlock / 64][4][65]; /* per wave: 4 regions of 64 x 16 B (+16 B skew) */
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t wave_seed = mix(blockIdx.x * 4 + wave);
    uint32_t r = next_rec(wave_seed, lane, G, n);
    uint32_t acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int r0 = __builtin_amdgcn_update_dpp(0, (int)r, 0x00, 0xf, 0xf, false); /* quad_perm [0,0,0,0] */
        const int r1 = __builtin_amdgcn_update_dpp(0, (int)r, 0x55, 0xf, 0xf, false); /* [1,1,1,1] */
        const int r2 = __builtin_amdgcn_update_dpp(0, (int)r, 0xaa, 0xf, 0xf, false); /* [2,2,2,2] */
        const int r3 = __builtin_amdgcn_update_dpp(0, (int)r, 0xff, 0xf, 0xf, false); /* [3,3,3,3] */
        const uint32_t q = lane & 3;
        __builtin_amdgcn_global_load_lds((const void *)(tab + 4 * (size_t)(uint32_t)r0 + q), &stage[wave][0][0], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(tab + 4 * (size_t)(uint32_t)r1 + q), &stage[wave][1][0], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(tab + 4 * (size_t)(uint32_t)r2 + q), &stage[wave][2][0], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(tab + 4 * (size_t)(uint32_t)r3 + q), &stage[wave][3][0], 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint4 *mine = &stage[wave][q][lane & ~3u];
        const uint4 a = mine[0], b = mine[1], c = mine[2], d = mine[3];
        const uint32_t h = a.x ^ b.y ^ c.z ^ d.w;
        acc += h;
        r = next_rec(__builtin_amdgcn_readfirstlane(h) + (uint32_t)s, lane, G, n);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* reads done before the next DMA overwrites */
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

/* C: transposed in registers (DPP): instruction k as in B, then each lane gathers its
   quarters from its quad-mates with row-uniform DPP reads plus selects. */
__global__ __launch_bounds__(kBlock, 5) void k_quad_dpp(const uint4 *__restrict__ tab, uint32_t n, int steps, uint32_t G,
                                                       uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t wave_seed = mix(blockIdx.x * 4 + wave);
    uint32_t r = next_rec(wave_seed, lane, G, n);
    uint32_t acc = 0;
    const uint32_t q = lane & 3;
    for (int s = 0; s < steps; ++s) {
        uint4 v[4];
        v[0] = tab[4 * (size_t)dpp<0x00>(r) + q];
        v[1] = tab[4 * (size_t)dpp<0x55>(r) + q];
        v[2] = tab[4 * (size_t)dpp<0xaa>(r) + q];
        v[3] = tab[4 * (size_t)dpp<0xff>(r) + q];
        /* lane q needs quarter m of its record = v[q] of quad-mate m: per round, select
           the register by lane, rotate within the quad (cost model: 16 DPP + 48 selects) */
        const uint32_t h = round_m<0>(v, q) ^ round_m<1>(v, q) ^ round_m<2>(v, q) ^ round_m<3>(v, q);
        acc += h;
        r = next_rec(__builtin_amdgcn_readfirstlane(h) + (uint32_t)s, lane, G, n);
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

int main(int argc, char **argv)
{
    const double mb = argc > 1 ? atof(argv[1]) : 16.0;
    const int steps = argc > 2 ? atoi(argv[2]) : 2000;
    const uint32_t G = argc > 3 ? (uint32_t)atoi(argv[3]) : 64;
    const uint32_t n = (uint32_t)(mb * 1024 * 1024 / 64);
    std::vector<uint32_t> h((size_t)n * 16);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
    uint4 *tab;
    uint32_t *out;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 5;
    CHK(hipMalloc(&tab, h.size() * 4));
    CHK(hipMalloc(&out, (size_t)blocks * kBlock * 4));
    CHK(hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const char *names[3] = {"direct 4x dwordx4", "quad LDS-DMA", "quad DPP"};
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 3; ++v) {
            CHK(hipEventRecord(e0));
            if (v == 0) k_direct<<<blocks, kBlock>>>(tab, n, steps, G, out);
            if (v == 1) k_quad_lds<<<blocks, kBlock>>>(tab, n, steps, G, out);
            if (v == 2) k_quad_dpp<<<blocks, kBlock>>>(tab, n, steps, G, out);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const double recs = (double)blocks * kBlock * steps;
            if (rep == 1)
                printf("table %.0f MB G=%u %-20s %8.3f ms  %7.2f Grec/s  %6.2f TB/s (64 B/lane-step)\n", mb, G, names[v], ms,
                       recs / ms / 1e6, recs * 64 / ms / 1e9);
        }
    return 0;
}
