// sim_pixel_paths.cpp — CPU model of where a pixel's traversal steps go (design tool, not product).
//
// Traces the dragon-class frame's paths for chosen pixels (the real camera of plymain.cpp via
// rt_camera_spherical, box bounces and shadow rays toward the light, std::mt19937 numbers — a
// statistical stand-in for the kernel's MWC streams) through the host-built 4-wide tree with the
// kernel's one-record-per-step traversal order, and reports steps per closest-hit and per shadow
// query, split by the segment's origin (camera / box floor / box walls+ceiling).
//   g++ -O2 -std=c++17 -I include -I pathtracer.cl_amd/csrc scripts/sim_pixel_paths.cpp \
//       pathtracer.cl_amd/csrc/rt_bvh.cpp -L pathtracer.cl_amd -lrtmi -Wl,-rpath,$PWD/pathtracer.cl_amd -o /tmp/simp
//   /tmp/simp X Y [samples]        (pixel of the 1920x1080 frame)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pathtracer_rt.h"
#include "rt_internal.h"
#include "rt_quant.h"

struct V {
    float x, y, z;
};
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V mul(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V norm(V a) { return mul(a, 1.0f / std::sqrt(dot(a, a))); }

static const float *g_n4, *g_tris;
static const uint32_t *g_q4; /* compressed nodes: the kernel's own cull (mode 7) */
static long g_node_steps, g_tri_steps; /* of all queries */
static long g_near[2], g_far[2];         /* shadow-query steps entered within / beyond t = 0.05 (node, tri) */
static bool g_track;
static bool g_from_mesh; /* the shadow query leaves a mesh hit */
static bool g_backface; /* ... a back face (the closest-hit ray met the triangle from behind) */
static float g_tmin_shadow = -1e-3f; /* experiment: node-cull tmin of shadow rays leaving the mesh */
static double g_occ[2], g_occ_steps[2]; /* camera-hit shadow queries: unoccluded / occluded, and their steps */
static int g_order = 0; /* 0 sorted push, 1 nearest first only, 2 sorted with any-hit origin boxes last, 3 and those by segment length, 5 = 3 for shadow rays leaving the mesh else 2 (k_tris) */
/* per 4-wide node: box of the unnormalised normals e2 x e1 of its subtree's triangles (det cull) */
static std::vector<float> g_nbox; /* 6 floats per node: lo xyz, hi xyz */
static int g_det_cull = 0; /* 1 per child at the parent, 2 per leaf in its first record, 3 inner children only */
static void leaf_nbox(int code, float *b)
{
    int enc = ~code, first = enc >> 3, cnt = (enc & 7) + 1;
    for (int k = 0; k < 3; ++k) b[k] = 1e30f, b[3 + k] = -1e30f;
    for (int j = 0; j < cnt; ++j) {
        const float *tr = g_tris + 12 * (first + j);
        V n = cross(V{tr[8], tr[9], tr[10]}, V{tr[4], tr[5], tr[6]});
        const float c[3] = {n.x, n.y, n.z};
        for (int k = 0; k < 3; ++k) b[k] = std::min(b[k], c[k]), b[3 + k] = std::max(b[3 + k], c[k]);
    }
}
static void build_nbox(int node)
{
    float *b = &g_nbox[6 * node];
    for (int k = 0; k < 3; ++k) b[k] = 1e30f, b[3 + k] = -1e30f;
    const float *f = g_n4 + 32 * node;
    for (int i = 0; i < 4; ++i) {
        int c;
        memcpy(&c, &f[24 + i], 4);
        if (c == RT_EMPTY_CHILD) continue;
        float cb[6];
        if (c >= 0) {
            build_nbox(c);
            memcpy(cb, &g_nbox[6 * c], sizeof(cb));
        } else leaf_nbox(c, cb);
        for (int k = 0; k < 3; ++k) b[k] = std::min(b[k], cb[k]), b[3 + k] = std::max(b[3 + k], cb[3 + k]);
    }
}
/* can any triangle under the normal box pass |det| >= 1e-4 for direction d? (2 % slack) */
static bool det_possible(const float *b, V d)
{
    const float dd[3] = {d.x, d.y, d.z};
    float fmax = 0, fmin = 0;
    for (int k = 0; k < 3; ++k) {
        const float p = dd[k] * b[k], q = dd[k] * b[3 + k];
        fmax += std::max(p, q);
        fmin += std::min(p, q);
    }
    return std::max(fmax, -fmin) * 1.02f >= 1e-4f;
}

static bool mt(const float *tr, V o, V d, float &t)
{
    V v0{tr[0], tr[1], tr[2]}, e1{tr[4], tr[5], tr[6]}, e2{tr[8], tr[9], tr[10]};
    V p = cross(d, e2);
    float det = dot(p, e1);
    if (std::fabs(det) < 1e-4f) return false;
    float inv = 1.0f / det;
    V to = sub(o, v0);
    V q = cross(to, e1);
    float u = dot(p, to) * inv, v = dot(q, d) * inv;
    t = dot(q, e2) * inv;
    return !(u < 0 || u > 1) && !(v < 0 || v + u > 1);
}

/* nearest-first DFS, one record (node or triangle) per step: k_tris's step count */
static const float *g_bin; /* the host's binary tree (16 floats per node) */
static int g_wide = 0;      /* > 0: traverse an n-wide collapse of it (query_wide) */
static long query_wide(V o, V d, float tmax, bool any, float &t_hit, int &hit);
static long query(V o, V d, float tmax, bool any, float &t_hit, int &hit)
{
    if (g_wide) return query_wide(o, d, tmax, any, t_hit, hit);
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    struct It {
        int c;
        float tn;
    };
    std::vector<It> st{{0, 0.0f}};
    float best = tmax;
    hit = -1;
    long steps = 0;
    while (!st.empty()) {
        It it = st.back();
        st.pop_back();
        if (g_track) (it.tn < 0.05f ? g_near : g_far)[it.c >= 0 ? 0 : 1] += it.c >= 0 ? 1 : ((~it.c) & 7) + 1;
        if (it.c >= 0) {
            ++steps;
            ++g_node_steps;
            if ((g_det_cull == 4 || g_det_cull == 5) && !det_possible(&g_nbox[6 * it.c], d)) continue; /* own box */
            if (g_det_cull == 7) { /* the kernel's formula on the encoded box (rt_kernels.hip trav_step_q) */
                const uint32_t *q = g_q4 + 16ull * it.c;
                auto sx = [](uint32_t w, int off) { return (int)((w >> off) & 0xff) - 128; };
                const float nsc = std::ldexp(1.0f, (int)(q[10] >> 24) - 128);
                const bool px = d.x >= 0, py = d.y >= 0, pz = d.z >= 0;
                const float fhi = std::fma(d.x, (float)(px ? sx(q[11], 0) : sx(q[10], 0)),
                                           std::fma(d.y, (float)(py ? sx(q[11], 8) : sx(q[10], 8)),
                                                    d.z * (float)(pz ? sx(q[11], 16) : sx(q[10], 16))));
                const float flo = std::fma(d.x, (float)(px ? sx(q[10], 0) : sx(q[11], 0)),
                                           std::fma(d.y, (float)(py ? sx(q[10], 8) : sx(q[11], 8)),
                                                    d.z * (float)(pz ? sx(q[10], 16) : sx(q[11], 16))));
                const float l1 = std::fabs(d.x) + std::fabs(d.y) + std::fabs(d.z);
                if (std::fma(std::max(fhi, -flo) * nsc, 1.02f, 5e-7f * l1) < 1e-4f) continue;
            }
            if (g_det_cull == 6) { /* own box as centre + one radius: |d.c| + r |d|_1 */
                const float *b = &g_nbox[6 * it.c];
                float c[3], r = 0;
                for (int k = 0; k < 3; ++k) c[k] = 0.5f * (b[k] + b[3 + k]), r = std::max(r, 0.5f * (b[3 + k] - b[k]));
                const float bound = std::fabs(d.x * c[0] + d.y * c[1] + d.z * c[2]) +
                                    r * (std::fabs(d.x) + std::fabs(d.y) + std::fabs(d.z));
                if (bound * 1.02f < 1e-4f) continue;
            }
            const float *f = g_n4 + 32 * it.c;
            It buf[4];
            float bt[4];
            int k = 0;
            for (int i = 0; i < 4; ++i) {
                int c;
                memcpy(&c, &f[24 + i], 4);
                if (c == RT_EMPTY_CHILD) continue;
                float tx0 = (f[0 + i] - o.x) * inv.x, tx1 = (f[4 + i] - o.x) * inv.x;
                float ty0 = (f[8 + i] - o.y) * inv.y, ty1 = (f[12 + i] - o.y) * inv.y;
                float tz0 = (f[16 + i] - o.z) * inv.z, tz1 = (f[20 + i] - o.z) * inv.z;
                float tn = std::max(std::max(std::min(tx0, tx1), std::min(ty0, ty1)),
                                    std::max(std::min(tz0, tz1), any && g_from_mesh ? g_tmin_shadow : -1e-3f));
                float tf = std::min(std::min(std::max(tx0, tx1), std::max(ty0, ty1)),
                                    std::min(std::max(tz0, tz1), best * 1.0009765625f + 1e-4f));
                if (!(tn <= tf)) continue;
                if (g_det_cull == 1 || (g_det_cull == 3 && c >= 0)) { /* at the parent: per child */
                    float cb[6];
                    if (c >= 0) memcpy(cb, &g_nbox[6 * c], sizeof(cb));
                    else leaf_nbox(c, cb);
                    if (!det_possible(cb, d)) continue;
                }
                bt[k] = tf;
                buf[k++] = {c, tn};
            }
            if (g_order >= 2 && any) { /* any-hit: children holding the origin visited last */
                It key[4];
                for (int j = 0; j < k; ++j) {
                    const bool longest = g_order == 3 || (g_order == 5 && g_from_mesh) ||
                                         (g_order == 8 && g_from_mesh && !g_backface);
                    float kk = longest ? -(bt[j] - buf[j].tn) : g_order == 4 ? -buf[j].tn : buf[j].tn;
                    /* 6: far exit first, 7: far entry first (shadow rays leaving the mesh); 8: far exit
                       first for those leaving a back face (the origin inside the closed surface) */
                    if (g_from_mesh && (g_order == 6 || (g_order == 8 && g_backface))) kk = -bt[j];
                    if (g_from_mesh && g_order == 7) kk = -buf[j].tn;
                    bool origin_last = buf[j].tn <= -1e-3f;
                    /* 9: nearest entry first for rays leaving the mesh, origin boxes not postponed;
                       10: nearest exit first for them */
                    if (g_from_mesh && g_order == 9) kk = buf[j].tn, origin_last = false;
                    if (g_from_mesh && g_order == 10) kk = bt[j], origin_last = false;
                    key[j] = {buf[j].c, origin_last ? kk + 1e4f : kk};
                }
                std::sort(key, key + k, [](const It &a, const It &b) { return a.tn > b.tn; });
                for (int j = 0; j < k; ++j) buf[j] = {key[j].c, 0.0f};
            } else if (g_order != 1) {
                std::sort(buf, buf + k, [](const It &a, const It &b) { return a.tn > b.tn; });
            } else if (k > 1) { /* nearest visited first, the others pushed in slot order */
                int m = 0;
                for (int j = 1; j < k; ++j)
                    if (buf[j].tn < buf[m].tn) m = j;
                std::swap(buf[m], buf[k - 1]);
            }
            for (int j = 0; j < k; ++j) st.push_back(buf[j]);
        } else {
            int enc = ~it.c, first = enc >> 3, cnt = (enc & 7) + 1;
            if (g_det_cull == 2 || g_det_cull == 5) { /* the leaf's normal box rides in its first triangle record */
                float cb[6];
                leaf_nbox(it.c, cb);
                if (!det_possible(cb, d)) cnt = 1;
            }
            for (int j = 0; j < cnt; ++j) {
                ++steps;
                ++g_tri_steps;
                float t;
                if (mt(g_tris + 12 * (first + j), o, d, t)) {
                    if (any) {
                        if (t > 1e-4f && t < tmax) {
                            hit = first + j;
                            t_hit = t;
                            return steps;
                        }
                    } else if (!(t < 1e-4f) && t < best) {
                        best = t;
                        hit = first + j;
                    }
                }
            }
        }
    }
    t_hit = best;
    return steps;
}

/* An n-wide tree collapsed on the fly from the host's binary tree (largest-area inner child
   expanded first, as rt_bvh.cpp collapses to 4-wide), one step per wide node and per triangle:
   how many steps an 8-wide layout would save (g_wide = 4 / 8; no determinant cull). */
static long query_wide(V o, V d, float tmax, bool any, float &t_hit, int &hit)
{
    struct E {
        float lo[3], hi[3];
        int code;
    };
    auto child = [](int node, int side) {
        const float *n = g_bin + 16 * node;
        E e;
        const int b = side ? 4 : 0;
        e.lo[0] = n[b + 0]; e.hi[0] = n[b + 1]; e.lo[1] = n[b + 2]; e.hi[1] = n[b + 3];
        e.lo[2] = n[8 + 2 * side]; e.hi[2] = n[9 + 2 * side];
        memcpy(&e.code, &n[12 + side], 4);
        return e;
    };
    auto area = [](const E &e) {
        const float x = e.hi[0] - e.lo[0], y = e.hi[1] - e.lo[1], z = e.hi[2] - e.lo[2];
        return x * y + y * z + z * x;
    };
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    struct It {
        int c; /* binary node whose children form a wide node (>= 0) or a leaf code (< 0) */
        float key;
    };
    std::vector<It> st{{0, 0.0f}};
    float best = tmax;
    hit = -1;
    long steps = 0;
    while (!st.empty()) {
        It it = st.back();
        st.pop_back();
        if (it.c >= 0) {
            ++steps;
            ++g_node_steps;
            std::vector<E> k{child(it.c, 0), child(it.c, 1)};
            while ((int)k.size() < g_wide) {
                int bi = -1;
                float ba = -1.0f;
                for (int i = 0; i < (int)k.size(); ++i)
                    if (k[i].code >= 0 && area(k[i]) > ba) ba = area(k[i]), bi = i;
                if (bi < 0) break;
                const int e = k[bi].code;
                k[bi] = child(e, 0);
                k.push_back(child(e, 1));
            }
            std::vector<It> buf;
            for (const E &e : k) {
                float tx0 = (e.lo[0] - o.x) * inv.x, tx1 = (e.hi[0] - o.x) * inv.x;
                float ty0 = (e.lo[1] - o.y) * inv.y, ty1 = (e.hi[1] - o.y) * inv.y;
                float tz0 = (e.lo[2] - o.z) * inv.z, tz1 = (e.hi[2] - o.z) * inv.z;
                float tn = std::max(std::max(std::min(tx0, tx1), std::min(ty0, ty1)), std::max(std::min(tz0, tz1), -1e-3f));
                float tf = std::min(std::min(std::max(tx0, tx1), std::max(ty0, ty1)),
                                    std::min(std::max(tz0, tz1), best * 1.0009765625f + 1e-4f));
                if (!(tn <= tf)) continue;
                float key = tn;
                if (any && g_order >= 2) key = (g_order == 3 || (g_order == 5 && g_from_mesh) ? tn - tf : tn) + (tn <= 0.0f ? 1e4f : 0.0f);
                buf.push_back({e.code, key});
            }
            std::sort(buf.begin(), buf.end(), [](const It &a, const It &b) { return a.key > b.key; });
            for (const It &b : buf) st.push_back(b);
        } else {
            int enc = ~it.c, first = enc >> 3, cnt = (enc & 7) + 1;
            for (int j = 0; j < cnt; ++j) {
                ++steps;
                ++g_tri_steps;
                float t;
                if (mt(g_tris + 12 * (first + j), o, d, t)) {
                    if (any) {
                        if (t > 1e-4f && t < tmax) {
                            hit = first + j;
                            return steps;
                        }
                    } else if (!(t < 1e-4f) && t < best) {
                        best = t;
                        hit = first + j;
                    }
                }
            }
        }
    }
    t_hit = best;
    return steps;
}

static float box_hit(V o, V d, V &n)
{
    const float s[3] = {6.0f, 5.0f, 6.0f};
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    float best = 1e30f;
    int ax = 0;
    for (int a = 0; a < 3; ++a) {
        if (dd[a] == 0) continue;
        float t = ((dd[a] > 0 ? s[a] : -s[a]) - oo[a]) / dd[a];
        if (t > 1e-4f && t < best) {
            best = t;
            ax = a;
        }
    }
    n = {0, 0, 0};
    (&n.x)[ax] = dd[ax] > 0 ? -1.0f : 1.0f;
    return best;
}

static V frame_dir(V n, float r1, float r2) /* cosine-weighted about n */
{
    float ct = std::sqrt(1 - r1), st = std::sqrt(1 - ct * ct), ph = 6.2831853f * r2;
    V a = std::fabs(n.x) > 0.5f ? V{0, 1, 0} : V{1, 0, 0};
    V t = norm(cross(a, n)), b = cross(n, t);
    return norm(add(add(mul(t, std::cos(ph) * st), mul(b, std::sin(ph) * st)), mul(n, ct)));
}

int main(int argc, char **argv)
{
    const uint32_t W = 1920, H = 1080, n_tris = 871414;
    const int px = argc > 1 ? atoi(argv[1]) : 1807, py = argc > 2 ? atoi(argv[2]) : 633;
    const int spp = argc > 3 ? atoi(argv[3]) : 256;
    std::vector<float> verts(3ull * rt_mesh_vertex_count(n_tris));
    std::vector<int32_t> idx(3ull * n_tris);
    rt_make_mesh(n_tris, 0.0f, -2.2f, 0.0f, 2.5f, verts.data(), idx.data());
    RtBvh bvh;
    std::string err;
    if (!rt_build_bvh(verts.data(), (uint32_t)(verts.size() / 3), idx.data(), n_tris, bvh, err)) return 1;
    g_n4 = bvh.nodes4.data();
    g_tris = bvh.tris.data();
    g_q4 = bvh.nodes4q.data();
    g_nbox.resize(6ull * bvh.n_nodes4);
    build_nbox(0);
    g_det_cull = argc > 4 ? atoi(argv[4]) : 0;
    g_order = argc > 5 ? atoi(argv[5]) : 0;
    if (argc > 6) g_tmin_shadow = (float)atof(argv[6]);
    if (argc > 7) g_wide = atoi(argv[7]);
    g_bin = bvh.nodes.data();
    float cam[16];
    rt_camera_spherical(0, -4, 0, 40, 105, 5, 53, W, reinterpret_cast<rt_camera *>(cam));
    const V view{cam[0], cam[1], cam[2]}, up{cam[4], cam[5], cam[6]}, right{cam[8], cam[9], cam[10]},
        pos{cam[12], cam[13], cam[14]};
    const V light{0, 4, 2};
    std::mt19937 rng(11);
    std::uniform_real_distribution<float> U(0, 1);
    const char *names[3] = {"camera", "floor", "walls/ceiling"};
    double st_c[3] = {}, n_c[3] = {}, st_s[3] = {}, n_s[3] = {}, mesh_hits[3] = {};
    long total = 0;
    for (int s = 0; s < spp; ++s) {
        V d = norm(add(add(view, mul(right, px + U(rng) - W / 2.0f)), mul(up, py + U(rng) - H / 2.0f)));
        V o = pos;
        int src = 0;
        for (int depth = 0; depth <= 6; ++depth) {
            float t;
            int hit;
            long k = query(o, d, 1e30f, false, t, hit);
            if (g_det_cull) {
                const int m = g_det_cull;
                g_det_cull = 0;
                float t0;
                int h0;
                query(o, d, 1e30f, false, t0, h0);
                g_det_cull = m;
                if (h0 != hit || (hit >= 0 && t0 != t)) printf("MISMATCH closest: %d vs %d\n", hit, h0);
            }
            st_c[src] += k;
            n_c[src] += 1;
            total += k;
            V n, p;
            if (hit >= 0) {
                mesh_hits[src] += 1;
                p = add(o, mul(d, t));
                const float *tr = g_tris + 12 * hit;
                n = norm(cross(V{tr[8], tr[9], tr[10]}, V{tr[4], tr[5], tr[6]}));
            } else {
                float tb = box_hit(o, d, n);
                p = add(o, mul(d, tb));
            }
            V so = add(p, mul(n, 1e-4f));
            V ld = norm(sub(add(light, V{U(rng) * 0.5f - 0.25f, U(rng) * 0.5f - 0.25f, 0}), so));
            if (dot(ld, n) > 0) {
                float tl = std::sqrt(dot(sub(light, so), sub(light, so))) - 0.5f;
                int h2;
                float t2;
                g_track = src == 0;
                g_from_mesh = hit >= 0;
                long k2 = query(so, ld, tl, true, t2, h2);
                g_track = false;
                st_s[src] += k2;
                n_s[src] += 1;
                if (src == 0) {
                    g_occ[h2 >= 0] += 1;
                    g_occ_steps[h2 >= 0] += k2;
                }
                total += k2;
            }
            if (hit >= 0) break;
            o = p;
            d = frame_dir(n, U(rng), U(rng));
            src = n.y > 0.5f ? 1 : 2;
        }
    }
    printf("pixel (%d, %d), %d samples: %ld steps (%ld node, %ld triangle)\n", px, py, spp, total, g_node_steps,
           g_tri_steps);
    for (int i = 0; i < 3; ++i)
        printf("  from %-14s closest %6.0f x %5.1f steps (%4.1f%% hit mesh)   shadow %6.0f x %5.1f steps\n", names[i],
               n_c[i], n_c[i] ? st_c[i] / n_c[i] : 0, n_c[i] ? 100 * mesh_hits[i] / n_c[i] : 0, n_s[i],
               n_s[i] ? st_s[i] / n_s[i] : 0);
    printf("camera-hit shadow queries: near (t < 0.05) %ld node + %ld tri steps, far %ld node + %ld tri\n", g_near[0],
           g_near[1], g_far[0], g_far[1]);
    printf("camera-hit shadow queries: %.0f unoccluded x %.1f steps, %.0f occluded x %.1f steps\n", g_occ[0],
           g_occ[0] ? g_occ_steps[0] / g_occ[0] : 0, g_occ[1], g_occ[1] ? g_occ_steps[1] / g_occ[1] : 0);
    return 0;
}
