// sim_group_trav.cpp — CPU model of per-lane vs lane-group BVH traversal (design tool, not product).
//
// For box-path queries of the dragon-class scene (Lambert bounces from the box walls and shadow
// rays toward the light), counts the dependent rounds one query needs when
//   seq : one lane walks the 4-wide tree nearest-first, one record (node or triangle) per step
//         (the k_tris traversal), and
//   G   : a group of G lanes pops the top G items of a shared stack per round (nodes, or single
//         triangles: leaf children are expanded into triangle items when pushed),
// and the lane-slots (work) each spends.  Build:
//   g++ -O2 -std=c++17 -I include -I pathtracer.cl_amd/csrc scripts/sim_group_trav.cpp \
//       pathtracer.cl_amd/csrc/rt_bvh.cpp -L pathtracer.cl_amd -lrtmi -Wl,-rpath,$PWD/pathtracer.cl_amd -o /tmp/simg
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pathtracer_rt.h"
#include "rt_internal.h"

struct V {
    float x, y, z;
};
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct Scene {
    const float *n4;
    const float *tris;
};

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

struct Item {
    int code; /* >= 0 node; < 0: ~slot (single triangle) */
    float tn;
};

static float slack(float t) { return t * 1.0009765625f + 1e-4f; }

/* children of node n hit by the ray within [tmin_c, slack(best)] */
static int children(const Scene &s, int n, V o, V inv, float best, Item *out, int &n_tri_items, bool expand)
{
    const float *f = s.n4 + 32 * n;
    int k = 0;
    for (int i = 0; i < 4; ++i) {
        int c;
        memcpy(&c, &f[24 + i], 4);
        if (c == RT_EMPTY_CHILD) continue;
        float tx0 = (f[0 + i] - o.x) * inv.x, tx1 = (f[4 + i] - o.x) * inv.x;
        float ty0 = (f[8 + i] - o.y) * inv.y, ty1 = (f[12 + i] - o.y) * inv.y;
        float tz0 = (f[16 + i] - o.z) * inv.z, tz1 = (f[20 + i] - o.z) * inv.z;
        float tn = std::max(std::max(std::min(tx0, tx1), std::min(ty0, ty1)), std::max(std::min(tz0, tz1), -1e-3f));
        float tf = std::min(std::min(std::max(tx0, tx1), std::max(ty0, ty1)), std::min(std::max(tz0, tz1), slack(best)));
        if (!(tn <= tf)) continue;
        if (c >= 0 || !expand) {
            out[k++] = {c, tn};
        } else {
            int enc = ~c, first = enc >> 3, cnt = (enc & 7) + 1;
            for (int j = 0; j < cnt; ++j) out[k++] = {~(first + j), tn};
            n_tri_items += cnt;
        }
    }
    return k;
}

struct Res {
    long rounds, slots, items;
    int hit;
};

/* sequential per-lane traversal: nearest-first DFS, one record per step */
static Res seq(const Scene &s, V o, V d, float tmax, bool any)
{
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    std::vector<Item> st;
    st.push_back({0, 0.0f});
    float best = tmax;
    int hit = -1;
    long steps = 0;
    Item buf[64];
    while (!st.empty()) {
        Item it = st.back();
        st.pop_back();
        if (it.code >= 0) {
            ++steps;
            int dummy = 0;
            int k = children(s, it.code, o, inv, best, buf, dummy, false);
            std::sort(buf, buf + k, [](const Item &a, const Item &b) { return a.tn > b.tn; });
            for (int j = 0; j < k; ++j) st.push_back(buf[j]);
        } else {
            /* leaf code or triangle */
            int enc = ~it.code, first = enc >> 3, cnt = (enc & 7) + 1;
            for (int j = 0; j < cnt; ++j) {
                ++steps;
                float t;
                if (mt(s.tris + 12 * (first + j), o, d, t)) {
                    if (any) {
                        if (t > 1e-4f && t < tmax) return {steps, steps, steps, 1};
                    } else if (!(t < 1e-4f) && t < best) {
                        best = t;
                        hit = first + j;
                    }
                }
            }
        }
    }
    return {steps, steps, steps, hit};
}

/* lane group: G items per round from the top of a shared stack */
static Res group(const Scene &s, V o, V d, float tmax, bool any, int G, bool sorted_push, bool cull_pop)
{
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    std::vector<Item> st;
    st.push_back({0, 0.0f});
    float best = tmax;
    int hit = -1;
    long rounds = 0, items = 0;
    std::vector<Item> pushed;
    Item buf[64];
    while (!st.empty()) {
        ++rounds;
        std::vector<Item> pop;
        while (!st.empty() && (int)pop.size() < G) {
            Item it = st.back();
            st.pop_back();
            if (cull_pop && it.tn > slack(best)) continue;
            pop.push_back(it);
        }
        if (pop.empty()) break;
        items += pop.size();
        float nb = best;
        pushed.clear();
        bool done = false;
        for (int l = 0; l < (int)pop.size(); ++l) {
            Item it = pop[l];
            if (it.code >= 0) {
                int nt = 0;
                int k = children(s, it.code, o, inv, best, buf, nt, true);
                std::sort(buf, buf + k, [](const Item &a, const Item &b) { return a.tn > b.tn; });
                for (int j = 0; j < k; ++j) pushed.push_back(buf[j]);
            } else {
                float t;
                int slot = ~it.code;
                if (mt(s.tris + 12 * slot, o, d, t)) {
                    if (any) {
                        if (t > 1e-4f && t < tmax) done = true;
                    } else if (!(t < 1e-4f) && t < nb) {
                        nb = t;
                        hit = slot;
                    }
                }
            }
        }
        best = nb;
        if (done) return {rounds, rounds * G, items, 1};
        if (sorted_push)
            std::stable_sort(pushed.begin(), pushed.end(), [](const Item &a, const Item &b) { return a.tn > b.tn; });
        for (auto &p : pushed) st.push_back(p);
    }
    return {rounds, rounds * G, items, hit};
}


/* existence query, one lane, nearest-first DFS: steps until the first accepted triangle (or the end) */
static long seq_exist_from(const Scene &s, int root, V o, V d, bool &found)
{
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    std::vector<Item> st;
    st.push_back({root, 0.0f});
    long steps = 0;
    Item buf[64];
    found = false;
    while (!st.empty()) {
        Item it = st.back();
        st.pop_back();
        if (it.code >= 0) {
            ++steps;
            int dummy = 0;
            int k = children(s, it.code, o, inv, INFINITY, buf, dummy, false);
            std::sort(buf, buf + k, [](const Item &a, const Item &b) { return a.tn > b.tn; });
            for (int j = 0; j < k; ++j) st.push_back(buf[j]);
        } else {
            int enc = ~it.code, first = enc >> 3, cnt = (enc & 7) + 1;
            for (int j = 0; j < cnt; ++j) {
                ++steps;
                float t;
                if (mt(s.tris + 12 * (first + j), o, d, t) && !(t < 1e-4f)) {
                    found = true;
                    return steps;
                }
            }
        }
    }
    return steps;
}

/* a cut of the tree into at most F items (nodes or leaf codes), expanded breadth-first */
static std::vector<int> frontier(const Scene &s, int F)
{
    std::vector<int> cur{0};
    for (;;) {
        bool grew = false;
        std::vector<int> nxt;
        size_t i = 0;
        for (; i < cur.size(); ++i) {
            int c = cur[i];
            if (c < 0) { nxt.push_back(c); continue; }
            const float *f = s.n4 + 32 * c;
            std::vector<int> ch;
            for (int k = 0; k < 4; ++k) {
                int v;
                memcpy(&v, &f[24 + k], 4);
                if (v != RT_EMPTY_CHILD) ch.push_back(v);
            }
            size_t rest = cur.size() - i - 1;
            if (nxt.size() + ch.size() + rest <= (size_t)F) {
                for (int v : ch) nxt.push_back(v);
                grew = true;
            } else {
                nxt.push_back(c);
            }
        }
        cur = nxt;
        if (!grew) return cur;
    }
}

/* subtree-parallel existence: lane l walks subtree frontier[l] alone (after a box test of its
   root from registers); the query ends at the first round some lane accepts, else when all end */
static long subtree_exist(const Scene &s, const std::vector<int> &fr, V o, V d, bool &found)
{
    long best_hit = -1, longest = 0;
    for (int c : fr) {
        bool f = false;
        long n;
        if (c >= 0) n = seq_exist_from(s, c, o, d, f);
        else {
            /* a leaf item: its triangles one per step */
            int enc = ~c, first = enc >> 3, cnt = (enc & 7) + 1;
            n = 0;
            for (int j = 0; j < cnt && !f; ++j) {
                ++n;
                float t;
                if (mt(s.tris + 12 * (first + j), o, d, t) && !(t < 1e-4f)) f = true;
            }
        }
        if (f && (best_hit < 0 || n < best_hit)) best_hit = n;
        longest = std::max(longest, n);
    }
    found = best_hit >= 0;
    return found ? best_hit : longest;
}

int main(int argc, char **argv)
{
    uint32_t n_tris = argc > 1 ? (uint32_t)atoi(argv[1]) : 871414;
    int n_q = argc > 2 ? atoi(argv[2]) : 4000;
    std::vector<float> verts(3ull * rt_mesh_vertex_count(n_tris));
    std::vector<int32_t> idx(3ull * n_tris);
    rt_make_mesh(n_tris, 0.0f, -2.2f, 0.0f, 2.5f, verts.data(), idx.data());
    RtBvh bvh;
    std::string err;
    if (!rt_build_bvh(verts.data(), (uint32_t)(verts.size() / 3), idx.data(), n_tris, bvh, err)) {
        fprintf(stderr, "build: %s\n", err.c_str());
        return 1;
    }
    printf("nodes4 %u depth4 %u tree tris %u\n", bvh.n_nodes4, bvh.depth4, bvh.n_hit);
    Scene s{bvh.nodes4.data(), bvh.tris.data()};
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    const V light{0.0f, 4.0f, 2.0f};
    const int Gs[] = {4, 8, 16, 32};
    double seq_c = 0, seq_s = 0;
    double g_r[4][4] = {}, g_slots[4][4] = {}, g_items[4][4] = {};
    int hits_c = 0, n_c = 0, n_s = 0;
    const int Fs[] = {1, 4, 8, 16, 32, 64};
    std::vector<std::vector<int>> frs;
    for (int F : Fs) frs.push_back(frontier(s, F));
    double ex_steps[6] = {}, ex_hit_steps[6] = {};
    long ex_n = 0, ex_hits = 0;
    auto run_query = [&](V o, V d, float tmax, bool any, int &hit_out) {
        Res r0 = seq(s, o, d, tmax, any);
        hit_out = r0.hit;
        if (!any) {
            bool f0 = false;
            for (int fi = 0; fi < 6; ++fi) {
                bool f = false;
                long n = subtree_exist(s, frs[fi], o, d, f);
                if (fi == 0) f0 = f;
                else if (f != f0) fprintf(stderr, "existence mismatch F %d\n", Fs[fi]);
                ex_steps[fi] += n;
                if (f) ex_hit_steps[fi] += n;
            }
            ++ex_n;
            ex_hits += f0;
            seq_c += r0.rounds;
            ++n_c;
            hits_c += r0.hit >= 0;
        } else {
            seq_s += r0.rounds;
            ++n_s;
        }
        for (int gi = 0; gi < 4; ++gi)
            for (int v = 0; v < 4; ++v) {
                Res r = group(s, o, d, tmax, any, Gs[gi], v & 1, v & 2);
                if (!any && r.hit != r0.hit) fprintf(stderr, "mismatch G %d v %d: %d vs %d\n", Gs[gi], v, r.hit, r0.hit);
                g_r[gi][v] += r.rounds;
                g_slots[gi][v] += r.slots;
                g_items[gi][v] += r.items;
            }
    };
    for (int q = 0; q < n_q; ++q) {
        /* a box path starting on the floor beside the mesh (the box pixels the camera sees) */
        const float rlo = getenv("SIM_RLO") ? atof(getenv("SIM_RLO")) : 2.4f, rw = getenv("SIM_RW") ? atof(getenv("SIM_RW")) : 2.0f;
        if (getenv("SIM_PRIMARY")) { /* camera-like rays toward the mesh, then stop */
            V cam{3.0f, -0.8f, 2.0f};
            V tgt{(U(rng) * 2 - 1) * 2.5f, -2.2f + (U(rng) * 2 - 1) * 2.5f, (U(rng) * 2 - 1) * 2.5f};
            V d = sub(tgt, cam);
            float l = std::sqrt(dot(d, d));
            d = {d.x / l, d.y / l, d.z / l};
            int h;
            run_query(cam, d, INFINITY, false, h);
            continue;
        }
        float ang = 6.2831853f * U(rng), rad = rlo + rw * U(rng);
        V p{rad * std::cos(ang), -5.0f, rad * std::sin(ang)}, n{0, 1, 0};
        for (int depth = 0; depth < 7; ++depth) {
            V o{p.x + n.x * 1e-4f, p.y + n.y * 1e-4f, p.z + n.z * 1e-4f};
            /* shadow ray toward the light centre */
            V l = sub(light, o);
            float ll = std::sqrt(dot(l, l));
            V ld{l.x / ll, l.y / ll, l.z / ll};
            int h;
            if (dot(ld, n) > 0) run_query(o, ld, ll - 0.5f - 1e-4f, true, h);
            /* cosine-weighted bounce */
            float r1 = U(rng), r2 = U(rng);
            float ct = std::sqrt(1 - r1), stt = std::sqrt(1 - ct * ct), ph = 6.2831853f * r2;
            V t1 = std::fabs(n.y) > 0.9f ? V{1, 0, 0} : V{0, 1, 0};
            V a = cross(n, t1);
            float la = std::sqrt(dot(a, a));
            a = {a.x / la, a.y / la, a.z / la};
            V b = cross(n, a);
            V d{a.x * std::cos(ph) * stt + b.x * std::sin(ph) * stt + n.x * ct,
                a.y * std::cos(ph) * stt + b.y * std::sin(ph) * stt + n.y * ct,
                a.z * std::cos(ph) * stt + b.z * std::sin(ph) * stt + n.z * ct};
            V o2 = p; /* the bounce starts at the hit point (rtcommon.h:455) */
            run_query(o2, d, INFINITY, false, h);
            if (h >= 0) break; /* mesh hit: shadow ray then the path ends */
            /* box exit */
            float tb = INFINITY;
            const float hs[3] = {6, 5, 6};
            const float oc[3] = {o2.x, o2.y, o2.z}, dc[3] = {d.x, d.y, d.z};
            int ax = 0;
            for (int k = 0; k < 3; ++k) {
                if (dc[k] == 0) continue;
                float t = ((dc[k] > 0 ? hs[k] : -hs[k]) - oc[k]) / dc[k];
                if (t > 1e-4f && t < tb) tb = t, ax = k;
            }
            p = {o2.x + d.x * tb, o2.y + d.y * tb, o2.z + d.z * tb};
            n = {0, 0, 0};
            if (ax == 0) n.x = d.x > 0 ? -1.f : 1.f;
            if (ax == 1) n.y = d.y > 0 ? -1.f : 1.f;
            if (ax == 2) n.z = d.z > 0 ? -1.f : 1.f;
        }
    }
    int nq = n_c + n_s;
    printf("queries: %d closest (%.1f%% hit the mesh), %d shadow\n", n_c, 100.0 * hits_c / n_c, n_s);
    printf("seq: %.2f steps per closest, %.2f per shadow, %.2f mean\n", seq_c / n_c, seq_s / n_s, (seq_c + seq_s) / nq);
    printf("existence queries %ld (%.1f%% find a triangle)\n", ex_n, 100.0 * ex_hits / ex_n);
    for (int fi = 0; fi < 6; ++fi)
        printf("subtree lanes F=%2d (cut of %zu items): %.2f steps per query (hit queries %.2f, miss %.2f)\n", Fs[fi],
               frs[fi].size(), ex_steps[fi] / ex_n, ex_hit_steps[fi] / std::max(1L, ex_hits),
               (ex_steps[fi] - ex_hit_steps[fi]) / std::max(1L, ex_n - ex_hits));
    const char *vn[4] = {"lane-order push", "sorted push", "lane-order + pop cull", "sorted + pop cull"};
    for (int gi = 0; gi < 4; ++gi)
        for (int v = 0; v < 4; ++v)
            printf("G=%2d %-22s rounds %.2f  items %.2f  slots %.1f  (speedup %.2fx, lane util %.2f)\n", Gs[gi], vn[v],
                   g_r[gi][v] / nq, g_items[gi][v] / nq, g_slots[gi][v] / nq, (seq_c + seq_s) / g_r[gi][v],
                   g_items[gi][v] / g_slots[gi][v]);
    return 0;
}
