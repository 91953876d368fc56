// sim_frame_mix.cpp — CPU model of the dragon-class frame's query mix (design tool, not product).
//
// Samples pixels uniformly over the 1920x1080 frame (the real camera of plymain.cpp), traces their
// paths with sim_pixel_paths.cpp's model (the kernel's traversal: one record per step, determinant
// cull, any-hit child order; std::mt19937 numbers as a statistical stand-in for the MWC streams)
// and reports, per query kind, the queries and traversal steps: camera rays (which k_tris answers
// through candidate lists), bounce rays from the box, shadow rays leaving the mesh and shadow rays
// leaving the box.  For the shadow rays leaving the mesh it also estimates what a per-triangle
// light-visibility certificate could answer without a traversal: a triangle counts as "clear" when
// K probe rays from random points of it to random points of the light sphere are all unoccluded.
//   g++ -O2 -std=c++17 -I include -I pathtracer.cl_amd/csrc scripts/sim_frame_mix.cpp \
//       pathtracer.cl_amd/csrc/rt_bvh.cpp -L pathtracer.cl_amd -lrtmi -Wl,-rpath,$PWD/pathtracer.cl_amd -o /tmp/simf
//   /tmp/simf [pixels] [samples] [probes]
#define main pixel_paths_main
#include "sim_pixel_paths.cpp"
#undef main

#include <unordered_map>

int main(int argc, char **argv)
{
    const uint32_t W = 1920, H = 1080, n_tris = 871414;
    const int n_px = argc > 1 ? atoi(argv[1]) : 3000, spp = argc > 2 ? atoi(argv[2]) : 8;
    const int probes = argc > 3 ? atoi(argv[3]) : 32;
    std::vector<float> verts(3ull * rt_mesh_vertex_count(n_tris));
    std::vector<int32_t> idx(3ull * n_tris);
    rt_make_mesh(n_tris, 0.0f, -2.2f, 0.0f, 2.5f, verts.data(), idx.data());
    RtBvh bvh;
    std::string err;
    if (!rt_build_bvh(verts.data(), (uint32_t)(verts.size() / 3), idx.data(), n_tris, bvh, err)) return 1;
    g_n4 = bvh.nodes4.data();
    g_tris = bvh.tris.data();
    g_q4 = bvh.nodes4q.data();
    g_bin = bvh.nodes.data();
    g_det_cull = 7;
    g_order = argc > 4 ? atoi(argv[4]) : 5;
    /* per triangle slot: the depth of the node holding its leaf (root 0) and its place in the leaf:
       the fewest steps any order can take to reach it (node steps root..parent + triangle steps) */
    std::vector<int> slot_min_steps(bvh.tris.size() / 12, -1);
    {
        std::vector<std::pair<int, int>> q{{0, 0}};
        while (!q.empty()) {
            auto [nd, dep] = q.back();
            q.pop_back();
            const float *f = g_n4 + 32 * nd;
            for (int i = 0; i < 4; ++i) {
                int c;
                memcpy(&c, &f[24 + i], 4);
                if (c == RT_EMPTY_CHILD) continue;
                if (c >= 0) q.push_back({c, dep + 1});
                else {
                    const int enc = ~c, first = enc >> 3, cnt = (enc & 7) + 1;
                    for (int j = 0; j < cnt; ++j) slot_min_steps[first + j] = dep + 1 + j + 1;
                }
            }
        }
    }
    double n_boxs = 0, n_boxs_only = 0;
    double n_back = 0, n_meshhit = 0, occ_t_hist[5] = {}, occ_t_steps[5] = {};
    int dbg_n = 0;
    double occ_steps = 0, occ_lb = 0, occ_n = 0, unocc_steps = 0, unocc_n = 0;
    float cam[16];
    rt_camera_spherical(0, -4, 0, 40, 105, 5, 53, W, reinterpret_cast<rt_camera *>(cam));
    const V view{cam[0], cam[1], cam[2]}, up{cam[4], cam[5], cam[6]}, right{cam[8], cam[9], cam[10]},
        pos{cam[12], cam[13], cam[14]};
    const V light{0, 4, 2};
    const float lr = 0.5f;
    std::mt19937 rng(11);
    std::uniform_real_distribution<float> U(0, 1);
    enum { CAM, BOUNCE, SH_MESH, SH_BOX, NK };
    const char *names[NK] = {"camera (closest)", "box bounce (closest)", "shadow from mesh", "shadow from box"};
    double nq[NK] = {}, ns[NK] = {}, nocc[NK] = {}, nskip[NK] = {};
    double clear_q = 0, clear_s = 0, clear_occ = 0;
    std::unordered_map<int, bool> clear_cache;
    auto sphere_point = [&](void) {
        for (;;) {
            V p{U(rng) * 2 - 1, U(rng) * 2 - 1, U(rng) * 2 - 1};
            if (dot(p, p) <= 1.0f) return add(light, mul(p, lr));
        }
    };
    auto tri_clear = [&](int slot) {
        auto it = clear_cache.find(slot);
        if (it != clear_cache.end()) return it->second;
        const float *tr = g_tris + 12 * slot;
        const V v0{tr[0], tr[1], tr[2]}, e1{tr[4], tr[5], tr[6]}, e2{tr[8], tr[9], tr[10]};
        const V nn = cross(e2, e1);
        bool ok = true;
        const int saved = g_det_cull;
        for (int k = 0; k < probes && ok; ++k) {
            float a = U(rng), b = U(rng);
            if (a + b > 1) a = 1 - a, b = 1 - b;
            const V p = add(add(add(v0, mul(e1, a)), mul(e2, b)), mul(nn, 1e-4f));
            const V q = sphere_point();
            const V d = norm(sub(q, p));
            if (dot(d, nn) <= 0) continue; /* answered without a traversal anyway */
            float t;
            int h;
            g_from_mesh = true;
            query(p, d, std::sqrt(dot(sub(q, p), sub(q, p))), true, t, h);
            ok = h < 0;
        }
        g_det_cull = saved;
        clear_cache[slot] = ok;
        return ok;
    };
    for (int i = 0; i < n_px; ++i) {
        const int px = (int)(U(rng) * W), py = (int)(U(rng) * H);
        for (int s = 0; s < spp; ++s) {
            V d = norm(add(add(view, mul(right, px + U(rng) - W / 2.0f)), mul(up, py + U(rng) - H / 2.0f)));
            V o = pos;
            bool box_sample = false, mesh_later = false;
            for (int depth = 0; depth <= 6; ++depth) {
                float t;
                int hit;
                const int kc = depth == 0 ? CAM : BOUNCE;
                long k = query(o, d, 1e30f, false, t, hit);
                nq[kc] += 1;
                ns[kc] += k;
                V n, p;
                if (hit >= 0) {
                    p = add(o, mul(d, t));
                    n_back += dot(d, norm(cross(V{g_tris[12 * hit + 8], g_tris[12 * hit + 9], g_tris[12 * hit + 10]},
                                                V{g_tris[12 * hit + 4], g_tris[12 * hit + 5], g_tris[12 * hit + 6]}))) > 0;
                    n_meshhit += 1;
                    const float *tr = g_tris + 12 * hit;
                    n = norm(cross(V{tr[8], tr[9], tr[10]}, V{tr[4], tr[5], tr[6]}));
                } else {
                    float tb = box_hit(o, d, n);
                    p = add(o, mul(d, tb));
                }
                const int ks = hit >= 0 ? SH_MESH : SH_BOX;
                V so = add(p, mul(n, 1e-4f));
                V lp = sphere_point();
                V ld = norm(sub(lp, so));
                if (dot(ld, n) > 0) {
                    float tl = std::sqrt(dot(sub(light, so), sub(light, so))) - lr;
                    int h2;
                    float t2;
                    g_from_mesh = hit >= 0;
                    g_backface = hit >= 0 && dot(d, n) > 0;
                    long k2 = query(so, ld, tl, true, t2, h2);
                    nq[ks] += 1;
                    ns[ks] += k2;
                    nocc[ks] += h2 >= 0;
                    if (getenv("SIM_DEBUG") && hit >= 0 && dbg_n < 12) {
                        ++dbg_n;
                        printf("origin (%.3f %.3f %.3f) |p-c| %.3f  n (%.2f %.2f %.2f)  ld (%.2f %.2f %.2f)  cos %.3f  occ %d t %.4f "
                               "tmax %.3f\n", so.x, so.y, so.z, std::sqrt(dot(sub(p, V{0, -2.2f, 0}), sub(p, V{0, -2.2f, 0}))),
                               n.x, n.y, n.z, ld.x, ld.y, ld.z, dot(ld, n), h2 >= 0, t2, tl);
                    }
                    if (hit >= 0) {
                        if (h2 >= 0) {
                            occ_steps += k2, occ_lb += slot_min_steps[h2], occ_n += 1;
                            const int b = t2 < 0.01f ? 0 : t2 < 0.1f ? 1 : t2 < 0.5f ? 2 : t2 < 1.5f ? 3 : 4;
                            occ_t_hist[b] += 1;
                            occ_t_steps[b] += k2;
                        }
                        else unocc_steps += k2, unocc_n += 1;
                    }
                    if (hit >= 0 && tri_clear(hit)) {
                        clear_q += 1;
                        clear_s += k2;
                        clear_occ += h2 >= 0;
                    }
                } else {
                    nskip[ks] += 1;
                }
                if (depth == 0 && hit < 0) box_sample = true;
                if (depth > 0 && hit >= 0) mesh_later = true;
                if (hit >= 0) break;
                o = p;
                d = frame_dir(n, U(rng), U(rng));
            }
            if (box_sample) {
                n_boxs += 1;
                n_boxs_only += !mesh_later;
            }
        }
    }
    printf("box samples (camera ray misses the mesh): %.0f, box-only paths (no bounce hits the mesh): %.1f%%\n", n_boxs,
           100 * n_boxs_only / std::max(1.0, n_boxs));
    double tot = 0;
    for (int k = 0; k < NK; ++k) tot += ns[k];
    printf("%d pixels x %d samples: %.0f traversal steps\n", n_px, spp, tot);
    for (int k = 0; k < NK; ++k)
        printf("  %-22s %9.0f traversed queries x %5.2f steps = %5.1f%% of steps (%4.1f%% occluded), %8.0f answered "
               "without traversal\n",
               names[k], nq[k], nq[k] ? ns[k] / nq[k] : 0, 100 * ns[k] / tot, nq[k] ? 100 * nocc[k] / nq[k] : 0,
               nskip[k]);
    printf("occluder distance t: <0.01 %.0f (%.1f steps), <0.1 %.0f (%.1f), <0.5 %.0f (%.1f), <1.5 %.0f (%.1f), more %.0f (%.1f)\n",
           occ_t_hist[0], occ_t_steps[0] / std::max(1.0, occ_t_hist[0]), occ_t_hist[1], occ_t_steps[1] / std::max(1.0, occ_t_hist[1]),
           occ_t_hist[2], occ_t_steps[2] / std::max(1.0, occ_t_hist[2]), occ_t_hist[3], occ_t_steps[3] / std::max(1.0, occ_t_hist[3]),
           occ_t_hist[4], occ_t_steps[4] / std::max(1.0, occ_t_hist[4]));
    printf("mesh hits: %.0f, %.1f%% on back faces\n", n_meshhit, 100 * n_back / std::max(1.0, n_meshhit));
    printf("shadow from mesh: occluded %.0f x %.2f steps (the found occluder's depth + place: %.2f), unoccluded %.0f x "
           "%.2f steps\n", occ_n, occ_n ? occ_steps / occ_n : 0, occ_n ? occ_lb / occ_n : 0, unocc_n,
           unocc_n ? unocc_steps / unocc_n : 0);
    printf("shadow from mesh on 'clear' triangles (%d probes): %.0f queries (%.1f%%), %.0f steps = %.1f%% of all "
           "steps; %.0f of them occluded (the estimate's misses)\n",
           probes, clear_q, nq[SH_MESH] ? 100 * clear_q / nq[SH_MESH] : 0, clear_s, 100 * clear_s / tot, clear_occ);
    return 0;
}
