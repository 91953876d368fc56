/*
 * rt_render — headless C++ host over RayTracerHIP.hpp: the reference's
 * clrt/main.cpp (sphere scene) and clrt/plymain.cpp (+ a triangle mesh) without
 * the GLUT window.  Frames are driven like GlutCLWindow (progression 0, 1, 2, ...;
 * GlutCLWindow.cpp:144-158) and the last frame is written as raw RGBA32F
 * (W*H*4 little-endian floats) and/or a PFM.
 *
 *   rt_render [--scene main|ply] [--width W] [--height H] [--frames F]
 *             [--sample-rate S] [--depth D] [--mesh N_TRIS | --ply FILE] [--linear]
 *             [--raw out.f32] [--pfm out.pfm] [--device K]
 *             [--events d,d,l,d,m:5:-3,s:64:32,d,...]   (interactive replay: ProgressiveViewHIP
 *              display / arrow keys l r u n / drag motion / reshape, GlutCLWindow.cpp:136-301;
 *              one JSON line per event on stdout: the view state and whether a redisplay was
 *              posted) [--max-progression N] [--frames-out FILE]   (every displayed frame,
 *              appended as raw RGBA32F)
 *             [--tile STRIPE,N,R]   (this process renders rank R's row stripes of N: the raw output
 *              is the compact tile — the sharding path rehearsed as separate processes)
 *             [--comm-ranks N --comm-rank R --comm-id FILE]   (native multi-GPU: one process per
 *              GPU, librtmi's RCCL communicator; rank 0 writes the id to FILE, the others read
 *              it; rt_comm_render per frame, the assembled frame written by rank 0)
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ProgressiveViewHIP.hpp"
#include "RayTracerHIP.hpp"

namespace {

/* init_material / init_sphere, clrt/main.cpp:13-42 */
rt_sphere init_sphere()
{
    rt_sphere s;
    std::memset(&s, 0, sizeof(s));
    s.radius = 1.0f;
    s.mat.specExp = 1000000.0f;
    s.mat.ior = 1.0f;
    s.mat.refExp = 1000000.0f;
    return s;
}

/* clrt/main.cpp:44-110 (ply = clrt/plymain.cpp:45-111) */
void add_scene(RayTracerHIP &rt, bool ply)
{
    rt_sphere s = init_sphere();
    s.center = {-2.0f, -4.0f, -2.0f};
    s.mat.kd = 1.0f;
    s.mat.diffuse = {0.0f, 0.7f, 0.7f};
    rt.addSphere(s);
    s = init_sphere();
    s.center = {2.0f, -3.0f, 2.0f};
    s.mat.ks = 0.2f;
    s.mat.kt = 0.8f;
    s.mat.extinction = ply ? rt_vec3{0.95f, 0.85f, 0.90f} : rt_vec3{0.99f, 0.95f, 0.95f};
    s.mat.ior = 1.1f;
    rt.addSphere(s);
    s = init_sphere();
    s.center = {0.0f, -4.0f, 0.0f};
    s.mat.ks = 1.0f;
    rt.addSphere(s);
    s = init_sphere();
    s.center = {2.0f, -4.0f, -2.0f};
    s.mat.kd = 0.2f;
    s.mat.ks = 0.8f;
    s.mat.diffuse = {0.7f, 0.7f, 0.0f};
    s.mat.specExp = 100.0f;
    rt.addSphere(s);
    s = init_sphere();
    s.center = {-2.0f, -4.0f, 2.0f};
    s.mat.kd = 0.6f;
    s.mat.ks = 0.4f;
    s.mat.diffuse = {0.7f, 0.0f, 0.8f};
    s.mat.specExp = 1000.0f;
    rt.addSphere(s);
    s = init_sphere();
    s.center = ply ? rt_vec3{0.0f, 4.0f, 2.0f} : rt_vec3{2.2f, 1.0f, 2.0f};
    s.radius = 0.5f;
    s.mat.emission_power = 1.0f;
    const float e = ply ? 1.1f : 1.8f;
    s.mat.emission = {e, e, e};
    rt.addSphere(s);
}

int usage()
{
    std::fprintf(stderr, "usage: rt_render [--scene main|ply] [--width W] [--height H] [--frames F] "
                         "[--sample-rate S] [--depth D] [--mesh N | --ply FILE] [--linear] [--raw f] [--pfm f] "
                         "[--device K] [--tile STRIPE,N,R] [--comm-ranks N --comm-rank R --comm-id FILE]\n");
    return 2;
}

/* The communicator id travels through a file: rank 0 writes it (rename makes it appear
   whole), the other ranks wait for it. */
bool share_comm_id(const std::string &path, int rank, uint8_t id[RT_COMM_ID_BYTES])
{
    if (rank == 0) {
        if (rt_comm_get_unique_id(id) != RT_OK) return false;
        const std::string tmp = path + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f || std::fwrite(id, 1, RT_COMM_ID_BYTES, f) != RT_COMM_ID_BYTES) return false;
        std::fclose(f);
        return std::rename(tmp.c_str(), path.c_str()) == 0;
    }
    for (int i = 0; i < 600; ++i) {
        if (FILE *f = std::fopen(path.c_str(), "rb")) {
            const size_t n = std::fread(id, 1, RT_COMM_ID_BYTES, f);
            std::fclose(f);
            if (n == RT_COMM_ID_BYTES) return true;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    return false;
}

} // namespace

int main(int argc, char **argv)
{
    std::string scene = "main", raw, pfm, ply_path, events, comm_id, frames_out;
    unsigned W = 512, H = 512, frames = 1, sr = 1, depth = 6, n_tris = 0, max_prog = 10000;
    int device = 0, comm_ranks = 0, comm_rank = 0;
    rt_tile tile{8, 1, 0};
    bool linear = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char * { return i + 1 < argc ? argv[++i] : nullptr; };
        const char *v = nullptr;
        if (a == "--linear") {
            linear = true;
            continue;
        }
        if (!(v = next())) return usage();
        if (a == "--scene") scene = v;
        else if (a == "--width") W = (unsigned)std::atoi(v);
        else if (a == "--height") H = (unsigned)std::atoi(v);
        else if (a == "--frames") frames = (unsigned)std::atoi(v);
        else if (a == "--sample-rate") sr = (unsigned)std::atoi(v);
        else if (a == "--depth") depth = (unsigned)std::atoi(v);
        else if (a == "--mesh") n_tris = (unsigned)std::atoi(v);
        else if (a == "--ply") ply_path = v;
        else if (a == "--events") events = v;
        else if (a == "--max-progression") max_prog = (unsigned)std::atoi(v);
        else if (a == "--frames-out") frames_out = v;
        else if (a == "--raw") raw = v;
        else if (a == "--pfm") pfm = v;
        else if (a == "--device") device = std::atoi(v);
        else if (a == "--tile") {
            if (std::sscanf(v, "%u,%u,%u", &tile.stripe_rows, &tile.n_ranks, &tile.rank) != 3) return usage();
        } else if (a == "--comm-ranks") comm_ranks = std::atoi(v);
        else if (a == "--comm-rank") comm_rank = std::atoi(v);
        else if (a == "--comm-id") comm_id = v;
        else return usage();
    }
    const bool ply = scene == "ply" || n_tris > 0 || !ply_path.empty();
    try {
        RayTracerHIP rt(device);
        add_scene(rt, ply);
        rt.setSampleRate(sr);
        rt.setMaxPathDepth(depth);
        const float target[3] = {0.0f, -4.0f, 0.0f};
        if (ply) rt.setCameraSpherical(target, 40.0f, 105.0f, 5.0f); /* plymain.cpp:115-117 */
        else rt.setCameraSpherical(target, 14.0f, 118.0f, 5.0f);     /* main.cpp:127-128 */
        int kernel = RT_KERNEL_SPHERES;
        if (!ply_path.empty()) { /* plymain.cpp:121, with the mesh actually handed to the tracer */
            rt.setMeshFromPly(ply_path.c_str());
            rt.setTraversal(linear ? RT_TRAVERSAL_LINEAR : RT_TRAVERSAL_BVH);
            kernel = RT_KERNEL_TRIS;
        } else if (n_tris) {
            std::vector<float> v(3ull * rt_mesh_vertex_count(n_tris));
            std::vector<int> idx(3ull * n_tris);
            if (rt_make_mesh(n_tris, 0.0f, -2.2f, 0.0f, 2.5f, v.data(), idx.data()) != RT_OK) return 1;
            rt.setMesh(v.data(), (unsigned)(v.size() / 3), idx.data(), n_tris);
            rt.setTraversal(linear ? RT_TRAVERSAL_LINEAR : RT_TRAVERSAL_BVH);
            kernel = RT_KERNEL_TRIS;
        }
        if (!events.empty()) { /* interactive replay through the display state machine */
            ProgressiveViewHIP view(rt, W, H, kernel);
            view.setProgressive(max_prog);
            FILE *fo = frames_out.empty() ? nullptr : std::fopen(frames_out.c_str(), "wb");
            if (!frames_out.empty() && !fo) return 1;
            size_t pos = 0;
            while (pos <= events.size()) {
                const size_t end = std::min(events.find(',', pos), events.size());
                const std::string ev = events.substr(pos, end - pos);
                pos = end + 1;
                if (ev.empty()) continue;
                bool post = false, traced = false;
                if (ev == "d") {
                    post = view.display();
                    traced = view.rendered();
                    if (traced && fo) {
                        const std::vector<float> &px = view.pixels();
                        if (std::fwrite(px.data(), 4, px.size(), fo) != px.size()) return 1;
                    }
                } else if (ev == "l") post = view.specialKey(ProgressiveViewHIP::KEY_LEFT);
                else if (ev == "r") post = view.specialKey(ProgressiveViewHIP::KEY_RIGHT);
                else if (ev == "u") post = view.specialKey(ProgressiveViewHIP::KEY_UP);
                else if (ev == "n") post = view.specialKey(ProgressiveViewHIP::KEY_DOWN);
                else if (ev[0] == 'm' || ev[0] == 's') {
                    int a1 = 0, a2 = 0;
                    if (std::sscanf(ev.c_str() + 1, ":%d:%d", &a1, &a2) != 2) return usage();
                    if (ev[0] == 'm') post = view.motion(a1, a2);
                    else view.reshape((unsigned)a1, (unsigned)a2);
                } else return usage();
                std::printf("{\"event\": \"%s\", \"rendered\": %s, \"redisplay\": %s, \"progression\": %u, "
                            "\"azimuth\": %.9g, \"elevation\": %.9g, \"width\": %u, \"height\": %u}\n",
                            ev.c_str(), traced ? "true" : "false", post ? "true" : "false", view.progression(),
                            view.azimuth(), view.elevation(), view.width(), view.height());
            }
            if (fo) std::fclose(fo);
            std::printf("{\"progression\": %u, \"azimuth\": %.9g, \"elevation\": %.9g, \"width\": %u, "
                        "\"height\": %u}\n",
                        view.progression(), view.azimuth(), view.elevation(), view.width(), view.height());
            if (!raw.empty()) {
                FILE *f = std::fopen(raw.c_str(), "wb");
                const std::vector<float> &px = view.pixels();
                if (!f || std::fwrite(px.data(), 4, px.size(), f) != px.size()) return 1;
                std::fclose(f);
            }
            return 0;
        }
        rt_comm *comm = nullptr;
        if (comm_ranks > 0) { /* native multi-GPU: librtmi's RCCL communicator */
            uint8_t id[RT_COMM_ID_BYTES];
            if (comm_id.empty() || !share_comm_id(comm_id, comm_rank, id)) {
                std::fprintf(stderr, "rt_render: no communicator id (--comm-id)\n");
                return 1;
            }
            if (rt_comm_create(id, comm_ranks, comm_rank, device, &comm) != RT_OK) {
                std::fprintf(stderr, "rt_render: rt_comm_create failed\n");
                return 1;
            }
        }
        const bool tiled = !comm && tile.n_ranks > 1;
        const unsigned rows = tiled ? rt_tile_rows(H, &tile) : H;
        float *dbuf = nullptr;
        if (hipMalloc(&dbuf, (size_t)W * std::max(rows, 1u) * 16) != hipSuccess) return 1;
        double rays = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned p = 0; p < frames; ++p) {
            if (comm) {
                rt.flushScene();
                if (rt_comm_render(comm, rt.handle(), dbuf, W, H, p, kernel, 8, 0) != RT_OK) {
                    std::fprintf(stderr, "rt_render: rt_comm_render: %s\n", rt_comm_last_error(comm));
                    return 1;
                }
            } else {
                rt.rayTrace(dbuf, W, H, p, kernel, true, tiled ? &tile : nullptr);
            }
            const rt_counters c = rt.counters();
            rays += (double)(c.rays_closest + c.rays_shadow);
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (comm) rt_comm_destroy(comm);
        if (comm && comm_rank != 0) { /* the frame lives on rank 0 */
            (void)hipFree(dbuf);
            return 0;
        }
        std::vector<float> img((size_t)W * rows * 4);
        if (hipMemcpy(img.data(), dbuf, img.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        (void)hipFree(dbuf);
        std::printf("{\"frames\": %u, \"seconds\": %.6f, \"frames_per_sec\": %.4f, \"mrays_per_sec\": %.2f}\n", frames,
                    dt, frames / dt, rays / dt / 1e6);
        if (!raw.empty()) {
            FILE *f = std::fopen(raw.c_str(), "wb");
            if (!f || std::fwrite(img.data(), 4, img.size(), f) != img.size()) return 1;
            std::fclose(f);
        }
        if (!pfm.empty()) { /* PFM: bottom-to-top rows, RGB, little-endian */
            FILE *f = std::fopen(pfm.c_str(), "wb");
            if (!f) return 1;
            std::fprintf(f, "PF\n%u %u\n-1.0\n", W, rows);
            for (int y = (int)rows - 1; y >= 0; --y)
                for (unsigned x = 0; x < W; ++x) std::fwrite(&img[((size_t)y * W + x) * 4], 4, 3, f);
            std::fclose(f);
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "rt_render: %s\n", e.what());
        return 1;
    }
    return 0;
}
