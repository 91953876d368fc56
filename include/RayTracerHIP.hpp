/*
 * RayTracerHIP.hpp — header-only C++ host class over the C-ABI (librtmi.so).
 *
 * The drop-in for the reference's C++ host API: the public surface of
 * RayTracer (clrt/RayTracer.h:51-70) and RayTracerCL::rayTrace
 * (clrt/RayTracerCL.h:111-112) with the same method names, argument meaning,
 * defaults (fov 53, sampleRate 8, maxPathDepth 4: RayTracer.cpp:16-22) and
 * RGBA32F framebuffer layout.  Like the reference (which throws cl::Error),
 * failures throw — here std::runtime_error carrying the C-ABI status text.
 *
 * The scene is re-uploaded only when it changed, as RayTracerCL does when the
 * sphere count changes (RayTracerCL.cpp:251-264).
 *
 * Source compatibility with the reference's callers (clrt/main.cpp, plymain.cpp,
 * GlutCLWindow.cpp): when the reference's own headers are on the include path
 * (-I<reference>/clrt/ocl for geometry.h, -I<reference>/include for gmtl), the
 * overloads taking its types are compiled in:
 *   addSphere / removeSphere (Sphere const &)              RayTracer.h:68-69
 *   setCameraMatrix(gmtl::Matrix44f const &)               RayTracer.h:56
 *   setCameraSpherical(gmtl::Point3f const &, el, az, d)   RayTracer.h:57
 * so `window.rayTracer.addSphere(sphere)` and
 * `setCameraSpherical(gmtl::Point3f(0, -4, -0), 14.0f, 118.0f, 5)` compile unchanged
 * (tests/cpp/ref_main_replay.cpp replays main.cpp / plymain.cpp through this class).
 * Define RT_HIP_NO_REFERENCE_TYPES to leave them out.
 */
#ifndef RAYTRACER_HIP_HPP
#define RAYTRACER_HIP_HPP

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "pathtracer_rt.h"

#if !defined(RT_HIP_NO_REFERENCE_TYPES) && defined(__has_include)
#if __has_include("geometry.h") && __has_include(<CL/cl.h>)
#include "geometry.h" /* clrt/ocl/geometry.h: Sphere, material_t, vec3 */
#define RT_HIP_HAVE_REF_GEOMETRY 1
#endif
#if __has_include(<gmtl/Matrix.h>) && __has_include(<gmtl/Point.h>)
#include <gmtl/Matrix.h>
#include <gmtl/Point.h>
#define RT_HIP_HAVE_GMTL 1
#endif
#endif

class RayTracerHIP {
public:
    explicit RayTracerHIP(int device = 0)
    {
        check(rt_create(device, &ctx_), "rt_create");
        check(rt_set_params(ctx_, sampleRate_, maxPathDepth_), "rt_set_params");
    }
    ~RayTracerHIP()
    {
        if (ctx_) rt_destroy(ctx_);
    }
    RayTracerHIP(const RayTracerHIP &) = delete;
    RayTracerHIP &operator=(const RayTracerHIP &) = delete;

    /* ---- camera: RayTracer.h:56-60 ---- */
    /* 4x4 matrix, column-major (gmtl's storage order). */
    void setCameraMatrix(const float m_colmajor[16]) { check(rt_set_view_matrix(ctx_, m_colmajor), "setCameraMatrix"); }
    void setCameraSpherical(const float target[3], float elevationDeg, float azimuthDeg, float distance)
    {
        check(rt_set_camera_spherical(ctx_, target[0], target[1], target[2], elevationDeg, azimuthDeg, distance),
              "setCameraSpherical");
    }
    void setFoVAngle(float fovDeg)
    {
        fov_ = fovDeg;
        check(rt_set_fov(ctx_, fovDeg), "setFoVAngle");
    }
    float getFoVAngle() const { return fov_; }
#ifdef RT_HIP_HAVE_GMTL
    /* gmtl stores matrices column-major (gmtl/Matrix.h: getData()), the order
       rt_set_view_matrix takes. */
    void setCameraMatrix(gmtl::Matrix44f const &mat) { setCameraMatrix(mat.getData()); }
    void setCameraSpherical(gmtl::Point3f const &target, float elevationDeg, float azimuthDeg, float distance)
    {
        const float t[3] = {target[0], target[1], target[2]};
        setCameraSpherical(t, elevationDeg, azimuthDeg, distance);
    }
#endif

    /* ---- settings: RayTracer.h:62-66 ---- */
    void setSampleRate(unsigned s)
    {
        sampleRate_ = s;
        check(rt_set_params(ctx_, sampleRate_, maxPathDepth_), "setSampleRate");
    }
    unsigned getSampleRate() const { return sampleRate_; }
    void setMaxPathDepth(unsigned d)
    {
        maxPathDepth_ = d;
        check(rt_set_params(ctx_, sampleRate_, maxPathDepth_), "setMaxPathDepth");
    }
    unsigned getMaxPathDepth() const { return maxPathDepth_; }

    /* ---- scene: RayTracer.h:68-70 ---- */
    void addSphere(const rt_sphere &s)
    {
        spheres_.push_back(s);
        dirty_ = true;
    }
    /* The reference leaves removeSphere a stub (RayTracer.cpp:55-58); this removes
       the first byte-identical sphere. */
    void removeSphere(const rt_sphere &s)
    {
        for (size_t i = 0; i < spheres_.size(); ++i)
            if (std::memcmp(&spheres_[i], &s, sizeof(rt_sphere)) == 0) {
                spheres_.erase(spheres_.begin() + (long)i);
                dirty_ = true;
                return;
            }
    }
#ifdef RT_HIP_HAVE_REF_GEOMETRY
    /* The reference's Sphere (geometry.h:156-163), copied field by field into the
       80-byte rt_sphere record the kernels read (same members, same order). */
    static rt_sphere to_rt(Sphere const &r)
    {
        rt_sphere s;
        s.mat.diffuse = {r.mat.diffuse.x, r.mat.diffuse.y, r.mat.diffuse.z};
        s.mat.kd = r.mat.kd;
        s.mat.extinction = {r.mat.extinction.x, r.mat.extinction.y, r.mat.extinction.z};
        s.mat.kt = r.mat.kt;
        s.mat.emission = {r.mat.emission.x, r.mat.emission.y, r.mat.emission.z};
        s.mat.emission_power = r.mat.emission_power;
        s.mat.ks = r.mat.ks;
        s.mat.specExp = r.mat.specExp;
        s.mat.ior = r.mat.ior;
        s.mat.refExp = r.mat.refExp;
        s.center = {r.center.x, r.center.y, r.center.z};
        s.radius = r.radius;
        return s;
    }
    void addSphere(Sphere const &sphere) { addSphere(to_rt(sphere)); }
    void removeSphere(Sphere const &sphere) { removeSphere(to_rt(sphere)); }
#endif
    void clearSpheres()
    {
        spheres_.clear();
        dirty_ = true;
    }

    /* ---- mesh for raytrace_tris (raytracer.cl:184-188); builds the BVH, its cost area leaning
       toward the lights of the spheres added so far (uploaded first; culling only) ---- */
    void setMesh(const float *verts_xyz, unsigned n_verts, const int *idx, unsigned n_tris)
    {
        flushScene();
        check(rt_set_mesh(ctx_, verts_xyz, n_verts, idx, n_tris), "setMesh");
    }
    void setTraversal(int traversal) { check(rt_set_traversal(ctx_, traversal), "setTraversal"); }
    /* BVH builder for the next setMesh: RT_BUILD_HOST (binned SAH) or RT_BUILD_GPU (LBVH). */
    void setBuilder(int builder) { check(rt_set_builder(ctx_, builder), "setBuilder"); }

    /* plymain.cpp's PLYLoader (PLYLoader.cpp:4-90) with the mesh actually handed over:
       read a PLY file, optionally normalise it (extent 3, resting on y = -5, centred on
       x = z = 0) and set it as the mesh. */
    void setMeshFromPly(const char *path, bool normalize = true)
    {
        rt_ply *ply = nullptr;
        uint32_t nv = 0, nt = 0;
        if (rt_ply_open(path, &ply, &nv, &nt) != RT_OK)
            throw std::runtime_error(std::string("setMeshFromPly: ") + rt_ply_last_error());
        std::vector<float> v(3ull * nv);
        std::vector<int32_t> idx(3ull * nt);
        const int r = rt_ply_read(ply, v.data(), idx.data());
        rt_ply_close(ply);
        check(r, "setMeshFromPly: read");
        if (normalize) check(rt_normalize_mesh(v.data(), nv, 3.0f, -5.0f), "setMeshFromPly: normalise");
        setMesh(v.data(), nv, idx.data(), nt);
    }

    /* ---- RayTracerCL::rayTrace(cl_mem*, W, H, progression) ----
       `buff` is W*H*4 floats; a device pointer when on_device, else host memory. */
    void rayTrace(float *buff, unsigned width, unsigned height, unsigned progression,
                  int kernel = RT_KERNEL_SPHERES, bool on_device = false, const rt_tile *tile = nullptr)
    {
        if (dirty_) {
            check(rt_set_spheres(ctx_, spheres_.empty() ? nullptr : spheres_.data(), (uint32_t)spheres_.size()),
                  "scene upload");
            dirty_ = false;
        }
        check(rt_render(ctx_, buff, width, height, progression, kernel, tile, on_device ? RT_OUT_DEVICE : 0),
              "rayTrace");
    }

    /* Upload a changed sphere list now (rayTrace does it itself; callers that drive the
       C-ABI directly with handle(), e.g. rt_comm_render, call this first). */
    void flushScene()
    {
        if (dirty_) {
            check(rt_set_spheres(ctx_, spheres_.empty() ? nullptr : spheres_.data(), (uint32_t)spheres_.size()),
                  "scene upload");
            dirty_ = false;
        }
    }

    /* Blocking readback of the last frame into host memory (the non-sharing display
       path, GlutCLWindow.cpp:214-225); n_floats = capacity of `host`. */
    void read(float *host, size_t n_floats) { check(rt_read(ctx_, host, n_floats), "read"); }

    rt_counters counters() const
    {
        rt_counters c;
        check(rt_get_counters(ctx_, &c), "counters");
        return c;
    }
    rt_ctx *handle() { return ctx_; }

private:
    void check(int st, const char *what) const
    {
        if (st != RT_OK)
            throw std::runtime_error(std::string(what) + ": " + rt_status_string(st) + " (" +
                                     (ctx_ ? rt_last_error(ctx_) : "") + ")");
    }
    rt_ctx *ctx_ = nullptr;
    std::vector<rt_sphere> spheres_;
    bool dirty_ = true;
    float fov_ = 53.0f;
    unsigned sampleRate_ = 8, maxPathDepth_ = 4;
};

#endif /* RAYTRACER_HIP_HPP */
