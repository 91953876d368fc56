/*
 * ref_main_replay — the reference's clrt/main.cpp (and plymain.cpp) calls, written
 * against the reference's own types, compiled against include/RayTracerHIP.hpp.
 *
 * Built with the reference's headers read in place (never copied):
 *   -I<reference>/clrt/ocl  (geometry.h: Sphere, material_t)
 *   -I<reference>/include   (gmtl, CL/cl.h)
 * so it proves that a caller written for RayTracer (RayTracer.h:56-70) compiles
 * unchanged: addSphere(Sphere const &) x6, setSampleRate, setMaxPathDepth,
 * setCameraSpherical(gmtl::Point3f(...), ...) and setCameraMatrix(gmtl::Matrix44f).
 * GlutCLWindow is replaced by its progression loop (GlutCLWindow.cpp:144-158):
 * `frames` renders at progression 0, 1, ... and the last frame is written raw
 * (W*H*4 float32).
 *
 *   ref_main_replay main|ply W H FRAMES OUT.f32 [matrix]
 *
 * `matrix` sets the same camera through setCameraMatrix(gmtl::Matrix44f) built by
 * gmtl from the spherical parameters (RayTracer.cpp:33-47's formula) instead of
 * setCameraSpherical, exercising the matrix overload.
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <vector>

#include "RayTracerHIP.hpp"

#if !defined(RT_HIP_HAVE_REF_GEOMETRY) || !defined(RT_HIP_HAVE_GMTL)
#error "build with the reference's geometry.h and gmtl on the include path"
#endif

#include <cmath>

#include <gmtl/EulerAngle.h>
#include <gmtl/Generate.h>
#include <gmtl/Quat.h>
#include <gmtl/Vec.h>
#include <gmtl/VecOps.h>
#include <gmtl/Xforms.h>

/* main.cpp:13-42: every material/sphere field starts from these values. */
static void reset_material(material_t *m)
{
    m->diffuse.x = m->diffuse.y = m->diffuse.z = 0.0f;
    m->kd = 0.0f;
    m->extinction.x = m->extinction.y = m->extinction.z = 0.0f;
    m->kt = 0.0f;
    m->emission.x = m->emission.y = m->emission.z = 0.0f;
    m->emission_power = 0.0f;
    m->ks = 0.0f;
    m->specExp = 1000000.0f;
    m->ior = 1.0f;
    m->refExp = 1000000.0f;
}

static void reset_sphere(Sphere *s)
{
    s->center.x = s->center.y = s->center.z = 0.0f;
    s->radius = 1.0f;
    reset_material(&s->mat);
}

static void place(Sphere *s, float x, float y, float z)
{
    s->center.x = x;
    s->center.y = y;
    s->center.z = z;
}

static void rgb(vec3 *v, float r, float g, float b)
{
    v->x = r;
    v->y = g;
    v->z = b;
}

/* The six spheres of main.cpp:44-110 (plymain.cpp:45-111 differs in the glass
   sphere's extinction and the light). */
static void add_scene(RayTracerHIP &rt, bool ply)
{
    Sphere s;
    reset_sphere(&s);
    place(&s, -2.0f, -4.0f, -2.0f);
    s.mat.kd = 1.0f;
    rgb(&s.mat.diffuse, 0.0f, 0.7f, 0.7f);
    rt.addSphere(s);

    reset_sphere(&s);
    place(&s, 2.0f, -3.0f, 2.0f);
    s.mat.ks = 0.2f;
    s.mat.kt = 0.8f;
    if (ply)
        rgb(&s.mat.extinction, 0.95f, 0.85f, 0.90f);
    else
        rgb(&s.mat.extinction, 0.99f, 0.95f, 0.95f);
    s.mat.ior = 1.1f;
    rt.addSphere(s);

    reset_sphere(&s);
    place(&s, 0.0f, -4.0f, 0.0f);
    s.mat.ks = 1.0f;
    rt.addSphere(s);

    reset_sphere(&s);
    place(&s, 2.0f, -4.0f, -2.0f);
    s.mat.kd = 0.2f;
    s.mat.ks = 0.8f;
    rgb(&s.mat.diffuse, 0.7f, 0.7f, 0.0f);
    s.mat.specExp = 100.0f;
    rt.addSphere(s);

    reset_sphere(&s);
    place(&s, -2.0f, -4.0f, 2.0f);
    s.mat.kd = 0.6f;
    s.mat.ks = 0.4f;
    rgb(&s.mat.diffuse, 0.7f, 0.0f, 0.8f);
    s.mat.specExp = 1000.0f;
    rt.addSphere(s);

    reset_sphere(&s);
    if (ply) {
        place(&s, 0.0f, 4.0f, 2.0f);
        rgb(&s.mat.emission, 1.1f, 1.1f, 1.1f);
    } else {
        place(&s, 2.2f, 1.0f, 2.0f);
        rgb(&s.mat.emission, 1.8f, 1.8f, 1.8f);
    }
    s.radius = 0.5f;
    s.mat.emission_power = 1.0;
    rt.addSphere(s);
}

/* RayTracer::setCameraSpherical's view matrix (RayTracer.cpp:33-47), built with the
   same gmtl calls, handed over through setCameraMatrix(gmtl::Matrix44f). */
static gmtl::Matrix44f spherical_matrix(gmtl::Point3f const &target, float el, float az, float dist)
{
    const auto d2r = [](float deg) { return deg * M_PI / 180.0f; }; /* RayTracer.cpp:14 */
    gmtl::Quatf rotation;
    gmtl::setRot(rotation, gmtl::EulerAngle<float, gmtl::ZYX>(0.0f, -d2r(az) + M_PI, -d2r(el)));
    gmtl::Vec3f position(0.0f, 0.0f, dist);
    position *= rotation;
    gmtl::Matrix44f m;
    gmtl::setRot(m, rotation);
    gmtl::setTrans(m, position + target);
    return m;
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s main|ply W H FRAMES OUT.f32 [matrix]\n", argv[0]);
        return 2;
    }
    const bool ply = std::strcmp(argv[1], "ply") == 0;
    const unsigned W = (unsigned)std::atoi(argv[2]), H = (unsigned)std::atoi(argv[3]);
    const unsigned frames = (unsigned)std::atoi(argv[4]);
    const bool use_matrix = argc > 6 && std::strcmp(argv[6], "matrix") == 0;
    try {
        RayTracerHIP rayTracer; /* GlutCLWindow's `RayTracerCL rayTracer` member */
        add_scene(rayTracer, ply);
        rayTracer.setSampleRate(1);
        rayTracer.setMaxPathDepth(6);
        const gmtl::Point3f target(0, -4, -0);
        const float el = ply ? 40.0f : 14.0f, az = ply ? 105.0f : 118.0f;
        if (use_matrix)
            rayTracer.setCameraMatrix(spherical_matrix(target, el, az, 5));
        else
            rayTracer.setCameraSpherical(target, el, az, 5);
        std::vector<float> frame((size_t)W * H * 4);
        for (unsigned p = 0; p < frames; ++p) rayTracer.rayTrace(frame.data(), W, H, p);
        FILE *f = std::fopen(argv[5], "wb");
        if (!f || std::fwrite(frame.data(), sizeof(float), frame.size(), f) != frame.size()) {
            std::fprintf(stderr, "cannot write %s\n", argv[5]);
            return 1;
        }
        std::fclose(f);
    } catch (std::exception const &e) {
        std::fprintf(stderr, "ref_main_replay: %s\n", e.what());
        return 3;
    }
    return 0;
}
