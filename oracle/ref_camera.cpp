/*
 * ref_camera.cpp — the reference's host camera math, compiled against the
 * reference's own vendored gmtl headers (TEST INFRASTRUCTURE ONLY;
 * container-side, part of oracle/_ref/libptref.so).
 *
 * Restates the ~15 lines of host logic that produce the Camera struct the
 * kernel receives: RayTracer::setCameraSpherical (clrt/RayTracer.cpp:33-47)
 * followed by RayTracerCL::updateCLCamera (clrt/RayTracerCL.cpp:178-215),
 * calling the same gmtl templates (Generate.h setRot/setTrans, Xforms.h
 * Quat/Matrix xforms).  The product library restates the same math without
 * gmtl (pathtracer.cl_amd/csrc/rt_host.cpp); tests compare the two.
 */
#include <cmath>
#include <cstdint>

#include "gmtl/EulerAngle.h"
#include "gmtl/Generate.h"
#include "gmtl/Matrix.h"
#include "gmtl/Point.h"
#include "gmtl/Quat.h"
#include "gmtl/Vec.h"
#include "gmtl/VecOps.h"
#include "gmtl/Xforms.h"

#define D2R(x) (x * M_PI / 180.0f) /* RayTracer.cpp:14, RayTracerCL.cpp:36 */

extern "C" __attribute__((visibility("default"))) void
ref_camera_spherical(float tx, float ty, float tz, float elevation_deg, float azimuth_deg, float distance,
                     float fov_deg, uint32_t width, float *out16)
{
    /* RayTracer::setCameraSpherical */
    gmtl::Matrix44f view_matrix;
    gmtl::Point3f target(tx, ty, tz);
    gmtl::Quatf rotation;
    gmtl::setRot(rotation,
                 gmtl::EulerAngle<float, gmtl::ZYX>(0.0f, -D2R(azimuth_deg) + M_PI, -D2R(elevation_deg)));
    gmtl::Vec3f position(0.0f, 0.0f, distance);
    position *= rotation;
    gmtl::setRot(view_matrix, rotation);
    gmtl::setTrans(view_matrix, position + target);

    /* RayTracerCL::updateCLCamera */
    gmtl::Vec3f view(0.0f, 0.0f, -1.0f);
    gmtl::Vec3f up(0.0f, 1.0f, 0.0f);
    view = view_matrix * view;
    up = view_matrix * up;
    gmtl::Vec3f right;
    gmtl::cross(right, view, up);
    view *= (float)((width / 2.0) / tan(D2R(fov_deg) / 2.0));

    const float v[16] = {view[0],  view[1],  view[2],  0.0f, up[0], up[1], up[2], 0.0f,
                         right[0], right[1], right[2], 0.0f, view_matrix(0, 3), view_matrix(1, 3),
                         view_matrix(2, 3), 0.0f};
    for (int i = 0; i < 16; ++i) out16[i] = v[i];
}
