/*
 * GlPboTargetHIP.hpp — the display side of GlutCLWindow::rayTrace (clrt/GlutCLWindow.cpp:190-227)
 * for RayTracerHIP: renders a frame into an OpenGL pixel-unpack buffer (PBO).
 *
 * GlutCLWindow has two paths, chosen by RayTracerCL::supportsGLSharing():
 *   sharing     clEnqueueAcquireGLObjects on the PBO, rayTrace(&clPBO, ...) writes the frame
 *               straight into it, clEnqueueReleaseGLObjects hands it back to GL (:196-212);
 *   no sharing  rayTrace into a CL buffer, then glMapBuffer(GL_PIXEL_UNPACK_BUFFER, WRITE_ONLY)
 *               and a blocking enqueueReadBuffer into the mapped PBO (:213-226).
 * Here the same two paths:
 *   sharing     hipGraphicsGLRegisterBuffer once per PBO, then per frame
 *               hipGraphicsMapResources → hipGraphicsResourceGetMappedPointer → rt_render with
 *               RT_OUT_DEVICE into the PBO's memory → hipGraphicsUnmapResources;
 *   no sharing  (registration refused: no GL context on the GPU's device, a remote display)
 *               rt_render into a device framebuffer this object owns, then glMapBuffer and
 *               rt_read (the blocking readback) into the mapped PBO.
 * The PBO is registered without WriteDiscard: a progressive frame (progression p > 0) mixes
 * with the frame already in it (GlutCLWindow.cpp:144-158), exactly as the CL kernel read the
 * shared buffer.  In the fallback the device framebuffer carries the accumulated frame, as
 * the reference's clPBOBuff did.
 *
 * Needs a current GL context with GL_PIXEL_UNPACK_BUFFER (GL 2.1 / ARB_pixel_buffer_object)
 * and GL_GLEXT_PROTOTYPES (or a loader) for glBindBuffer / glMapBuffer, and linking with
 * -lGL.  Only the window's rayTrace() changes:
 *
 *     GlPboTargetHIP target(pbo, width, height);        // allocatePBO()
 *     target.rayTrace(rayTracer, progression);          // rayTrace()
 *     target.resize(pbo, width, height);                // reshape: a new PBO
 */
#ifndef GL_PBO_TARGET_HIP_HPP
#define GL_PBO_TARGET_HIP_HPP

#include <GL/gl.h>
#include <GL/glext.h>
#include <hip/hip_runtime_api.h> /* before the interop header, which uses its types */
#include <hip/hip_gl_interop.h>

#include <cstddef>
#include <stdexcept>
#include <string>

#include "RayTracerHIP.hpp"

class GlPboTargetHIP {
public:
    /* try_sharing = false forces the readback path (RayTracerCL's supportsGLSharing() false) */
    GlPboTargetHIP(GLuint pbo, unsigned width, unsigned height, bool try_sharing = true)
        : try_sharing_(try_sharing)
    {
        attach(pbo, width, height);
    }
    ~GlPboTargetHIP() { detach(); }
    GlPboTargetHIP(const GlPboTargetHIP &) = delete;
    GlPboTargetHIP &operator=(const GlPboTargetHIP &) = delete;

    /* a reshaped window's new PBO (GlutCLWindow::allocatePBO after reshape) */
    void resize(GLuint pbo, unsigned width, unsigned height)
    {
        detach();
        attach(pbo, width, height);
    }

    bool sharing() const { return res_ != nullptr; }

    /* GlutCLWindow::rayTrace: one frame (kernel as RayTracerHIP::rayTrace) into the PBO */
    void rayTrace(RayTracerHIP &rt, unsigned progression, int kernel = RT_KERNEL_SPHERES)
    {
        const size_t n_floats = (size_t)w_ * h_ * 4;
        if (res_) {
            hip(hipGraphicsMapResources(1, &res_, nullptr), "hipGraphicsMapResources");
            void *ptr = nullptr;
            size_t bytes = 0;
            hipError_t e = hipGraphicsResourceGetMappedPointer(&ptr, &bytes, res_);
            if (e == hipSuccess && bytes < n_floats * sizeof(float)) e = hipErrorInvalidValue;
            if (e != hipSuccess) {
                (void)hipGraphicsUnmapResources(1, &res_, nullptr);
                hip(e, "PBO mapped pointer (or PBO smaller than width*height*16 bytes)");
            }
            try {
                rt.rayTrace(static_cast<float *>(ptr), w_, h_, progression, kernel, /*on_device=*/true);
            } catch (...) {
                (void)hipGraphicsUnmapResources(1, &res_, nullptr);
                throw;
            }
            hip(hipGraphicsUnmapResources(1, &res_, nullptr), "hipGraphicsUnmapResources");
            return;
        }
        rt.rayTrace(frame_, w_, h_, progression, kernel, /*on_device=*/true);
        glBindBuffer(GL_PIXEL_UNPACK_BUFFER, pbo_);
        float *mapped = static_cast<float *>(glMapBuffer(GL_PIXEL_UNPACK_BUFFER, GL_WRITE_ONLY));
        if (!mapped) {
            glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
            throw std::runtime_error("GlPboTargetHIP: glMapBuffer(GL_PIXEL_UNPACK_BUFFER) failed");
        }
        try {
            rt.read(mapped, n_floats); /* blocking, as enqueueReadBuffer(..., CL_TRUE, ...) */
        } catch (...) {
            glUnmapBuffer(GL_PIXEL_UNPACK_BUFFER);
            glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
            throw;
        }
        glUnmapBuffer(GL_PIXEL_UNPACK_BUFFER);
        glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
    }

private:
    static void hip(hipError_t e, const char *what)
    {
        if (e != hipSuccess)
            throw std::runtime_error(std::string("GlPboTargetHIP: ") + what + ": " + hipGetErrorString(e));
    }

    void attach(GLuint pbo, unsigned width, unsigned height)
    {
        if (!width || !height) throw std::runtime_error("GlPboTargetHIP: empty frame");
        pbo_ = pbo;
        w_ = width;
        h_ = height;
        res_ = nullptr;
        if (try_sharing_ &&
            hipGraphicsGLRegisterBuffer(&res_, pbo, hipGraphicsRegisterFlagsNone) == hipSuccess)
            return;
        res_ = nullptr;
        (void)hipGetLastError(); /* a refused registration is the no-sharing path, not an error */
        hip(hipMalloc(reinterpret_cast<void **>(&frame_), (size_t)w_ * h_ * 4 * sizeof(float)),
            "hipMalloc(framebuffer)");
    }

    void detach()
    {
        if (res_) (void)hipGraphicsUnregisterResource(res_);
        res_ = nullptr;
        if (frame_) (void)hipFree(frame_);
        frame_ = nullptr;
    }

    bool try_sharing_;
    GLuint pbo_ = 0;
    unsigned w_ = 0, h_ = 0;
    hipGraphicsResource_t res_ = nullptr;
    float *frame_ = nullptr; /* no-sharing path: the accumulated frame on the GPU */
};

#endif
