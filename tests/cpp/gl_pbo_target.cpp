// tests/cpp/gl_pbo_target.cpp — TEST PROGRAM: GlutCLWindow::rayTrace's display side through
// include/GlPboTargetHIP.hpp (GlutCLWindow.cpp:190-227), compiled and linked against libGL,
// the HIP runtime and librtmi.  With no GL context (this container, the GPU box) it only checks
// that the adapter builds and that a render without a device fails loudly; a desktop session
// with a current GL context runs both PBO paths (run with `window`: not automated here).
#define GL_GLEXT_PROTOTYPES 1
#include "GlPboTargetHIP.hpp"

#include <cstdio>
#include <cstring>

int main(int argc, char **argv)
{
    if (argc > 1 && !strcmp(argv[1], "window")) { /* needs a current GL context and a PBO */
        GLuint pbo = 0;
        glGenBuffers(1, &pbo);
        glBindBuffer(GL_PIXEL_UNPACK_BUFFER, pbo);
        glBufferData(GL_PIXEL_UNPACK_BUFFER, 64 * 64 * 16, nullptr, GL_DYNAMIC_DRAW);
        glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
        RayTracerHIP rt;
        for (int sharing = 1; sharing >= 0; --sharing) {
            GlPboTargetHIP target(pbo, 64, 64, sharing != 0);
            for (unsigned p = 0; p < 3; ++p) target.rayTrace(rt, p);
            std::printf("sharing=%d ok\n", (int)target.sharing());
        }
        return 0;
    }
    try {
        RayTracerHIP rt; /* no GPU: rt_create fails, RayTracerHIP throws */
        std::printf("a device is visible\n");
        return 0;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 3;
    }
}
