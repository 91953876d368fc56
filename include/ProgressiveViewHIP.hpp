/*
 * ProgressiveViewHIP.hpp — the interactive display step above the path tracer
 * (SURVEY.md §8f item 3), windowing-system free.
 *
 * GlutCLWindow (clrt/GlutCLWindow.cpp:136-301) owns the progressive-refinement loop,
 * the camera controls and the readback into the pixel buffer object it draws.  This
 * class is that state machine with the GL calls left to the host toolkit:
 *
 *   display()        glutDisplayCallback (:136-188): after a (re)allocation render with
 *                    progression 0, else refine while progression < maxProgression
 *                    (progression++), then the non-sharing readback (:214-225) into
 *                    pixels(); returns true when another redisplay should be posted
 *                    (glutPostRedisplay, :149-150, :157); rendered() tells whether it traced;
 *   reshape(w, h)    glutReshapeCallback (:113-134): new buffer at the next display;
 *   specialKey(k)    glutSpecialKeypressCallback (:228-262): arrows orbit the camera by
 *                    3 degrees (azimuth mod 360, elevation clamped to [10, 90]) about
 *                    (0, -4, 0), then restart();
 *   motion(dx, dy)   glutMotionCallback (:270-281): drag orbits by (dx, dy) degrees;
 *   restart()        (:294-301): progression back to 0.  Returns true when a redisplay must
 *                    be posted: refinement had finished (progression >= maxProgression), so
 *                    no display is pending — without it the window would stay frozen on the
 *                    old view.  specialKey and motion return restart()'s answer.
 *
 * The orbit state starts at GlutCLWindow's constructor values (azimuth 105, elevation
 * 40, distance 5, :24-28), independent of the camera the application set — as in the
 * reference.  A GLUT (or any toolkit) window forwards its callbacks here and draws
 * pixels() (RGBA32F, W*H*4, bottom row first as glDrawPixels expects: the tracer's row 0).
 */
#ifndef PROGRESSIVE_VIEW_HIP_HPP
#define PROGRESSIVE_VIEW_HIP_HPP

#include <hip/hip_runtime_api.h>

#include <cmath>
#include <stdexcept>
#include <vector>

#include "RayTracerHIP.hpp"

class ProgressiveViewHIP {
public:
    enum Key { KEY_LEFT, KEY_RIGHT, KEY_UP, KEY_DOWN };

    ProgressiveViewHIP(RayTracerHIP &rt, unsigned width, unsigned height, int kernel = RT_KERNEL_SPHERES)
        : rt_(rt), width_(width), height_(height), kernel_(kernel)
    {
    }
    ~ProgressiveViewHIP() { release(); }
    ProgressiveViewHIP(const ProgressiveViewHIP &) = delete;
    ProgressiveViewHIP &operator=(const ProgressiveViewHIP &) = delete;

    void setProgressive(unsigned maxProgression) { maxProgression_ = maxProgression; } /* GlutCLWindow.h */

    bool display()
    {
        bool again = false;
        rendered_ = false;
        if (realloc_) {
            allocate();
            progression_ = 0;
            trace();
            realloc_ = false;
            again = maxProgression_ > 0;
        } else if (progression_ < maxProgression_) {
            ++progression_;
            trace();
            again = true;
        }
        return again;
    }

    void reshape(unsigned w, unsigned h)
    {
        width_ = w;
        height_ = h;
        realloc_ = true;
    }

    bool specialKey(Key k)
    {
        switch (k) {
        case KEY_LEFT: azimuth_ = std::fmod(azimuth_ + 3.0f, 360.0f); break;
        case KEY_RIGHT: azimuth_ = std::fmod(azimuth_ - 3.0f, 360.0f); break;
        case KEY_UP: elevation_ = std::fmin(elevation_ + 3.0f, 90.0f); break;
        case KEY_DOWN: elevation_ = std::fmax(elevation_ - 3.0f, 10.0f); break;
        }
        orbit();
        return restart();
    }

    bool motion(int dx, int dy)
    {
        azimuth_ = std::fmod(azimuth_ + (float)dx, 360.0f);
        elevation_ = std::fmax(std::fmin(elevation_ + (float)dy, 90.0f), 10.0f);
        orbit();
        return restart();
    }

    bool restart()
    {
        const bool post = progression_ >= maxProgression_;
        progression_ = 0;
        return post;
    }

    const std::vector<float> &pixels() const { return pbo_; }
    unsigned progression() const { return progression_; }
    unsigned maxProgression() const { return maxProgression_; }
    bool rendered() const { return rendered_; }
    float azimuth() const { return azimuth_; }
    float elevation() const { return elevation_; }
    float distance() const { return distance_; }
    unsigned width() const { return width_; }
    unsigned height() const { return height_; }

private:
    void orbit()
    {
        const float target[3] = {0.0f, -4.0f, 0.0f};
        rt_.setCameraSpherical(target, elevation_, azimuth_, distance_);
    }
    void allocate()
    {
        release();
        if (hipMalloc(&dev_, (size_t)width_ * height_ * 4 * sizeof(float)) != hipSuccess)
            throw std::runtime_error("ProgressiveViewHIP: framebuffer allocation failed");
        pbo_.assign((size_t)width_ * height_ * 4, 0.0f);
    }
    void release()
    {
        if (dev_) (void)hipFree(dev_);
        dev_ = nullptr;
    }
    void trace()
    {
        rt_.rayTrace(dev_, width_, height_, progression_, kernel_, true);
        rt_.read(pbo_.data(), pbo_.size()); /* the non-sharing readback into the PBO */
        rendered_ = true;
    }

    RayTracerHIP &rt_;
    unsigned width_, height_;
    int kernel_;
    float *dev_ = nullptr;
    std::vector<float> pbo_;
    bool realloc_ = true, rendered_ = false;
    unsigned progression_ = 0, maxProgression_ = 10000;
    float azimuth_ = 105.0f, elevation_ = 40.0f, distance_ = 5.0f;
};

#endif /* PROGRESSIVE_VIEW_HIP_HPP */
