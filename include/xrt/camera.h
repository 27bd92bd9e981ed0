// xrt/camera.h — Camera / PinholeCamera (Src/camera.h:7-60).  The host computes
// scale = tan(0.5*deg2rad(FOV)) exactly like the reference constructor; ray generation
// runs on the GPU.
#pragma once
#include "geometry.h"

class Camera {
public:
    Camera(float aspect_ratio_, const Matrix44f& c2w) : aspect_ratio(aspect_ratio_), camera2world(c2w) {}
    virtual ~Camera() = default;
    void setTransform(const Matrix44f& c2w) { camera2world = c2w; }
    float aspectRatio() const { return aspect_ratio; }
    const Matrix44f& cameraToWorld() const { return camera2world; }
    virtual float scale() const = 0;

protected:
    float aspect_ratio;
    Matrix44f camera2world;
};

// scale = tan(0.5*deg2rad(FOV)) (Src/camera.h:45).  Every reference example passes a
// compile-time-constant FOV, and GCC -O2 folds std::tan of that constant with MPFR, i.e.
// correctly rounded — glibc's run-time tanf can differ by 1 ulp (FOV 60: 0x1.279a74p-1 vs
// 0x1.279a76p-1).  Computing the correctly rounded value explicitly makes the result the
// same whether or not the caller's FOV is a constant, and equal to the GCC-built reference.
inline float pinhole_scale(float FOV) { return (float)std::tan((long double)(0.5f * deg2rad(FOV))); }

class PinholeCamera : public Camera {
public:
    PinholeCamera(float aspect_ratio_, const Matrix44f& c2w, float FOV = 90.0f)
        : Camera(aspect_ratio_, c2w), FOV_(FOV), scale_(pinhole_scale(FOV)) {}
    float scale() const override { return scale_; }

private:
    float FOV_;
    float scale_;
};
