// xrt/camera.h — Camera / PinholeCamera (Src/camera.h:7-60).  The host computes
// scale = tan(0.5*deg2rad(FOV)) exactly like the reference constructor; the renderer
// generates its rays on the GPU (path_common.h camera_ray), and sampleRay is the same
// expression for host code that asks the camera for a ray.
#pragma once
#include "geometry.h"
#include "ray.h"
#include "sampler.h"

class Camera {
public:
    Camera(float aspect_ratio_, const Matrix44f& c2w) : aspect_ratio(aspect_ratio_), camera2world(c2w) {}
    virtual ~Camera() = default;
    void setTransform(const Matrix44f& c2w) { camera2world = c2w; }
    float aspectRatio() const { return aspect_ratio; }
    const Matrix44f& cameraToWorld() const { return camera2world; }
    virtual float scale() const = 0;
    // sample a ray from sensor coordinates uv in [0, 1)^2 (Src/camera.h:28-30)
    virtual bool sampleRay(const Vec2f& uv, Sampler& sampler, Ray& ray, float& pdf) const = 0;

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
    // PinholeCamera::sampleRay (Src/camera.h:49-60)
    bool sampleRay(const Vec2f& pixel, Sampler&, Ray& ray, float& pdf) const override {
        const Vec3f dir((2 * pixel[0] - 1) * scale_, (1 - 2 * pixel[1]) * scale_ / aspect_ratio, -1);
        ray.direction = normalize(multDirMatrix(dir, camera2world));
        ray.origin = Vec3f(camera2world[3][0], camera2world[3][1], camera2world[3][2]);
        pdf = 1.0f;
        return true;
    }

private:
    float FOV_;
    float scale_;
};
