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

class PinholeCamera : public Camera {
public:
    PinholeCamera(float aspect_ratio_, const Matrix44f& c2w, float FOV = 90.0f)
        : Camera(aspect_ratio_, c2w), FOV_(FOV), scale_(std::tan(0.5f * deg2rad(FOV))) {}
    float scale() const override { return scale_; }

private:
    float FOV_;
    float scale_;
};
