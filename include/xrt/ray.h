// xrt/ray.h — Ray and AABB (Src/ray.h:5-44).  SurfaceInfo/IntersectInfo are device-side
// records in this build (xraytracer_amd/csrc/wavefront.h) and are not part of the host API.
#pragma once
#include "geometry.h"

class Ray {
public:
    Vec3f origin;
    Vec3f direction;
    Vec3f throughput;
    int depth = 0;
    Ray() {}
    Ray(const Vec3f& o, const Vec3f& d) : origin(o), direction(d) {}
    Vec3f operator()(float t) const { return origin + t * direction; }
};

struct AABB {
    Vec3f pMin;
    Vec3f pMax;
};
