// xrt/ray.h — Ray, SurfaceInfo, IntersectInfo and AABB (Src/ray.h:5-44).  The renderer keeps
// these records on the device; the host structs are what Scene::intersect fills
// (a GPU query, xrt_query).
#pragma once
#include <cfloat>

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

struct SurfaceInfo {
    Vec3f position;
    Vec3f ng;      // geometric normal
    Vec3f ns;      // shading normal
    Vec3f dpdu;    // tangent vector
    Vec3f dpdv;    // bitangent vector
    Vec2f texcoords;
    Vec2f barycentric;
};

class Object;
struct IntersectInfo {
    float t1 = FLT_MAX;   // [medium]: distance to the surface (kInfinity)
    float t = FLT_MAX;    // distance to the hit point
    SurfaceInfo surfaceInfo;
    const Object* hitObject = nullptr;
};

struct AABB {
    Vec3f pMin;
    Vec3f pMax;
};
