// xrt/light.h — AreaLight, QuadLight, TriangleLight, SphereLight (Src/light.h:54-210,
// Src/light.cpp).  Construction applies lightToWorld with multVecMatrix exactly like the
// reference constructors (Src/light.cpp:7-14,32-39,84-91); sampling runs on the GPU.
// makeObject() builds the same emitter objects as the reference (Src/light.cpp:35-41,70-82,93-97).
// Delta lights (PointLight/DistantLight) are only used by WhittedIntegrator, which is out of
// scope, and are not provided.
#pragma once
#include <memory>

#include "geometry.h"
#include "primitive.h"

class AreaLight {
public:
    enum class Kind { Quad, Triangle, Sphere };
    AreaLight(Kind kind, const Matrix44f& l2w, const Vec3f& Le) : m_kind(kind), Le_(Le), lightToWorld(l2w) {}
    virtual ~AreaLight() = default;
    virtual std::unique_ptr<Object> makeObject() = 0;
    Kind kind() const { return m_kind; }
    const Vec3f& Le() const { return Le_; }

protected:
    Kind m_kind;
    Vec3f Le_;
    Matrix44f lightToWorld;
};

class QuadLight : public AreaLight {
public:
    QuadLight(const Vec3f& v0, const Vec3f& v1, const Vec3f& v2, const Matrix44f& l2w, const Vec3f& Le);
    std::unique_ptr<Object> makeObject() override;
    const Vec3f& v0() const { return v0_; }
    const Vec3f& v1() const { return v1_; }
    const Vec3f& v2() const { return v2_; }

private:
    Vec3f v0_, v1_, v2_, e1_, e2_, Ng_;
};

class TriangleLight : public AreaLight {
public:
    TriangleLight(const Vec3f& v0, const Vec3f& v1, const Vec3f& v2, const Matrix44f& l2w, const Vec3f& Le);
    std::unique_ptr<Object> makeObject() override;
    const Vec3f& v0() const { return v0_; }
    const Vec3f& v1() const { return v1_; }
    const Vec3f& v2() const { return v2_; }

private:
    Vec3f v0_, v1_, v2_, e1_, e2_, Ng_;
};

class SphereLight : public AreaLight {
public:
    // The reference picks SphereLight::sample's branch at compile time (Src/light.h:131-197):
    // the default cone sampling, or a uniform point on the sphere with AREA_SAMPLING (off in
    // its build, Src/cmakelists.txt:63).  Here the choice is per light: Sampling::Area renders
    // exactly what a reference built with -DAREA_SAMPLING renders.
    enum class Sampling { Cone, Area };
    SphereLight(const Vec3f& center, float radius, const Matrix44f& l2w, const Vec3f& Le,
                Sampling sampling = Sampling::Cone);
    std::unique_ptr<Object> makeObject() override;
    const Vec3f& center() const { return center_; }
    float radius() const { return radius_; }
    Sampling sampling() const { return sampling_; }

private:
    Vec3f center_;
    float radius_;
    Sampling sampling_;
};
