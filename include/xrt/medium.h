// xrt/medium.h — Medium / HeterogeneousMedium (Src/medium.h:71-119, 280-387,
// Src/medium.cpp).  Delta tracking runs on the GPU.  The homogeneous variants are at the
// end of this file.
#pragma once
#include <memory>

#include "geometry.h"
#include "grid.h"
#include "primitive.h"

class Medium {
public:
    explicit Medium(float g) : g_(g) {}
    virtual ~Medium() = default;
    virtual std::unique_ptr<Object> makeObject() = 0;
    float g() const { return g_; }

protected:
    float g_;
};

class HeterogeneousMedium : public Medium {
public:
    HeterogeneousMedium(float g, const DensityGrid* densityGridPtr, const Vec3f& absorptionColor,
                        const Vec3f& scatteringColor, float densityMultiplier = 1.0f);
    std::unique_ptr<Object> makeObject() override;   // BoxMesh over getBounds() (Src/medium.cpp:19-22)
    const DensityGrid* grid() const { return densityGridPtr; }
    const Vec3f& absorptionColor() const { return absorption; }
    const Vec3f& scatteringColor() const { return scattering; }
    float densityMultiplier() const { return multiplier; }

private:
    const DensityGrid* densityGridPtr;
    Vec3f absorption, scattering;
    float multiplier;
};

// HomogeneousMedium (Src/medium.h:122-145) and its three sampleMedium variants: MIS
// (:148-192), Achromatic (:195-231), NoMIS (:234-277).  Free-flight sampling and the
// analytic transmittance run on the GPU.
class HomogeneousMedium : public Medium {
public:
    HomogeneousMedium(float g, Vec3f a, Vec3f s, AABB box) : Medium(g), sigma_a(a), sigma_s(s), box(box) {}
    std::unique_ptr<Object> makeObject() override { return std::make_unique<BoxMesh>(box, this); }
    const Vec3f& sigmaA() const { return sigma_a; }
    const Vec3f& sigmaS() const { return sigma_s; }
    const AABB& bounds() const { return box; }

protected:
    Vec3f sigma_a, sigma_s;
    AABB box;
};

class HomogeneousMediumMIS : public HomogeneousMedium {
public:
    HomogeneousMediumMIS(float g, Vec3f a, Vec3f s, AABB box) : HomogeneousMedium(g, a, s, box) {}
};

class HomogeneousMediumAchromatic : public HomogeneousMedium {
public:
    HomogeneousMediumAchromatic(float g, float a, float s, AABB box)
        : HomogeneousMedium(g, Vec3f(a, a, a), Vec3f(s, s, s), box) {}
};

class HomogeneousMediumNoMIS : public HomogeneousMedium {
public:
    HomogeneousMediumNoMIS(float g, Vec3f a, Vec3f s, AABB box) : HomogeneousMedium(g, a, s, box) {}
};
