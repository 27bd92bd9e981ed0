// xrt/medium.h — Medium / HeterogeneousMedium (Src/medium.h:71-119, 280-387,
// Src/medium.cpp).  Delta tracking runs on the GPU.  The homogeneous variants are only used
// by examples outside the benchmark configs and are not provided.
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
