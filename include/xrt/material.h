// xrt/material.h — Material / Lambert (Src/material.h:6-77).  BxDF evaluation and sampling
// run on the GPU; the host object carries the albedo.
#pragma once
#include "geometry.h"

class Material {
public:
    virtual ~Material() = default;
    virtual MaterialType materialType() const = 0;
};

class Lambert : public Material {
public:
    explicit Lambert(Vec3f albedo) : m_albedo(albedo) {}
    MaterialType materialType() const override { return MaterialType::Lambert; }
    const Vec3f& albedo() const { return m_albedo; }

private:
    Vec3f m_albedo = Vec3f(0.0f);
};
