// xrt/integrator.h — the integrators of the benchmark configs (Src/integrator.h):
// GIIntegrator (:198-291), DirectIntegrator (:76-120), VolumePathTracing (:401-478).
// The host objects select the GPU pass schedule; they do not integrate on the CPU.
// Normal/Indirect/Whitted/VPT-NEE are outside SURVEY.md §8 and not provided yet.
#pragma once
#include <cstdint>

class Integrator {
public:
    enum class Kind { GI, Direct, VolumePathTracing };
    explicit Integrator(Kind k, uint32_t maxDepth) : kind_(k), maxDepth_(maxDepth) {}
    virtual ~Integrator() = default;
    Kind kind() const { return kind_; }
    uint32_t maxDepth() const { return maxDepth_; }

private:
    Kind kind_;
    uint32_t maxDepth_;
};

class GIIntegrator : public Integrator {
public:
    explicit GIIntegrator(int maxDepth) : Integrator(Kind::GI, (uint32_t)maxDepth) {}
};

class DirectIntegrator : public Integrator {
public:
    DirectIntegrator() : Integrator(Kind::Direct, 1) {}
};

class VolumePathTracing : public Integrator {
public:
    explicit VolumePathTracing(uint32_t maxDepth) : Integrator(Kind::VolumePathTracing, maxDepth) {}
};
