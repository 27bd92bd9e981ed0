// xrt/integrator.h — the reference's integrators (Src/integrator.h): GIIntegrator
// (:198-291), DirectIntegrator (:76-120), VolumePathTracing (:401-478) — the benchmark
// configs — and IndirectIntegrator (:122-190), NormalIntegrator (:22-74),
// VolumePathTracingNEE (:481-636).  The host objects select the GPU pass
// schedule; they do not integrate on the CPU.  Whitted (delta lights) is not provided.
#pragma once
#include <cstdint>

class Integrator {
public:
    enum class Kind { GI, Direct, VolumePathTracing, Indirect, Normal, VolumePathTracingNEE };
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

class IndirectIntegrator : public Integrator {
public:
    explicit IndirectIntegrator(int maxDepth) : Integrator(Kind::Indirect, (uint32_t)maxDepth) {}
};

class NormalIntegrator : public Integrator {
public:
    NormalIntegrator() : Integrator(Kind::Normal, 1) {}
};

class VolumePathTracingNEE : public Integrator {
public:
    explicit VolumePathTracingNEE(uint32_t maxDepth) : Integrator(Kind::VolumePathTracingNEE, maxDepth) {}
};
