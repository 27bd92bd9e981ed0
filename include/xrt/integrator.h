// xrt/integrator.h — the reference's integrators (Src/integrator.h): GIIntegrator
// (:198-291), DirectIntegrator (:76-120), VolumePathTracing (:401-478) — the benchmark
// configs — and IndirectIntegrator (:122-190), NormalIntegrator (:22-74),
// VolumePathTracingNEE (:481-636).  The host objects select the GPU pass
// schedule; they do not integrate on the CPU.  Whitted (delta lights) is not provided.
#pragma once
#include <cstdint>
#include <cstdio>
#include <limits>

#include "geometry.h"
#include "ray.h"
#include "sampler.h"

class Scene;

class Integrator {
public:
    // Custom: a subclass written against the reference interface (default constructor +
    // integrate override, Src/integrator.h:9-17).  HipRenderer renders the built-in kinds
    // on the GPU and reports XRT_ERR_UNSUPPORTED for custom ones, which only a CPU
    // renderer calling integrate() per sample can run.
    enum class Kind { GI, Direct, VolumePathTracing, Indirect, Normal, VolumePathTracingNEE, Custom };
    Integrator() : kind_(Kind::Custom), maxDepth_(0) {}
    explicit Integrator(Kind k, uint32_t maxDepth) : kind_(k), maxDepth_(maxDepth) {}
    virtual ~Integrator() = default;
    Kind kind() const { return kind_; }
    uint32_t maxDepth() const { return maxDepth_; }
    // radiance along one ray (Src/integrator.h:14-16).  The built-in integrators run as GPU
    // passes over whole frames (HipRenderer) and have no per-ray host form: called on one
    // of them this logs once and returns NaN — the value the reference's renderer drops as
    // a rejected sample (Src/renderer.cpp:57-73).  Custom integrators override it.
    virtual Vec3f integrate(const Ray&, const Scene&, Sampler&) const {
        static bool warned = false;
        if (!warned) {
            warned = true;
            std::fprintf(stderr, "[xrt] Integrator::integrate: built-in integrators run on the GPU through "
                                 "HipRenderer; no per-ray host integrate\n");
        }
        return Vec3f(std::numeric_limits<float>::quiet_NaN());
    }

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
