// xrt/sampler.h — Sampler::SamplerType (Src/sampler.h:8-14).  Sampling itself is done on the
// GPU with an exact-stream restatement of the reference's std::mt19937 UniformSampler
// (xraytracer_amd/csrc/rng.h); the host API only names the sampler type.
#pragma once

class Sampler {
public:
    enum class SamplerType { Uniform };
    virtual ~Sampler() = default;
};

class UniformSampler : public Sampler {};
