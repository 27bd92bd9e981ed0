// xrt/sampler.h — Sampler / UniformSampler / DiscreteEmpiricalDistribution1D (Src/sampler.h:
// 8-94, Src/sampler.cpp:3-12) for host code written against the reference API.  The same
// libstdc++ std::mt19937 + uniform_real_distribution<float> as the reference, so a host
// Sampler seeded j + width*i draws exactly the stream the GPU path draws for that pixel
// (the device restates the generator: csrc/step_tri.hip k_refill_merged, path_common.h).
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <random>
#include <vector>

#include "geometry.h"

class Sampler {
public:
    enum class SamplerType { Uniform };

protected:
    std::mt19937 gen;

public:
    Sampler() {}
    Sampler(uint32_t seed) : gen(seed) {}
    virtual ~Sampler() = default;
    static std::unique_ptr<Sampler> makeSampler(SamplerType st);
    void setSeed(uint32_t seed) { gen.seed(seed); }
    void discard(unsigned long long nSkip) { gen.discard(nSkip); }
    virtual float getNext1D() = 0;
    virtual Vec2f getNext2D() = 0;
};

class UniformSampler : public Sampler {
private:
    std::uniform_real_distribution<float> dis;
    int count = 0;

public:
    UniformSampler() : Sampler(), dis(0.0f, 1.0f) {}
    UniformSampler(uint32_t seed) : Sampler(seed), dis(0.0f, 1.0f) {}
    float getNext1D() override {
        count++;
        return dis(gen);
    }
    // Vec2f(dis(gen), dis(gen)): GCC evaluates the second argument first (Src/sampler.h:49)
    Vec2f getNext2D() override {
        count += 2;
        const float b = dis(gen);
        const float a = dis(gen);
        return Vec2f(a, b);
    }
};

inline std::unique_ptr<Sampler> Sampler::makeSampler(SamplerType st) {   // Src/sampler.cpp:3-12
    switch (st) {
        case SamplerType::Uniform: return std::make_unique<UniformSampler>();
    }
    return nullptr;
}

// sample an index from a 1-D discrete empirical distribution (Src/sampler.h:55-94)
class DiscreteEmpiricalDistribution1D {
private:
    std::vector<float> cdf;
    std::vector<float> pdf;

public:
    DiscreteEmpiricalDistribution1D(const float* values, unsigned int N) {
        float sum = 0;
        for (std::size_t i = 0; i < N; ++i) sum += values[i];
        cdf.resize(N + 1);
        cdf[0] = 0;
        for (std::size_t i = 1; i < N + 1; ++i) cdf[i] = cdf[i - 1] + values[i - 1] / sum;
        pdf.resize(N);
        for (std::size_t i = 0; i < N; ++i) pdf[i] = cdf[i + 1] - cdf[i];
    }
    DiscreteEmpiricalDistribution1D(const std::vector<float>& values)
        : DiscreteEmpiricalDistribution1D(values.data(), (unsigned int)values.size()) {}
    uint32_t sample(float u, float& p) const {
        int x = (int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
        if (x == 0) x++;
        p = cdf[x] - cdf[x - 1];
        return (uint32_t)(x - 1);
    }
    float getPDF(uint32_t i) const { return pdf[i]; }
};
