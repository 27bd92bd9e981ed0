// xrt/renderer.h — Renderer (Src/renderer.h:8-20) and HipRenderer, the MI355X backend that
// replaces NormalRenderer / ParallelRenderer (Src/renderer.cpp).  HipRenderer::render has
// the reference's signature and contract: it fills `image` in place with the per-pixel mean
// of n_samples samples (seed j + width*i per pixel, NaN/Inf/negative samples dropped).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "camera.h"
#include "image.h"
#include "integrator.h"
#include "sampler.h"
#include "scene.h"

class Renderer {
public:
    Renderer(Camera* cam, Integrator* inte) : camera(cam), integrator(inte) {}
    virtual ~Renderer() = default;
    virtual void render(const Scene& scene, Sampler::SamplerType st, Image& image) const = 0;

protected:
    const Camera* camera;
    const Integrator* integrator;
};

struct xrt_ctx;
class HipRenderer : public Renderer {
public:
    HipRenderer(uint32_t spp, Camera* cam, Integrator* inte, int device = 0);
    // ParallelRenderer over several GPUs (Src/renderer.cpp:83-99): the image's rows are
    // interleaved over `devices` and assembled on devices[0] (xrt_create_multi)
    HipRenderer(uint32_t spp, Camera* cam, Integrator* inte, std::vector<int> devices);
    ~HipRenderer() override;
    // Errors are reported like the reference reports them (logged; the image is left as
    // rendered so far); lastStatus()/lastError() expose them to callers that care.
    void render(const Scene& scene, Sampler::SamplerType st, Image& image) const override;
    int lastStatus() const { return m_status; }
    const std::string& lastError() const { return m_error; }
    const xrt_stats& lastStats() const { return m_stats; }

private:
    const uint32_t n_samples;
    int m_device;
    std::vector<int> m_devices;   // empty: one GPU (m_device)
    mutable xrt_ctx* m_ctx = nullptr;
    mutable int m_status = 0;
    mutable std::string m_error;
    mutable xrt_stats m_stats{};
};
