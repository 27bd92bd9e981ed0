// examples/vpt.cpp — Src/examples/vpt.cpp written against the drop-in API: a homogeneous
// medium box (HomogeneousMediumMIS) lit by a quad light, VolumePathTracing(maxDepth 10),
// rendered by HipRenderer in place of NormalRenderer/ParallelRenderer.
//
//   vpt [width height spp out.raw]
// writes the linear framebuffer (height*width*3 float32) to out.raw (default vpt.ppm,
// gamma 2.2, like the reference example).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>

#include <xrt/camera.h>
#include <xrt/image.h>
#include <xrt/integrator.h>
#include <xrt/medium.h>
#include <xrt/renderer.h>
#include <xrt/scene.h>

int main(int argc, char** argv) {
    const uint32_t width = argc > 1 ? (uint32_t)atoi(argv[1]) : 512;
    const uint32_t height = argc > 2 ? (uint32_t)atoi(argv[2]) : 512;
    const uint32_t n_samples = argc > 3 ? (uint32_t)atoi(argv[3]) : 1024;
    const char* out = argc > 4 ? argv[4] : nullptr;
    const uint32_t max_depth = 10;

    Image image(width, height);
    const float aspect_ratio = static_cast<float>(width) / height;
    const Matrix44f c2w(1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 5.0, 1.0);
    const float FOV = 2.0f * 180.0f * atanf(1.0f / 3.0f) / PI;
    const auto camera = std::make_unique<PinholeCamera>(aspect_ratio, c2w, FOV);

    Scene scene;
    const auto medium = std::make_unique<HomogeneousMediumMIS>(0.0f, Vec3f(0.5f, 0.5f, 0.5f), Vec3f(0.5f),
                                                               AABB{Vec3f(-1.0f), Vec3f(1.0f)});
    scene.addObj("medium", medium->makeObject());
    scene.addAreaLight("QuadLight", std::make_unique<QuadLight>(Vec3f(0.5, 1.4, 0.5), Vec3f(-0.5, 1.4, 0.5),
                                                                Vec3f(0.5, 1.4, -0.5), Matrix44f(),
                                                                10.0f * Vec3f(1.0, 1.0, 1.0)));

    const auto integrator = std::make_unique<VolumePathTracing>(max_depth);
    auto renderer = std::make_unique<HipRenderer>(n_samples, camera.get(), integrator.get());
    renderer->render(scene, Sampler::SamplerType::Uniform, image);
    if (renderer->lastStatus() != 0) {
        std::fprintf(stderr, "render failed: %s\n", renderer->lastError().c_str());
        return 2;
    }
    const xrt_stats& st = renderer->lastStats();
    std::printf("rendered %ux%u x %u spp in %.2f ms: %.1f Msamples/s\n", width, height, n_samples, st.wall_ms,
                (double)st.samples / st.wall_ms / 1e3);
    std::printf("FOV %a\n", (double)FOV);
    if (out) {
        FILE* f = std::fopen(out, "wb");
        if (!f || std::fwrite(image.data(), sizeof(float), (size_t)width * height * 3, f) != (size_t)width * height * 3)
            return 3;
        std::fclose(f);
    } else {
        image.gammaCorrection(2.2f);
        image.writePPM("vpt.ppm");
    }
    return 0;
}
