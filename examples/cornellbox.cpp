// examples/cornellbox.cpp — Src/examples/cornellbox.cpp written against the drop-in API:
// the same scene, camera and integrator construction, with HipRenderer in place of
// NormalRenderer/ParallelRenderer.
//
//   cornellbox [width height spp integrator(gi|direct) out.raw devices]
// writes the linear framebuffer (height*width*3 float32) to out.raw (default
// cornellbox.ppm, gamma 1.2, like the reference example).  devices: a comma-separated GPU
// list ("0,1,2,3") renders with the multi-GPU HipRenderer (ParallelRenderer over the node).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <xrt/camera.h>
#include <xrt/image.h>
#include <xrt/integrator.h>
#include <xrt/renderer.h>
#include <xrt/scene.h>

#ifndef DATA_DIR
#define DATA_DIR "xraytracer_amd/data/"
#endif

int main(int argc, char** argv) {
    const uint32_t width = argc > 1 ? (uint32_t)atoi(argv[1]) : 780;
    const uint32_t height = argc > 2 ? (uint32_t)atoi(argv[2]) : 585;
    const uint32_t n_samples = argc > 3 ? (uint32_t)atoi(argv[3]) : 16;
    const std::string kind = argc > 4 ? argv[4] : "gi";
    const char* out = argc > 5 ? argv[5] : nullptr;
    const uint32_t max_depth = 3;

    Image image(width, height);
    const float aspect_ratio = static_cast<float>(width) / height;
    const Matrix44f c2w(-1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, -1.0, 0, 278, 274.4, -750.0, 1);
    const float FOV = 60.0f;
    const auto camera = std::make_unique<PinholeCamera>(aspect_ratio, c2w, FOV);

    Scene scene;
    const char* env = std::getenv("XRT_DATA_DIR");
    const std::string dataDir = env ? env : DATA_DIR;
    if (!scene.loadObj(dataDir + "cornell_box.obj")) {
        std::fprintf(stderr, "%s\n", scene.lastError().c_str());
        return 1;
    }
    scene.addAreaLight("QuadLight", std::make_unique<QuadLight>(Vec3f(343.0, 548.0, 227.0), Vec3f(343.0, 548.0, 332.0),
                                                                Vec3f(213.0, 548.0, 227.0), Matrix44f(),
                                                                25.0f * Vec3f(1.0, 1.0, 1.0)));
    scene.build();

    std::unique_ptr<Integrator> integrator;
    if (kind == "direct") integrator = std::make_unique<DirectIntegrator>();
    else integrator = std::make_unique<GIIntegrator>(max_depth);

    std::vector<int> devices;
    for (const char* p = argc > 6 ? argv[6] : ""; *p;) {
        devices.push_back((int)std::strtol(p, const_cast<char**>(&p), 10));
        if (*p == ',') ++p;
        else break;
    }
    auto renderer = devices.size() > 1
                        ? std::make_unique<HipRenderer>(n_samples, camera.get(), integrator.get(), devices)
                        : std::make_unique<HipRenderer>(n_samples, camera.get(), integrator.get());
    renderer->render(scene, Sampler::SamplerType::Uniform, image);
    if (renderer->lastStatus() != 0) {
        std::fprintf(stderr, "render failed: %s\n", renderer->lastError().c_str());
        return 2;
    }
    const xrt_stats& st = renderer->lastStats();
    std::printf("rendered %ux%u x %u spp in %.2f ms: %.1f Msamples/s, %.4f segments/sample\n", width, height,
                n_samples, st.wall_ms, (double)st.samples / st.wall_ms / 1e3, (double)st.segments / st.samples);
    if (out) {
        FILE* f = std::fopen(out, "wb");
        if (!f || std::fwrite(image.data(), sizeof(float), (size_t)width * height * 3, f) != (size_t)width * height * 3)
            return 3;
        std::fclose(f);
    } else {
        image.gammaCorrection(1.2f);
        image.writePPM("cornellbox.ppm");
    }
    return 0;
}
