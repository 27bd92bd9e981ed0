// examples/nee.cpp — Src/examples/nee.cpp written against the drop-in API: a heterogeneous
// medium (HeterogeneousMedium(g 0, absorption 0.01, scattering 0.05)) under a sphere light,
// VolumePathTracingNEE(maxDepth 32), rendered by HipRenderer.  The reference reads
// wdas_cloud_quarter.vdb through OpenVDB, which (library and asset) is absent from this
// image; the density comes from a raw float file instead, in a DenseGrid with OpenVDB's
// BoxSampler semantics.
//
//   nee grid.raw nx ny nz origin_x origin_y origin_z voxel [width height spp out.raw [sparse]]
// grid.raw holds nz*ny*nx float32 ([z][y][x]); out.raw receives the linear framebuffer
// (height*width*3 float32; default nee.ppm, gamma 2.2, like the reference example).
// "sparse" stores the density as 8^3 leaf bricks (SparseGrid, the NanoVDB layout) instead.
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include <xrt/camera.h>
#include <xrt/grid.h>
#include <xrt/image.h>
#include <xrt/integrator.h>
#include <xrt/medium.h>
#include <xrt/renderer.h>
#include <xrt/scene.h>

int main(int argc, char** argv) {
    if (argc < 9) {
        std::fprintf(stderr, "usage: nee grid.raw nx ny nz ox oy oz voxel [width height spp out.raw]\n");
        return 1;
    }
    const uint32_t nx = (uint32_t)atoi(argv[2]), ny = (uint32_t)atoi(argv[3]), nz = (uint32_t)atoi(argv[4]);
    const Vec3f origin((float)atof(argv[5]), (float)atof(argv[6]), (float)atof(argv[7]));
    const float voxel = (float)atof(argv[8]);
    const uint32_t width = argc > 9 ? (uint32_t)atoi(argv[9]) : 780;
    const uint32_t height = argc > 10 ? (uint32_t)atoi(argv[10]) : 585;
    const uint32_t n_samples = argc > 11 ? (uint32_t)atoi(argv[11]) : 1024;
    const char* out = argc > 12 ? argv[12] : nullptr;
    const uint32_t max_depth = 32;

    std::vector<float> density((size_t)nx * ny * nz);
    FILE* g = std::fopen(argv[1], "rb");
    if (!g || std::fread(density.data(), sizeof(float), density.size(), g) != density.size()) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 1;
    }
    std::fclose(g);

    Image image(width, height);
    const float aspect_ratio = static_cast<float>(width) / height;
    const Matrix44f c2w(1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 70.0, 550.0, 1.0);
    const float FOV = 60.0f;
    const auto camera = std::make_unique<PinholeCamera>(aspect_ratio, c2w, FOV);

    Scene scene;
    const bool sparse = argc > 13 && std::string(argv[13]) == "sparse";
    std::unique_ptr<DensityGrid> gridData;
    if (sparse)
        gridData = std::make_unique<SparseGrid>(SparseGrid::fromDense(nx, ny, nz, density, origin, voxel));
    else
        gridData = std::make_unique<DenseGrid>(nx, ny, nz, std::move(density), origin, voxel);
    const auto medium = std::make_unique<HeterogeneousMedium>(0.0f, gridData.get(), Vec3f(0.01f), Vec3f(0.05f));
    scene.addObj("medium", medium->makeObject());
    const Matrix44<float> xfm_sphere(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 400.0, 0.0, 1);
    scene.addAreaLight("SphereLight",
                       std::make_unique<SphereLight>(Vec3f(0.0f), 50.0f, xfm_sphere, Vec3f(30.0f, 30.0f, 30.0f)));

    const auto integrator = std::make_unique<VolumePathTracingNEE>(max_depth);
    auto renderer = std::make_unique<HipRenderer>(n_samples, camera.get(), integrator.get());
    renderer->render(scene, Sampler::SamplerType::Uniform, image);
    if (renderer->lastStatus() != 0) {
        std::fprintf(stderr, "render failed: %s\n", renderer->lastError().c_str());
        return 2;
    }
    const xrt_stats& st = renderer->lastStats();
    std::printf("rendered %ux%u x %u spp in %.2f ms: %.1f Msamples/s\n", width, height, n_samples, st.wall_ms,
                (double)st.samples / st.wall_ms / 1e3);
    if (out) {
        FILE* f = std::fopen(out, "wb");
        if (!f || std::fwrite(image.data(), sizeof(float), (size_t)width * height * 3, f) != (size_t)width * height * 3)
            return 3;
        std::fclose(f);
    } else {
        image.gammaCorrection(2.2f);
        image.writePPM("nee.ppm");
    }
    return 0;
}
