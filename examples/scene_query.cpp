// examples/scene_query.cpp — the reference's host-side query API, used the way a reference
// integrator uses it (Src/integrator.h): Sampler draws, PinholeCamera::sampleRay,
// Scene::intersect / Scene::occluded / Scene::sampleAreaLight on the Cornell box.  The
// scene queries run on the GPU (xrt_query); tests/test_gpu_query.py checks every field.
//
//   scene_query data_dir rays.raw n out.raw
// rays.raw: n x {ox, oy, oz, dx, dy, dz, tmax} float32.  out.raw: for every ray, the
// single-ray Scene::intersect record (21 floats: hit, object index, t, t1, position, ng, ns,
// dpdu, dpdv, barycentric — write_info), then the batched records, then
// occluded (single and batched); then 64 UniformSampler(12345) draws, 64 getNext2D pairs,
// 16 camera rays and 64 sampleAreaLight choices.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <xrt/camera.h>
#include <xrt/scene.h>

static std::vector<float> out;

static void write_info(const Scene& scene, bool hit, const IntersectInfo& info) {
    const int obj = info.hitObject ? scene.objectIndex(info.hitObject) : -1;   // iteration order
    out.push_back(hit ? 1.0f : 0.0f);
    out.push_back((float)obj);
    out.push_back(info.t);
    out.push_back(info.t1);
    const SurfaceInfo& s = info.surfaceInfo;
    for (const Vec3f* v : {&s.position, &s.ng, &s.ns, &s.dpdu, &s.dpdv})
        for (int c = 0; c < 3; ++c) out.push_back((*v)[c]);
    out.push_back(s.barycentric[0]);
    out.push_back(s.barycentric[1]);
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: scene_query data_dir rays.raw n out.raw\n");
        return 1;
    }
    const std::string dir = argv[1];
    const int n = atoi(argv[3]);
    std::vector<float> rays((size_t)n * 7);
    FILE* f = std::fopen(argv[2], "rb");
    if (!f || std::fread(rays.data(), sizeof(float), rays.size(), f) != rays.size()) return 1;
    std::fclose(f);

    Scene scene;
    if (!scene.loadObj(dir + "cornell_box.obj")) {
        std::fprintf(stderr, "%s\n", scene.lastError().c_str());
        return 1;
    }
    scene.addAreaLight("QuadLight", std::make_unique<QuadLight>(Vec3f(343.0, 548.0, 227.0), Vec3f(343.0, 548.0, 332.0),
                                                                Vec3f(213.0, 548.0, 227.0), Matrix44f(),
                                                                25.0f * Vec3f(1.0, 1.0, 1.0)));
    scene.build();

    std::vector<Ray> rv;
    std::vector<float> tmax;
    for (int i = 0; i < n; ++i) {
        const float* r = &rays[7 * (size_t)i];
        rv.emplace_back(Vec3f(r[0], r[1], r[2]), Vec3f(r[3], r[4], r[5]));
        tmax.push_back(r[6]);
    }
    // single-ray calls, as an integrator makes them
    for (int i = 0; i < n; ++i) {
        IntersectInfo info;
        const bool hit = scene.intersect(rv[i], info);
        write_info(scene, hit, info);
    }
    // the batched form
    std::vector<IntersectInfo> infos;
    std::vector<char> hits;
    scene.intersect(rv, infos, hits);
    for (int i = 0; i < n; ++i) write_info(scene, hits[i] != 0, infos[i]);
    for (int i = 0; i < n; ++i) out.push_back(scene.occluded(rv[i], tmax[i]) ? 1.0f : 0.0f);
    std::vector<char> occ;
    scene.occluded(rv, tmax, occ);
    for (int i = 0; i < n; ++i) out.push_back(occ[i] ? 1.0f : 0.0f);
    if (!scene.lastError().empty()) {
        std::fprintf(stderr, "%s\n", scene.lastError().c_str());
        return 2;
    }

    // Sampler (Src/sampler.h): getNext1D and getNext2D
    UniformSampler smp;
    smp.setSeed(12345);
    for (int k = 0; k < 64; ++k) {
        const Vec2f u = smp.getNext2D();
        out.push_back(u[0]);
        out.push_back(u[1]);
    }
    std::unique_ptr<Sampler> s2 = Sampler::makeSampler(Sampler::SamplerType::Uniform);
    s2->setSeed(0);
    for (int k = 0; k < 64; ++k) out.push_back(s2->getNext1D());
    // PinholeCamera::sampleRay for the Cornell camera at 800x600
    const Matrix44f c2w(-1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, -1.0, 0, 278, 274.4, -750.0, 1);
    PinholeCamera cam(800.0f / 600.0f, c2w, 60.0f);
    for (int k = 0; k < 16; ++k) {
        Ray ray;
        float pdf = 0.0f;
        const float u = s2->getNext1D();
        const float v = s2->getNext1D();
        cam.sampleRay(Vec2f(u, v), *s2, ray, pdf);
        for (int c = 0; c < 3; ++c) out.push_back(ray.origin[c]);
        for (int c = 0; c < 3; ++c) out.push_back(ray.direction[c]);
        out.push_back(pdf);
    }
    // Scene::sampleAreaLight: one light, pdf 1
    for (int k = 0; k < 64; ++k) {
        float pdf = 0.0f;
        const AreaLight* l = scene.sampleAreaLight(*s2, pdf);
        out.push_back(l == scene.getAreaLights()[0].get() ? 1.0f : 0.0f);
        out.push_back(pdf);
    }
    FILE* o = std::fopen(argv[4], "wb");
    if (!o || std::fwrite(out.data(), sizeof(float), out.size(), o) != out.size()) return 3;
    std::fclose(o);
    return 0;
}
