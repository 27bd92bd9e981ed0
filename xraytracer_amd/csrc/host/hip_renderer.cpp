// hip_renderer.cpp — HipRenderer: the Renderer subclass that drops in where the reference
// uses NormalRenderer / ParallelRenderer (Src/renderer.cpp).  It flattens the Scene,
// uploads it, and runs the MI355X wavefront through the C ABI (include/xrt.h).
#include <cstdio>
#include <cstring>

#include "xrt.h"
#include "xrt/renderer.h"

HipRenderer::HipRenderer(uint32_t spp, Camera* cam, Integrator* inte, int device)
    : Renderer(cam, inte), n_samples(spp), m_device(device) {}

HipRenderer::HipRenderer(uint32_t spp, Camera* cam, Integrator* inte, std::vector<int> devices)
    : Renderer(cam, inte), n_samples(spp), m_device(devices.empty() ? 0 : devices[0]), m_devices(std::move(devices)) {}

HipRenderer::~HipRenderer() {
    if (m_ctx) xrt_destroy(m_ctx);
}

void HipRenderer::render(const Scene& scene, Sampler::SamplerType, Image& image) const {
    auto fail = [&](int rc, const char* what) {
        m_status = rc;
        m_error = std::string(what) + ": " + (m_ctx ? xrt_last_error(m_ctx) : xrt_last_error(nullptr));
        std::fprintf(stderr, "[HipRenderer] %s\n", m_error.c_str());
    };
    m_status = XRT_OK;
    m_error.clear();
    if (!m_ctx) {
        const int rc = m_devices.size() > 1 ? xrt_create_multi(m_devices.data(), (int)m_devices.size(), &m_ctx)
                                            : xrt_create(m_device, &m_ctx);
        if (rc != XRT_OK) return fail(rc, "xrt_create");
    }
    xrt_scene_desc desc;
    int rc = scene.flatten(&desc);
    if (rc != XRT_OK) return fail(rc, "Scene::flatten");
    if ((rc = xrt_upload_scene(m_ctx, &desc)) != XRT_OK) return fail(rc, "xrt_upload_scene");

    const Matrix44f& m = camera->cameraToWorld();
    float c2w[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) c2w[4 * r + c] = m[r][c];
    if ((rc = xrt_set_camera(m_ctx, c2w, camera->scale(), camera->aspectRatio())) != XRT_OK)
        return fail(rc, "xrt_set_camera");

    xrt_render_params p;
    std::memset(&p, 0, sizeof(p));
    switch (integrator->kind()) {
        case Integrator::Kind::GI: p.integrator = XRT_INTEGRATOR_GI; break;
        case Integrator::Kind::Direct: p.integrator = XRT_INTEGRATOR_DIRECT; break;
        case Integrator::Kind::VolumePathTracing: p.integrator = XRT_INTEGRATOR_VPT; break;
        case Integrator::Kind::Indirect: p.integrator = XRT_INTEGRATOR_INDIRECT; break;
        case Integrator::Kind::Normal: p.integrator = XRT_INTEGRATOR_NORMAL; break;
        case Integrator::Kind::VolumePathTracingNEE: p.integrator = XRT_INTEGRATOR_VPT_NEE; break;
        case Integrator::Kind::Custom:
            return fail(XRT_ERR_UNSUPPORTED, "custom Integrator subclasses have no GPU form");
    }
    const HomogeneousMedium* hom = dynamic_cast<const HomogeneousMedium*>(scene.anyMedium());
    if ((p.integrator == XRT_INTEGRATOR_VPT || p.integrator == XRT_INTEGRATOR_VPT_NEE) && hom) {
        xrt_medium_desc md;
        std::memset(&md, 0, sizeof(md));
        md.kind = dynamic_cast<const HomogeneousMediumAchromatic*>(hom) ? XRT_MEDIUM_HOMOGENEOUS_ACHROMATIC
                  : dynamic_cast<const HomogeneousMediumNoMIS*>(hom)    ? XRT_MEDIUM_HOMOGENEOUS_NOMIS
                                                                        : XRT_MEDIUM_HOMOGENEOUS_MIS;
        for (int c = 0; c < 3; ++c) {
            md.bbox_min[c] = hom->bounds().pMin[c];
            md.bbox_max[c] = hom->bounds().pMax[c];
            md.absorption[c] = hom->sigmaA()[c];
            md.scattering[c] = hom->sigmaS()[c];
        }
        md.g = hom->g();
        if ((rc = xrt_set_medium(m_ctx, &md)) != XRT_OK) return fail(rc, "xrt_set_medium");
    } else if (p.integrator == XRT_INTEGRATOR_VPT || p.integrator == XRT_INTEGRATOR_VPT_NEE) {
        const HeterogeneousMedium* med = scene.medium();
        const DenseGrid* grid = med ? dynamic_cast<const DenseGrid*>(med->grid()) : nullptr;
        const SparseGrid* sparse = med ? dynamic_cast<const SparseGrid*>(med->grid()) : nullptr;
        if (!grid && !sparse)
            return fail(XRT_ERR_UNSUPPORTED, "VolumePathTracing needs a HeterogeneousMedium over a DenseGrid or SparseGrid");
        xrt_medium_desc md;
        std::memset(&md, 0, sizeof(md));
        md.nx = grid ? grid->nx() : sparse->nx(), md.ny = grid ? grid->ny() : sparse->ny();
        md.nz = grid ? grid->nz() : sparse->nz();
        const AABB b = med->grid()->getBounds();
        const Vec3f& origin = grid ? grid->origin() : sparse->origin();
        for (int c = 0; c < 3; ++c) {
            md.origin[c] = origin[c];
            md.bbox_min[c] = b.pMin[c];
            md.bbox_max[c] = b.pMax[c];
            md.absorption[c] = med->absorptionColor()[c];
            md.scattering[c] = med->scatteringColor()[c];
        }
        md.voxel_size = grid ? grid->voxelSize() : sparse->voxelSize();
        md.max_density = med->grid()->getMaxDensity();
        md.g = med->g();
        md.density_multiplier = med->densityMultiplier();
        if (grid) {
            md.density = grid->data().data();
            if ((rc = xrt_set_medium(m_ctx, &md)) != XRT_OK) return fail(rc, "xrt_set_medium");
        } else {   // leaf bricks (NanoVDB layout)
            const xrt_brick_grid bg{sparse->bricksX(), sparse->bricksY(), sparse->bricksZ(), sparse->table().data(),
                                    sparse->brickCount(), sparse->bricks().data()};
            if ((rc = xrt_set_medium_bricks(m_ctx, &md, &bg)) != XRT_OK) return fail(rc, "xrt_set_medium_bricks");
        }
    }
    p.max_depth = integrator->maxDepth();
    p.width = image.getWidth();
    p.height = image.getHeight();
    p.spp = n_samples;
    p.shard_index = 0;
    p.shard_count = 1;
    p.flags = XRT_FLAG_ACCUMULATE;   // samples are added to the Image in place (Src/renderer.cpp:75, 98)
    if ((rc = xrt_render(m_ctx, &p, image.data(), &m_stats)) != XRT_OK) return fail(rc, "xrt_render");
}
