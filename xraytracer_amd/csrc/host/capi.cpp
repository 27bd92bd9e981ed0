// capi.cpp — C facade (xrt_hscene_*) over the C++ Scene API, so non-C++ callers (the
// Python tests and bench) build scenes through exactly the same host code as a C++ user of
// include/xrt/scene.h — including the std::unordered_map object order.
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "xrt.h"
#include "xrt/camera.h"
#include "xrt/scene.h"

namespace {
// Identity-only medium for facade-built scenes: the box just marks "medium 0"; the grid
// and coefficients are uploaded separately with xrt_set_medium.
class FacadeMedium : public Medium {
public:
    FacadeMedium() : Medium(0.0f) {}
    std::unique_ptr<Object> makeObject() override { return nullptr; }
};
}  // namespace

struct xrt_hscene {
    Scene scene;
    std::string err;
    std::vector<std::unique_ptr<Medium>> media;
    std::vector<std::string> names;
};

static Vec3f v3(const float* p) { return Vec3f(p[0], p[1], p[2]); }

extern "C" {

xrt_hscene* xrt_hscene_create(void) {
    try {
        return new xrt_hscene();
    } catch (...) {
        return nullptr;
    }
}

void xrt_hscene_destroy(xrt_hscene* s) { delete s; }

const char* xrt_hscene_last_error(const xrt_hscene* s) { return s ? s->err.c_str() : "null scene"; }

int xrt_hscene_load_obj(xrt_hscene* s, const char* path) {
    if (!s || !path) return XRT_ERR_INVALID;
    try {
        if (!s->scene.loadObj(path)) {
            s->err = s->scene.lastError();
            return XRT_ERR_IO;
        }
    } catch (const std::exception& e) {
        s->err = e.what();
        return XRT_ERR_IO;
    }
    return XRT_OK;
}

int xrt_hscene_add_mesh(xrt_hscene* s, const char* name, const float* tri_v, const float* tri_n, uint32_t n,
                        const float albedo[3]) {
    if (!s || !name || (!tri_v && n) || !albedo) return XRT_ERR_INVALID;
    try {
        std::vector<Primitive> prims;
        prims.reserve(n);
        const std::vector<Vec2f> uv = {Vec2f(0, 0), Vec2f(1, 0), Vec2f(0, 1)};
        for (uint32_t t = 0; t < n; ++t) {
            std::vector<Vec3f> vs = {v3(tri_v + 9 * t), v3(tri_v + 9 * t + 3), v3(tri_v + 9 * t + 6)};
            std::vector<Vec3f> ns;
            if (tri_n) {
                ns = {v3(tri_n + 9 * t), v3(tri_n + 9 * t + 3), v3(tri_n + 9 * t + 6)};
            } else {  // Src/scene.cpp:118-125
                const Vec3f nn = normalize(cross(vs[1] - vs[0], vs[2] - vs[0]));
                ns = {nn, nn, nn};
            }
            prims.emplace_back(vs, ns, uv);
        }
        Material* m = s->scene.ownMaterial(std::make_unique<Lambert>(v3(albedo)));
        s->scene.addObj(name, std::make_unique<Mesh>(std::move(prims), m, nullptr));
    } catch (const std::exception& e) {
        s->err = e.what();
        return XRT_ERR_INVALID;
    }
    return XRT_OK;
}

int xrt_hscene_add_sphere_mesh(xrt_hscene* s, const char* name, const float center[3], float radius, int n_theta,
                               int n_phi, const float albedo[3]) {
    if (!s || !name || !center || !albedo || n_theta < 1 || n_phi < 1) return XRT_ERR_INVALID;
    Material* m = s->scene.ownMaterial(std::make_unique<Lambert>(v3(albedo)));
    s->scene.addObj(name, std::make_unique<SphereMesh>(v3(center), radius, n_theta, n_phi, m, nullptr));
    return XRT_OK;
}

int xrt_hscene_add_sphere(xrt_hscene* s, const char* name, const float center[3], float radius,
                          const float albedo[3]) {
    if (!s || !name || !center || !albedo) return XRT_ERR_INVALID;
    Material* m = s->scene.ownMaterial(std::make_unique<Lambert>(v3(albedo)));
    s->scene.addObj(name, std::make_unique<Sphere>(v3(center), radius, m, nullptr));
    return XRT_OK;
}

int xrt_hscene_add_quad_light(xrt_hscene* s, const char* name, const float v0[3], const float v1[3],
                              const float v2[3], const float Le[3]) {
    if (!s || !name || !v0 || !v1 || !v2 || !Le) return XRT_ERR_INVALID;
    s->scene.addAreaLight(name, std::make_unique<QuadLight>(v3(v0), v3(v1), v3(v2), Matrix44f(), v3(Le)));
    return XRT_OK;
}

int xrt_hscene_add_triangle_light(xrt_hscene* s, const char* name, const float v0[3], const float v1[3],
                                  const float v2[3], const float Le[3]) {
    if (!s || !name || !v0 || !v1 || !v2 || !Le) return XRT_ERR_INVALID;
    s->scene.addAreaLight(name, std::make_unique<TriangleLight>(v3(v0), v3(v1), v3(v2), Matrix44f(), v3(Le)));
    return XRT_OK;
}

int xrt_hscene_add_sphere_light(xrt_hscene* s, const char* name, const float center[3], float radius,
                                const float Le[3]) {
    if (!s || !name || !center || !Le) return XRT_ERR_INVALID;
    s->scene.addAreaLight(name, std::make_unique<SphereLight>(v3(center), radius, Matrix44f(), v3(Le)));
    return XRT_OK;
}

int xrt_hscene_add_sphere_light_area(xrt_hscene* s, const char* name, const float center[3], float radius,
                                     const float Le[3]) {
    if (!s || !name || !center || !Le) return XRT_ERR_INVALID;
    s->scene.addAreaLight(name, std::make_unique<SphereLight>(v3(center), radius, Matrix44f(), v3(Le),
                                                              SphereLight::Sampling::Area));
    return XRT_OK;
}

int xrt_hscene_add_medium_box(xrt_hscene* s, const char* name, const float pmin[3], const float pmax[3]) {
    if (!s || !name || !pmin || !pmax) return XRT_ERR_INVALID;
    if (s->media.empty()) s->media.push_back(std::make_unique<FacadeMedium>());
    s->scene.addObj(name, std::make_unique<BoxMesh>(AABB{v3(pmin), v3(pmax)}, s->media[0].get()));
    return XRT_OK;
}

int xrt_hscene_flatten(xrt_hscene* s, xrt_scene_desc* out) {
    if (!s || !out) return XRT_ERR_INVALID;
    const int rc = s->scene.flatten(out);
    if (rc != XRT_OK) s->err = "flatten failed (unsupported object, material or light)";
    s->names = s->scene.objectNames();
    return rc;
}

const char* xrt_hscene_object_name(const xrt_hscene* s, uint32_t i) {
    if (!s || i >= s->names.size()) return nullptr;
    return s->names[i].c_str();
}

float xrt_pinhole_scale(float fov_deg) {
    return PinholeCamera(1.0f, Matrix44f(), fov_deg).scale();
}

}  // extern "C"
