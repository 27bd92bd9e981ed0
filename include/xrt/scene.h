// xrt/scene.h — Scene (Src/scene.h:13-47, Src/scene.cpp).  Objects live in the same
// std::unordered_map<std::string, std::unique_ptr<Object>> as the reference, so the GPU
// sees them in exactly the reference's iteration order (which decides closest-hit ties and
// BoxMesh overwrites).  build() (empty in the reference) validates the scene; flatten()
// produces the C-ABI description uploaded by HipRenderer.
#pragma once
#include <memory>
#include <filesystem>
#include <string>
#include <unordered_map>
#include <vector>

#include "../xrt.h"
#include "light.h"
#include "material.h"
#include "medium.h"
#include "primitive.h"

class Sampler;

class Scene {
public:
    Scene() = default;
    ~Scene();
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;
    // Scene::loadObj (Src/scene.cpp:46-154) with tinyobjloader v2 parsing/triangulation;
    // same parameter as the reference (a std::string converts implicitly); returns false
    // (and sets lastError) where the reference calls exit(1) — callers that ignore the
    // result, as the reference's examples do, compile unchanged.
    bool loadObj(const std::filesystem::path& filepath);
    void addObj(std::string name, std::unique_ptr<Object> obj);
    void build() {}
    void addAreaLight(std::string name, std::unique_ptr<AreaLight> light);
    const std::vector<std::unique_ptr<AreaLight>>& getAreaLights() const { return m_areaLights; }
    // uniform choice among the area lights (Src/scene.cpp:182-188): one draw
    const AreaLight* sampleAreaLight(Sampler& sampler, float& pdf) const;
    // Scene::intersect / Scene::occluded (Src/scene.cpp:190-211), answered on the GPU by
    // the renderer's own trace kernels (xrt_query on a context of queryDevice(), created and
    // uploaded on first use and re-uploaded after addObj / loadObj / markChanged).  `info`
    // must be fresh (t = t1 = kInfinity), as at every call site of the reference; on a device
    // error intersect / occluded return false and lastError() says why.
    bool intersect(const Ray& ray, IntersectInfo& info) const;
    bool occluded(const Ray& ray, float t_max) const;
    // batched forms: one GPU pass for all rays
    void intersect(const std::vector<Ray>& rays, std::vector<IntersectInfo>& infos, std::vector<char>& hits) const;
    void occluded(const std::vector<Ray>& rays, const std::vector<float>& t_max, std::vector<char>& hits) const;

    // ---- additions for the GPU backend ----
    // HIP device that answers intersect / occluded (default 0).  Changing it drops the
    // current query context; the next query re-creates and re-uploads on the new device.
    void setQueryDevice(int device);
    int queryDevice() const { return m_qdevice; }
    // Geometry edited in place through an object pointer (not via addObj / loadObj) is not
    // seen by the query context until the scene is marked changed.
    void markChanged() { ++m_version; }
    // Flattened, in m_objects iteration order; valid until the scene changes.
    int flatten(xrt_scene_desc* out) const;
    // the one medium referenced by objects (VolumePathTracing scenes), or nullptr;
    // medium() only when it is a HeterogeneousMedium
    const Medium* anyMedium() const;
    const HeterogeneousMedium* medium() const;
    std::vector<std::string> objectNames() const;
    int objectIndex(const Object* obj) const;   // position in iteration order, -1 if absent
    const std::string& lastError() const { return m_error; }
    // materials created by loadObj are owned here (Src/scene.h:46)
    Material* ownMaterial(std::unique_ptr<Material> m);

private:
    std::vector<std::unique_ptr<AreaLight>> m_areaLights;
    std::unordered_map<std::string, std::unique_ptr<Object>> m_objects;
    std::vector<std::unique_ptr<Material>> m_material;
    mutable std::string m_error;
    // ray queries: device context, scene version uploaded to it, objects in iteration order
    uint64_t m_version = 0;
    mutable uint64_t m_qversion = ~0ull;
    mutable xrt_ctx* m_qctx = nullptr;
    int m_qdevice = 0;
    mutable std::vector<const Object*> m_order;
    bool query(const float* rays, const float* tmax, uint32_t n, int mode, xrt_hit* out) const;
    void fillInfo(const xrt_hit& h, IntersectInfo& info) const;
    // flatten() storage
    mutable std::vector<xrt_object> f_objects;
    mutable std::vector<float> f_triv, f_trin, f_sph, f_box;
    mutable std::vector<xrt_light> f_lights;
};
