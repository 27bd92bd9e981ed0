// xrt/scene.h — Scene (Src/scene.h:13-47, Src/scene.cpp).  Objects live in the same
// std::unordered_map<std::string, std::unique_ptr<Object>> as the reference, so the GPU
// sees them in exactly the reference's iteration order (which decides closest-hit ties and
// BoxMesh overwrites).  build() (empty in the reference) validates the scene; flatten()
// produces the C-ABI description uploaded by HipRenderer.
#pragma once
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../xrt.h"
#include "light.h"
#include "material.h"
#include "medium.h"
#include "primitive.h"

class Scene {
public:
    ~Scene() = default;
    // Scene::loadObj (Src/scene.cpp:46-154) with tinyobjloader v2 parsing/triangulation;
    // returns false (and sets lastError) where the reference calls exit(1).
    bool loadObj(const std::string& filepath);
    void addObj(std::string name, std::unique_ptr<Object> obj);
    void build() {}
    void addAreaLight(std::string name, std::unique_ptr<AreaLight> light);
    const std::vector<std::unique_ptr<AreaLight>>& getAreaLights() const { return m_areaLights; }

    // ---- additions for the GPU backend ----
    // Flattened, in m_objects iteration order; valid until the scene changes.
    int flatten(xrt_scene_desc* out) const;
    // the one medium referenced by objects (VolumePathTracing scenes), or nullptr;
    // medium() only when it is a HeterogeneousMedium
    const Medium* anyMedium() const;
    const HeterogeneousMedium* medium() const;
    std::vector<std::string> objectNames() const;
    const std::string& lastError() const { return m_error; }
    // materials created by loadObj are owned here (Src/scene.h:46)
    Material* ownMaterial(std::unique_ptr<Material> m);

private:
    std::vector<std::unique_ptr<AreaLight>> m_areaLights;
    std::unordered_map<std::string, std::unique_ptr<Object>> m_objects;
    std::vector<std::unique_ptr<Material>> m_material;
    std::string m_error;
    // flatten() storage
    mutable std::vector<xrt_object> f_objects;
    mutable std::vector<float> f_triv, f_trin, f_sph, f_box;
    mutable std::vector<xrt_light> f_lights;
};
