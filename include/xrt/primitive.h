// xrt/primitive.h — Primitive, Object, Mesh, Sphere, SphereMesh, BoxMesh
// (Src/primitive.h:6-273).  Same constructors and ownership rules as the reference
// (an Object keeps non-owning Material/AreaLight/Medium pointers).  Intersection runs on
// the GPU; the host objects are descriptors that Scene flattens for upload.
#pragma once
#include <vector>

#include "geometry.h"
#include "ray.h"

class Primitive {
public:
    Primitive(const std::vector<Vec3f>& vertices, const std::vector<Vec3f>& normals,
              const std::vector<Vec2f>& texcoords)
        : m_vertices(vertices), m_normals(normals), m_texcoords(texcoords) {}
    const std::vector<Vec3f>& vertices() const { return m_vertices; }
    const std::vector<Vec3f>& normals() const { return m_normals; }
    const std::vector<Vec2f>& texcoords() const { return m_texcoords; }

private:
    std::vector<Vec3f> m_vertices;
    std::vector<Vec3f> m_normals;
    std::vector<Vec2f> m_texcoords;
};

class Material;
class AreaLight;
class Medium;

class Object {
public:
    enum class Kind { Mesh, Sphere, Box };
    Object(Kind kind, Material* material, AreaLight* light, Medium* medium)
        : m_kind(kind), m_material(material), m_areaLight(light), m_medium(medium) {}
    virtual ~Object() = default;
    bool hasSurface() const { return m_material != nullptr; }
    bool hasAreaLight() const { return m_areaLight != nullptr; }
    bool hasMedium() const { return m_medium != nullptr; }
    MaterialType materialType() const;
    Kind kind() const { return m_kind; }
    const Material* material() const { return m_material; }
    const AreaLight* areaLight() const { return m_areaLight; }
    const Medium* medium() const { return m_medium; }

protected:
    Kind m_kind;
    Material* m_material = nullptr;
    AreaLight* m_areaLight = nullptr;
    Medium* m_medium = nullptr;
};

class Mesh : public Object {
public:
    Mesh(Material* material, AreaLight* light) : Object(Kind::Mesh, material, light, nullptr) {}
    Mesh(std::vector<Primitive>&& prims, Material* material, AreaLight* light = nullptr)
        : Object(Kind::Mesh, material, light, nullptr), m_primitives(std::move(prims)) {}
    Mesh(const std::vector<Primitive>& prims, Material* material, AreaLight* light = nullptr)
        : Object(Kind::Mesh, material, light, nullptr), m_primitives(prims) {}
    const std::vector<Primitive>& primitives() const { return m_primitives; }

protected:
    std::vector<Primitive> m_primitives;
};

// UV-sphere tessellation (Src/primitive.cpp:170-205)
class SphereMesh : public Mesh {
public:
    SphereMesh(Vec3f center, float radius, int thetaResolution, int phiResolution, Material* mt,
               AreaLight* light);

private:
    void Triangulate();
    Vec3f center_;
    float radius_;
    int num_theta_, num_phi_;
};

class Sphere : public Object {
public:
    Sphere(Vec3f center, float radius, Material* material, AreaLight* light = nullptr)
        : Object(Kind::Sphere, material, light, nullptr), m_center(center), m_radius(radius) {}
    const Vec3f& center() const { return m_center; }
    float radius() const { return m_radius; }

private:
    Vec3f m_center;
    float m_radius;
};

class BoxMesh : public Object {
public:
    BoxMesh(AABB box, Medium* medium) : Object(Kind::Box, nullptr, nullptr, medium), m_box(box) {}
    const AABB& box() const { return m_box; }

private:
    AABB m_box;
};
