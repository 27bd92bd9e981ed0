// scene.cpp — host side of the reference Scene API (include/xrt/*.h): object/light/medium
// construction, Scene::loadObj with tinyobjloader-v2 semantics, and flatten() into the C-ABI
// description in std::unordered_map iteration order.  No ray tracing happens here.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <sstream>

#include "xrt/grid.h"
#include "xrt/image.h"
#include "xrt/light.h"
#include "xrt/sampler.h"
#include "xrt/material.h"
#include "xrt/medium.h"
#include "xrt/primitive.h"
#include "xrt/scene.h"

// ------------------------------------------------------------------ objects ----
MaterialType Object::materialType() const {
    return m_material ? m_material->materialType() : MaterialType::Unknow;
}

// Src/primitive.cpp:170-205.  `sin`/`cos` of a float resolve to the C double functions in
// the reference's translation unit (oracle/overloads.cpp), so the vertex is computed in
// double and narrowed to float by the braced initialiser.
SphereMesh::SphereMesh(Vec3f center, float radius, int thetaResolution, int phiResolution, Material* mt,
                       AreaLight* light)
    : Mesh(mt, light), center_(center), radius_(radius), num_theta_(thetaResolution), num_phi_(phiResolution) {
    Triangulate();
}

void SphereMesh::Triangulate() {
    std::vector<Vec3f> verts, nrms;
    for (int i = 0; i <= num_theta_; ++i) {
        const float theta = PI * i / num_theta_;
        for (int j = 0; j <= num_phi_; ++j) {
            const float phi = 2 * PI * j / num_phi_;
            const double st = ::sin((double)theta), ct = ::cos((double)theta);
            const double sp = ::sin((double)phi), cp = ::cos((double)phi);
            const Vec3f vertex((float)(st * sp), (float)ct, (float)(st * cp));
            verts.push_back(center_ + radius_ * vertex);
            nrms.push_back(vertex);
        }
    }
    const std::vector<Vec2f> uv = {Vec2f(0, 0), Vec2f(1, 0), Vec2f(0, 1)};
    for (int i = 0; i < num_theta_; ++i) {
        for (int j = 0; j < num_phi_; ++j) {
            const int a = i * (num_phi_ + 1) + j, b = a + num_phi_ + 1;
            m_primitives.emplace_back(std::vector<Vec3f>{verts[a], verts[b], verts[a + 1]},
                                      std::vector<Vec3f>{nrms[a], nrms[b], nrms[a + 1]}, uv);
            m_primitives.emplace_back(std::vector<Vec3f>{verts[b], verts[b + 1], verts[a + 1]},
                                      std::vector<Vec3f>{nrms[b], nrms[b + 1], nrms[a + 1]}, uv);
        }
    }
}

// ------------------------------------------------------------------ lights ----
// Constructors apply l2w with multVecMatrix (Src/light.cpp:7-14, 32-39, 84-91).
QuadLight::QuadLight(const Vec3f& v0, const Vec3f& v1, const Vec3f& v2, const Matrix44f& l2w, const Vec3f& Le)
    : AreaLight(Kind::Quad, l2w, Le), v0_(multVecMatrix(v0, l2w)), v1_(multVecMatrix(v1, l2w)),
      v2_(multVecMatrix(v2, l2w)) {
    e1_ = v1_ - v0_;
    e2_ = v2_ - v0_;
    Ng_ = cross(e1_, e2_);
}

// Two triangles (v0,v1,v2), (v1,v0+e1+e2,v2) with normal normalize(Ng) (Src/light.cpp:70-82)
std::unique_ptr<Object> QuadLight::makeObject() {
    const Vec3f v3 = v0_ + e1_ + e2_;
    const Vec3f n = normalize(Ng_);
    const std::vector<Vec3f> nn = {n, n, n};
    const std::vector<Vec2f> uv = {Vec2f(0, 0), Vec2f(1, 0), Vec2f(0, 1)};
    std::vector<Primitive> prims = {Primitive({v0_, v1_, v2_}, nn, uv), Primitive({v1_, v3, v2_}, nn, uv)};
    return std::make_unique<Mesh>(std::move(prims), nullptr, this);
}

TriangleLight::TriangleLight(const Vec3f& v0, const Vec3f& v1, const Vec3f& v2, const Matrix44f& l2w,
                             const Vec3f& Le)
    : AreaLight(Kind::Triangle, l2w, Le), v0_(multVecMatrix(v0, l2w)), v1_(multVecMatrix(v1, l2w)),
      v2_(multVecMatrix(v2, l2w)) {
    e1_ = v1_ - v0_;
    e2_ = v2_ - v0_;
    Ng_ = cross(e1_, e2_);
}

std::unique_ptr<Object> TriangleLight::makeObject() {  // Src/light.cpp:35-41
    const Vec3f n = normalize(Ng_);
    std::vector<Primitive> prims = {Primitive({v0_, v1_, v2_}, {n, n, n}, {Vec2f(0, 0), Vec2f(1, 0), Vec2f(0, 1)})};
    return std::make_unique<Mesh>(std::move(prims), nullptr, this);
}

SphereLight::SphereLight(const Vec3f& center, float radius, const Matrix44f& l2w, const Vec3f& Le, Sampling sampling)
    : AreaLight(Kind::Sphere, l2w, Le), center_(multVecMatrix(center, l2w)), radius_(radius), sampling_(sampling) {}

std::unique_ptr<Object> SphereLight::makeObject() {  // Src/light.cpp:93-97
    return std::make_unique<Sphere>(center_, radius_, nullptr, this);
}

// ------------------------------------------------------------------ medium ----
DenseGrid::DenseGrid(uint32_t nx, uint32_t ny, uint32_t nz, std::vector<float> data, Vec3f origin, float voxelSize)
    : nx_(nx), ny_(ny), nz_(nz), data_(std::move(data)), origin_(origin), voxel_(voxelSize) {}

// OpenVDB indexToWorld(activeVoxelBBox.start/end) in double (Src/grid.h:58-69): voxel
// centres of the first and last voxel.
AABB DenseGrid::getBounds() const {
    AABB b;
    const double n[3] = {(double)nx_ - 1.0, (double)ny_ - 1.0, (double)nz_ - 1.0};
    for (int i = 0; i < 3; ++i) {
        b.pMin[i] = (float)(0.0 * (double)voxel_ + (double)origin_[i]);
        b.pMax[i] = (float)(n[i] * (double)voxel_ + (double)origin_[i]);
    }
    return b;
}

SparseGrid::SparseGrid(uint32_t nx, uint32_t ny, uint32_t nz, std::vector<int32_t> table, std::vector<float> bricks,
                       Vec3f origin, float voxelSize)
    : nx_(nx), ny_(ny), nz_(nz), table_(std::move(table)), bricks_(std::move(bricks)), origin_(origin), voxel_(voxelSize) {}

SparseGrid SparseGrid::fromDense(uint32_t nx, uint32_t ny, uint32_t nz, const std::vector<float>& d, Vec3f origin,
                                 float voxelSize) {
    const uint32_t B = kBrick, bx = (nx + B - 1) / B, by = (ny + B - 1) / B, bz = (nz + B - 1) / B;
    std::vector<int32_t> table((size_t)bx * by * bz, -1);
    std::vector<float> bricks;
    std::vector<float> leaf(B * B * B);
    for (uint32_t k = 0; k < bz; ++k)
        for (uint32_t j = 0; j < by; ++j)
            for (uint32_t i = 0; i < bx; ++i) {
                bool any = false;
                for (uint32_t z = 0; z < B; ++z)
                    for (uint32_t y = 0; y < B; ++y)
                        for (uint32_t x = 0; x < B; ++x) {
                            const uint32_t gx = i * B + x, gy = j * B + y, gz = k * B + z;
                            const float v = gx < nx && gy < ny && gz < nz ? d[((size_t)gz * ny + gy) * nx + gx] : 0.0f;
                            leaf[(z * B + y) * B + x] = v;
                            any |= v != 0.0f;
                        }
                if (!any) continue;
                table[((size_t)k * by + j) * bx + i] = (int32_t)(bricks.size() / leaf.size());
                bricks.insert(bricks.end(), leaf.begin(), leaf.end());
            }
    return SparseGrid(nx, ny, nz, std::move(table), std::move(bricks), origin, voxelSize);
}

AABB SparseGrid::getBounds() const {   // as DenseGrid::getBounds
    AABB b;
    const double n[3] = {(double)nx_ - 1.0, (double)ny_ - 1.0, (double)nz_ - 1.0};
    for (int i = 0; i < 3; ++i) {
        b.pMin[i] = (float)(0.0 * (double)voxel_ + (double)origin_[i]);
        b.pMax[i] = (float)(n[i] * (double)voxel_ + (double)origin_[i]);
    }
    return b;
}

float SparseGrid::getMaxDensity() const {   // inactive voxels read 0
    float m = 0.0f;
    for (float v : bricks_) m = std::max(m, v);
    return m;
}

float DenseGrid::getMaxDensity() const {  // evalMinMax (Src/grid.h:79-83)
    float m = data_.empty() ? 0.0f : data_[0];
    for (float v : data_) m = std::max(m, v);
    return m;
}

HeterogeneousMedium::HeterogeneousMedium(float g, const DensityGrid* grid, const Vec3f& absorptionColor,
                                         const Vec3f& scatteringColor, float densityMultiplier)
    : Medium(g), densityGridPtr(grid), absorption(absorptionColor), scattering(scatteringColor),
      multiplier(densityMultiplier) {}

std::unique_ptr<Object> HeterogeneousMedium::makeObject() {
    return std::make_unique<BoxMesh>(densityGridPtr->getBounds(), this);
}

// ------------------------------------------------------------------ image ----
Image& Image::operator/=(const Vec3f& rgb) {
    for (auto& p : pixels) p = p / rgb;
    return *this;
}
Image& Image::operator*=(const Vec3f& rgb) {
    for (auto& p : pixels) p = p * rgb;
    return *this;
}
void Image::gammaCorrection(float gamma) {  // Src/image.h:80-90
    for (auto& p : pixels)
        for (int c = 0; c < 3; ++c) p[c] = std::pow(p[c], 1.0f / gamma);
}
bool Image::writePPM(const std::string& filename) const {  // Src/image.h:92-114
    std::ofstream f(filename);
    if (!f) return false;
    f << "P3\n" << width << " " << height << "\n255\n";
    for (const auto& p : pixels) {
        for (int c = 0; c < 3; ++c) {
            const uint32_t v = std::clamp(static_cast<uint32_t>(255.0f * p[c]), 0u, 255u);
            f << v << (c < 2 ? " " : "\n");
        }
    }
    return (bool)f;
}

// ------------------------------------------------------------------ OBJ ----
// A restatement of the parts of tinyobjloader v2 (2.0.0rc13, the vcpkg port current at the
// reference snapshot; third-party, absent here) that Scene::loadObj relies on:
// tryParseDouble number parsing, 1-based/negative index fixing, shapes split at `o`/`g`,
// faces flushed at `usemtl` changes, quads split along the shorter diagonal, polygons of five
// or more vertices by tinyobjloader's built-in ear clipping (tinyobj_ear_clip below), MTL
// Kd/Ke/illum/unknown parameters.  Parity of the ear clipping is unpinned: the library is
// absent and no reference test or testdata file has such a face (tests/test_host_scene.py
// checks its invariants: n - 2 triangles covering the polygon).
namespace {

bool tinyobj_parse_double(const char* s, const char* end, double* result) {
    if (s >= end) return false;
    double mantissa = 0.0;
    int exponent = 0, read = 0;
    char sign = '+', exp_sign = '+';
    const char* c = s;
    bool leading_dot = false;
    if (*c == '+' || *c == '-') {
        sign = *c++;
        if (c != end && *c == '.') leading_dot = true;
    } else if (*c == '.') {
        leading_dot = true;
    } else if (!(*c >= '0' && *c <= '9')) {
        return false;
    }
    bool more = c != end;
    if (!leading_dot) {
        while (more && *c >= '0' && *c <= '9') {
            mantissa = mantissa * 10 + (double)(*c - '0');
            ++c, ++read;
            more = c != end;
        }
        if (read == 0) return false;
    }
    if (more) {
        if (*c == '.') {
            ++c;
            read = 1;
            more = c != end;
            static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            while (more && *c >= '0' && *c <= '9') {
                mantissa += (double)(int)(*c - '0') * (read < 8 ? lut[read] : std::pow(10.0, -read));
                ++read, ++c;
                more = c != end;
            }
        }
        if (more && (*c == 'e' || *c == 'E')) {
            ++c;
            more = c != end;
            if (more && (*c == '+' || *c == '-')) exp_sign = *c++;
            else if (!(more && *c >= '0' && *c <= '9')) return false;
            read = 0;
            more = c != end;
            while (more && *c >= '0' && *c <= '9') {
                if (exponent > 2147483647 / 10) return false;
                exponent = exponent * 10 + (*c - '0');
                ++c, ++read;
                more = c != end;
            }
            exponent *= (exp_sign == '+' ? 1 : -1);
            if (read == 0) return false;
        }
    }
    *result = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
    return true;
}

// parseReal: token up to whitespace, default on failure, cast to real_t (float)
float parse_real(const char*& p, double def = 0.0) {
    p += strspn(p, " \t");
    const char* e = p + strcspn(p, " \t\r\n");
    double v = def;
    tinyobj_parse_double(p, e, &v);
    p = e;
    return (float)v;
}

struct ObjMaterial {
    std::string name;
    float diffuse[3] = {0, 0, 0};
    float emission[3] = {0, 0, 0};
    int illum = 0;
    std::map<std::string, std::string> unknown;
};

struct VRef { int v, vt, vn; };

struct ObjShape {
    std::string name;
    std::vector<VRef> idx;       // 3 per triangle
    std::vector<int> material;   // per triangle
};

std::string trim(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

bool load_mtl(const std::string& path, std::vector<ObjMaterial>& mats, std::map<std::string, int>& ids,
              std::string& warn) {
    std::ifstream f(path);
    if (!f) {
        warn += "material file not found: " + path + "\n";
        return false;
    }
    std::string line;
    ObjMaterial cur;
    bool have = false;
    auto flush = [&]() {
        if (have) {
            ids[cur.name] = (int)mats.size();
            mats.push_back(cur);
        }
    };
    while (std::getline(f, line)) {
        const char* p = line.c_str();
        p += strspn(p, " \t");
        if (*p == '\0' || *p == '#' || *p == '\r') continue;
        if (!strncmp(p, "newmtl", 6) && (p[6] == ' ' || p[6] == '\t')) {
            flush();
            cur = ObjMaterial();
            cur.name = trim(p + 7);
            have = true;
        } else if ((p[0] == 'K' && p[1] == 'd') && (p[2] == ' ' || p[2] == '\t')) {
            p += 2;
            for (float& v : cur.diffuse) v = parse_real(p);
        } else if ((p[0] == 'K' && p[1] == 'e') && (p[2] == ' ' || p[2] == '\t')) {
            p += 2;
            for (float& v : cur.emission) v = parse_real(p);
        } else if (!strncmp(p, "illum", 5) && (p[5] == ' ' || p[5] == '\t')) {
            cur.illum = atoi(p + 6);
        } else if ((p[0] == 'K' && (p[1] == 'a' || p[1] == 's' || p[1] == 't')) || !strncmp(p, "Ns", 2) ||
                   !strncmp(p, "Ni", 2) || p[0] == 'd' || !strncmp(p, "Tr", 2) || !strncmp(p, "Tf", 2) ||
                   !strncmp(p, "map_", 4)) {
            // known tinyobj parameters that Scene::makeMaterial does not read
        } else {
            const char* e = p + strcspn(p, " \t");
            std::string key(p, e);
            cur.unknown[key] = trim(e);
        }
    }
    flush();
    return true;
}

// tinyobjloader's pnpoly: even-odd crossing test of (tx, ty) against the triangle (vx, vy)
int tinyobj_pnpoly(const float* vx, const float* vy, float tx, float ty) {
    int c = 0;
    for (int i = 0, j = 2; i < 3; j = i++)
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    return c;
}

// exportGroupsToShape's built-in ear clipping (tinyobjloader v2, no TINYOBJLOADER_USE_MAPBOX_
// EARCUT, real_t = float): project on the two axes that drop the largest component of the
// first corner's cross product; walk `guess` around the remaining polygon, emit the
// triangle (guess, guess + 1, guess + 2) unless it turns against the polygon's running
// "area" sign (an inner corner) or another remaining vertex lies in it, then remove vertex
// guess + 1; give up after a full lap without an ear; the last three vertices are the last
// triangle.  Appends the triangles (index triples) to `out`.
void tinyobj_ear_clip(const std::vector<VRef>& face, const std::vector<float>& v, std::vector<VRef>& out) {
    const size_t n0 = face.size();
    size_t axes[2] = {1, 2};
    for (size_t k = 0; k < n0; ++k) {
        const size_t a = (size_t)face[k % n0].v, b = (size_t)face[(k + 1) % n0].v, c = (size_t)face[(k + 2) % n0].v;
        if (3 * a + 2 >= v.size() || 3 * b + 2 >= v.size() || 3 * c + 2 >= v.size()) continue;
        const float e0x = v[3 * b] - v[3 * a], e0y = v[3 * b + 1] - v[3 * a + 1], e0z = v[3 * b + 2] - v[3 * a + 2];
        const float e1x = v[3 * c] - v[3 * b], e1y = v[3 * c + 1] - v[3 * b + 1], e1z = v[3 * c + 2] - v[3 * b + 2];
        const float cx = std::fabs(e0y * e1z - e0z * e1y), cy = std::fabs(e0z * e1x - e0x * e1z),
                    cz = std::fabs(e0x * e1y - e0y * e1x);
        const float eps = std::numeric_limits<float>::epsilon();
        if (cx > eps || cy > eps || cz > eps) {
            if (!(cx > cy && cx > cz)) {
                axes[0] = 0;
                if (cz > cx && cz > cy) axes[1] = 1;
            }
            break;
        }
    }
    std::vector<VRef> rem = face;
    size_t guess = 0, iters = n0, prev = rem.size();
    VRef ind[3];
    float vx[3], vy[3];
    while (rem.size() > 3 && iters > 0) {
        const size_t np = rem.size();
        if (guess >= np) guess -= np;
        if (prev != np) prev = np, iters = np;
        else --iters;
        for (int k = 0; k < 3; ++k) {
            ind[k] = rem[(guess + k) % np];
            const size_t vi = (size_t)ind[k].v;
            const bool bad = vi * 3 + axes[0] >= v.size() || vi * 3 + axes[1] >= v.size();
            vx[k] = bad ? 0.0f : v[vi * 3 + axes[0]];
            vy[k] = bad ? 0.0f : v[vi * 3 + axes[1]];
        }
        const float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
        const float cross = e0x * e1y - e0y * e1x;
        const float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
        if (cross * area < 0.0f) {   // an inner corner
            guess += 1;
            continue;
        }
        bool overlap = false;
        for (size_t other = 3; other < np; ++other) {
            const size_t idx = (guess + other) % np;
            const size_t ovi = (size_t)rem[idx].v;
            if (ovi * 3 + axes[0] >= v.size() || ovi * 3 + axes[1] >= v.size()) continue;
            if (tinyobj_pnpoly(vx, vy, v[ovi * 3 + axes[0]], v[ovi * 3 + axes[1]])) {
                overlap = true;
                break;
            }
        }
        if (overlap) {
            guess += 1;
            continue;
        }
        for (int k = 0; k < 3; ++k) out.push_back(ind[k]);   // an ear
        for (size_t r = (guess + 1) % np; r + 1 < np; ++r) rem[r] = rem[r + 1];
        rem.pop_back();
    }
    if (rem.size() == 3)
        for (int k = 0; k < 3; ++k) out.push_back(rem[k]);
}

int fix_index(int idx, int n, bool& ok) {
    if (idx > 0) return idx - 1;
    if (idx == 0) { ok = false; return 0; }
    return n + idx;
}

}  // namespace

// Scene::loadObj (Src/scene.cpp:46-154)
bool Scene::loadObj(const std::filesystem::path& path) {
    // tinyobjloader reads generic_string(); MTL files are looked up next to the OBJ
    // (reader_config.mtl_search_path = parent_path(), Src/scene.cpp:51-53)
    const std::string filepath = path.generic_string();
    std::ifstream f(filepath);
    if (!f) {
        m_error = "[Scene] failed to load " + filepath;
        return false;
    }
    const std::string dir = filepath.find('/') == std::string::npos ? "" : filepath.substr(0, filepath.rfind('/') + 1);
    std::vector<float> pos, nrm, tex;
    std::vector<ObjMaterial> mats;
    std::map<std::string, int> mat_ids;
    std::vector<ObjShape> shapes;
    std::vector<std::vector<VRef>> faces;  // current face group
    ObjShape cur;
    int material = -1;
    std::string warn, line;

    auto export_group = [&]() {  // exportGroupsToShape with triangulate = true
        for (const auto& fc : faces) {
            const size_t n = fc.size();
            if (n < 3) continue;
            if (n == 4) {
                auto P = [&](int k, int c) { return pos[3 * (size_t)fc[k].v + c]; };
                const float e02x = P(2, 0) - P(0, 0), e02y = P(2, 1) - P(0, 1), e02z = P(2, 2) - P(0, 2);
                const float e13x = P(3, 0) - P(1, 0), e13y = P(3, 1) - P(1, 1), e13z = P(3, 2) - P(1, 2);
                const float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
                const float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
                const int tri[2][3] = {{0, 1, 2}, {0, 2, 3}}, tri2[2][3] = {{0, 1, 3}, {1, 2, 3}};
                const int(*t)[3] = sqr02 < sqr13 ? tri : tri2;
                for (int k = 0; k < 2; ++k) {
                    for (int c = 0; c < 3; ++c) cur.idx.push_back(fc[t[k][c]]);
                    cur.material.push_back(material);
                }
            } else if (n == 3) {
                for (int c = 0; c < 3; ++c) cur.idx.push_back(fc[c]);
                cur.material.push_back(material);
            } else {
                const size_t before = cur.idx.size();
                tinyobj_ear_clip(fc, pos, cur.idx);
                for (size_t k = before; k < cur.idx.size(); k += 3) cur.material.push_back(material);
            }
        }
        faces.clear();
    };
    auto flush_shape = [&]() {
        export_group();
        if (!cur.idx.empty()) shapes.push_back(cur);
        cur = ObjShape();
    };

    while (std::getline(f, line)) {
        const char* p = line.c_str();
        p += strspn(p, " \t");
        if (*p == '\0' || *p == '#' || *p == '\r') continue;
        const bool sp1 = p[1] == ' ' || p[1] == '\t';
        if (p[0] == 'v' && sp1) {
            p += 1;
            for (int c = 0; c < 3; ++c) pos.push_back(parse_real(p));
        } else if (p[0] == 'v' && p[1] == 'n' && (p[2] == ' ' || p[2] == '\t')) {
            p += 2;
            for (int c = 0; c < 3; ++c) nrm.push_back(parse_real(p));
        } else if (p[0] == 'v' && p[1] == 't' && (p[2] == ' ' || p[2] == '\t')) {
            p += 2;
            for (int c = 0; c < 2; ++c) tex.push_back(parse_real(p));
        } else if (p[0] == 'f' && sp1) {
            p += 1;
            std::vector<VRef> fc;
            bool ok = true;
            for (;;) {
                p += strspn(p, " \t");
                if (*p == '\0' || *p == '\r' || *p == '\n') break;
                VRef r{0, -1, -1};
                const int nv = (int)pos.size() / 3, nt = (int)tex.size() / 2, nn = (int)nrm.size() / 3;
                r.v = fix_index(atoi(p), nv, ok);
                p += strcspn(p, "/ \t\r");
                if (*p == '/') {
                    ++p;
                    if (*p != '/') {
                        r.vt = fix_index(atoi(p), nt, ok);
                        p += strcspn(p, "/ \t\r");
                    }
                    if (*p == '/') {
                        ++p;
                        r.vn = fix_index(atoi(p), nn, ok);
                        p += strcspn(p, " \t\r");
                    }
                }
                if (r.v < 0 || r.v >= nv) ok = false;
                fc.push_back(r);
            }
            if (!ok) {
                m_error = "[Scene] failed to load " + filepath + " : invalid face index";
                return false;
            }
            faces.push_back(fc);
        } else if (!strncmp(p, "usemtl", 6) && (p[6] == ' ' || p[6] == '\t')) {
            const std::string name = trim(p + 7);
            auto it = mat_ids.find(name);
            const int id = it == mat_ids.end() ? -1 : it->second;
            if (it == mat_ids.end()) warn += "material [" + name + "] not found\n";
            if (id != material) {
                export_group();
                material = id;
            }
        } else if (!strncmp(p, "mtllib", 6) && (p[6] == ' ' || p[6] == '\t')) {
            std::istringstream ss(p + 7);
            std::string fn;
            while (ss >> fn) {
                if (load_mtl(dir + fn, mats, mat_ids, warn)) break;
            }
        } else if ((p[0] == 'o' || p[0] == 'g') && (sp1 || p[1] == '\0' || p[1] == '\r')) {
            flush_shape();
            cur.name = p[1] == '\0' ? std::string() : trim(p + 2);
        }
    }
    flush_shape();

    // Src/scene.cpp:69-71, 9-29: one Lambert(Kd) per MTL material, nullptr for "no_surface"
    std::vector<Material*> matptr;
    for (const auto& m : mats) {
        if (m.unknown.count("no_surface") == 1) {
            matptr.push_back(nullptr);
        } else {
            matptr.push_back(ownMaterial(std::make_unique<Lambert>(Vec3f(m.diffuse[0], m.diffuse[1], m.diffuse[2]))));
        }
    }
    // Src/scene.cpp:73-153
    for (const auto& sh : shapes) {
        int materialID = -1;
        std::vector<Primitive> prims;
        for (size_t t = 0; t < sh.material.size(); ++t) {
            std::vector<Vec3f> vs, ns;
            std::vector<Vec2f> ts;
            for (int k = 0; k < 3; ++k) {
                const VRef& r = sh.idx[3 * t + k];
                vs.push_back(Vec3f(pos[3 * (size_t)r.v], pos[3 * (size_t)r.v + 1], pos[3 * (size_t)r.v + 2]));
                if (r.vn >= 0) ns.push_back(Vec3f(nrm[3 * (size_t)r.vn], nrm[3 * (size_t)r.vn + 1], nrm[3 * (size_t)r.vn + 2]));
                if (r.vt >= 0) ts.push_back(Vec2f(tex[2 * (size_t)r.vt], tex[2 * (size_t)r.vt + 1]));
            }
            if (ns.empty()) {
                const Vec3f n = normalize(cross(vs[1] - vs[0], vs[2] - vs[0]));
                ns = {n, n, n};
            }
            if (ts.empty()) ts = {Vec2f(0, 0), Vec2f(1, 0), Vec2f(0, 1)};
            const int mID = sh.material[t];
            if (materialID != mID && materialID == -1) materialID = mID;
            prims.emplace_back(vs, ns, ts);
        }
        // m_material[-1] is undefined behaviour in the reference (an OBJ without materials,
        // e.g. testdata/sphere32.obj); here the mesh gets no material.
        Material* mp = (materialID >= 0 && materialID < (int)matptr.size()) ? matptr[materialID] : nullptr;
        m_objects[sh.name] = std::make_unique<Mesh>(std::move(prims), mp, nullptr);
        ++m_version;
    }
    (void)warn;
    return true;
}

Material* Scene::ownMaterial(std::unique_ptr<Material> m) {
    m_material.push_back(std::move(m));
    return m_material.back().get();
}

void Scene::addObj(std::string name, std::unique_ptr<Object> obj) {
    m_objects[name] = std::move(obj);
    ++m_version;
}

Scene::~Scene() {
    if (m_qctx) xrt_destroy(m_qctx);
}

// Scene::sampleAreaLight (Src/scene.cpp:182-188)
const AreaLight* Scene::sampleAreaLight(Sampler& sampler, float& pdf) const {
    unsigned int lightIdx = m_areaLights.size() * sampler.getNext1D();
    if (lightIdx == m_areaLights.size()) lightIdx--;
    pdf = 1.0f / m_areaLights.size();
    return m_areaLights[lightIdx].get();
}

void Scene::setQueryDevice(int device) {
    if (device == m_qdevice) return;
    if (m_qctx) xrt_destroy(m_qctx);
    m_qctx = nullptr;
    m_qversion = ~0ull;
    m_qdevice = device;
}

// GPU ray queries (xrt_query): upload on first use and after any change to the objects
bool Scene::query(const float* rays, const float* tmax, uint32_t n, int mode, xrt_hit* out) const {
    int rc = XRT_OK;
    if (!m_qctx && (rc = xrt_create(m_qdevice, &m_qctx)) != XRT_OK) {
        m_qctx = nullptr;
        m_error = std::string("[Scene] ray query: xrt_create failed: ") + xrt_last_error(nullptr);
        return false;
    }
    if (m_qversion != m_version) {
        xrt_scene_desc desc;
        if ((rc = flatten(&desc)) != XRT_OK || (rc = xrt_upload_scene(m_qctx, &desc)) != XRT_OK) {
            m_error = std::string("[Scene] ray query: upload failed: ") + xrt_last_error(m_qctx);
            return false;
        }
        m_order.clear();
        for (const auto& kv : m_objects) m_order.push_back(kv.second.get());   // flatten's order
        m_qversion = m_version;
    }
    if ((rc = xrt_query(m_qctx, n, rays, tmax, mode, out)) != XRT_OK) {
        m_error = std::string("[Scene] ray query failed: ") + xrt_last_error(m_qctx);
        return false;
    }
    return true;
}

void Scene::fillInfo(const xrt_hit& h, IntersectInfo& info) const {
    if (h.object < 0) return;   // nothing wrote the fresh IntersectInfo
    info.t = h.t;
    info.t1 = h.t1;
    SurfaceInfo& s = info.surfaceInfo;
    s.position = Vec3f(h.position[0], h.position[1], h.position[2]);
    s.ng = Vec3f(h.ng[0], h.ng[1], h.ng[2]);
    s.ns = Vec3f(h.ns[0], h.ns[1], h.ns[2]);
    s.dpdu = Vec3f(h.dpdu[0], h.dpdu[1], h.dpdu[2]);
    s.dpdv = Vec3f(h.dpdv[0], h.dpdv[1], h.dpdv[2]);
    info.hitObject = (size_t)h.object < m_order.size() ? m_order[h.object] : nullptr;
    if (h.primitive >= 0) {
        const float u = h.barycentric[0], v = h.barycentric[1];
        s.barycentric = Vec2f(u, v);
        // texcoords[0] * (1 - u - v) + texcoords[1] * u + texcoords[2] * v (Src/primitive.cpp:104)
        const Mesh* mesh = dynamic_cast<const Mesh*>(info.hitObject);
        if (mesh && (size_t)h.primitive < mesh->primitives().size()) {
            const std::vector<Vec2f>& tc = mesh->primitives()[h.primitive].texcoords();
            if (tc.size() >= 3) {
                const float w = 1.0f - u - v;
                s.texcoords = Vec2f(tc[0][0] * w + tc[1][0] * u + tc[2][0] * v, tc[0][1] * w + tc[1][1] * u + tc[2][1] * v);
            }
        }
    }
}

bool Scene::intersect(const Ray& ray, IntersectInfo& info) const {
    const float r[6] = {ray.origin[0], ray.origin[1], ray.origin[2], ray.direction[0], ray.direction[1], ray.direction[2]};
    xrt_hit h;
    if (!query(r, nullptr, 1, XRT_QUERY_INTERSECT, &h)) return false;
    fillInfo(h, info);
    return h.hit != 0;
}

bool Scene::occluded(const Ray& ray, float t_max) const {
    const float r[6] = {ray.origin[0], ray.origin[1], ray.origin[2], ray.direction[0], ray.direction[1], ray.direction[2]};
    xrt_hit h;
    return query(r, &t_max, 1, XRT_QUERY_OCCLUDED, &h) && h.hit != 0;
}

void Scene::intersect(const std::vector<Ray>& rays, std::vector<IntersectInfo>& infos, std::vector<char>& hits) const {
    const size_t n = rays.size();
    std::vector<float> r(6 * n);
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) r[6 * i + k] = rays[i].origin[k], r[6 * i + 3 + k] = rays[i].direction[k];
    std::vector<xrt_hit> h(n);
    infos.assign(n, IntersectInfo());
    hits.assign(n, 0);
    if (n == 0 || !query(r.data(), nullptr, (uint32_t)n, XRT_QUERY_INTERSECT, h.data())) return;
    for (size_t i = 0; i < n; ++i) {
        fillInfo(h[i], infos[i]);
        hits[i] = h[i].hit != 0;
    }
}

void Scene::occluded(const std::vector<Ray>& rays, const std::vector<float>& t_max, std::vector<char>& hits) const {
    const size_t n = rays.size();
    std::vector<float> r(6 * n);
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) r[6 * i + k] = rays[i].origin[k], r[6 * i + 3 + k] = rays[i].direction[k];
    std::vector<xrt_hit> h(n);
    hits.assign(n, 0);
    if (n == 0 || t_max.size() < n || !query(r.data(), t_max.data(), (uint32_t)n, XRT_QUERY_OCCLUDED, h.data())) return;
    for (size_t i = 0; i < n; ++i) hits[i] = h[i].hit != 0;
}

void Scene::addAreaLight(std::string name, std::unique_ptr<AreaLight> light) {
    addObj(name, light->makeObject());  // Src/scene.cpp:166-170
    m_areaLights.push_back(std::move(light));
}

int Scene::objectIndex(const Object* obj) const {
    int i = 0;
    for (const auto& kv : m_objects) {
        if (kv.second.get() == obj) return i;
        ++i;
    }
    return -1;
}

std::vector<std::string> Scene::objectNames() const {
    std::vector<std::string> n;
    for (const auto& kv : m_objects) n.push_back(kv.first);
    return n;
}

const Medium* Scene::anyMedium() const {
    for (const auto& kv : m_objects)
        if (kv.second->medium()) return kv.second->medium();
    return nullptr;
}

const HeterogeneousMedium* Scene::medium() const { return dynamic_cast<const HeterogeneousMedium*>(anyMedium()); }

static void put3(float* d, const Vec3f& v) {
    d[0] = v[0];
    d[1] = v[1];
    d[2] = v[2];
}

int Scene::flatten(xrt_scene_desc* out) const {
    f_objects.clear();
    f_triv.clear();
    f_trin.clear();
    f_sph.clear();
    f_box.clear();
    f_lights.clear();
    const Medium* the_medium = nullptr;
    for (const auto& l : m_areaLights) {
        xrt_light d;
        std::memset(&d, 0, sizeof(d));
        put3(d.Le, l->Le());
        if (auto* q = dynamic_cast<const QuadLight*>(l.get())) {
            d.kind = XRT_LIGHT_QUAD;
            put3(d.v0, q->v0()), put3(d.v1, q->v1()), put3(d.v2, q->v2());
        } else if (auto* t = dynamic_cast<const TriangleLight*>(l.get())) {
            d.kind = XRT_LIGHT_TRIANGLE;
            put3(d.v0, t->v0()), put3(d.v1, t->v1()), put3(d.v2, t->v2());
        } else if (auto* s = dynamic_cast<const SphereLight*>(l.get())) {
            d.kind = s->sampling() == SphereLight::Sampling::Area ? XRT_LIGHT_SPHERE_AREA : XRT_LIGHT_SPHERE;
            put3(d.center, s->center());
            d.radius = s->radius();
        } else {
            return XRT_ERR_UNSUPPORTED;
        }
        f_lights.push_back(d);
    }
    for (const auto& kv : m_objects) {  // Scene::m_objects iteration order
        const Object* ob = kv.second.get();
        xrt_object d;
        std::memset(&d, 0, sizeof(d));
        d.light = -1;
        d.medium = -1;
        if (const auto* lam = dynamic_cast<const Lambert*>(ob->material())) {
            d.material = XRT_MAT_LAMBERT;
            put3(d.albedo, lam->albedo());
        } else if (ob->material()) {
            return XRT_ERR_UNSUPPORTED;
        }
        if (ob->areaLight()) {
            for (size_t i = 0; i < m_areaLights.size(); ++i)
                if (m_areaLights[i].get() == ob->areaLight()) d.light = (int32_t)i;
            if (d.light < 0) return XRT_ERR_INVALID;  // light object without its light
        }
        if (ob->medium()) {
            if (the_medium && the_medium != ob->medium()) return XRT_ERR_UNSUPPORTED;
            the_medium = ob->medium();
            d.medium = 0;
        }
        if (const auto* m = dynamic_cast<const Mesh*>(ob)) {
            d.kind = XRT_OBJ_MESH;
            d.first = (int32_t)(f_triv.size() / 9);
            for (const auto& p : m->primitives()) {
                if (p.vertices().size() < 3 || p.normals().size() < 3) return XRT_ERR_INVALID;
                for (int k = 0; k < 3; ++k) {
                    for (int c = 0; c < 3; ++c) f_triv.push_back(p.vertices()[k][c]);
                    for (int c = 0; c < 3; ++c) f_trin.push_back(p.normals()[k][c]);
                }
            }
            d.count = (int32_t)(f_triv.size() / 9) - d.first;
        } else if (const auto* s = dynamic_cast<const Sphere*>(ob)) {
            d.kind = XRT_OBJ_SPHERE;
            d.first = (int32_t)(f_sph.size() / 4);
            d.count = 1;
            for (int c = 0; c < 3; ++c) f_sph.push_back(s->center()[c]);
            f_sph.push_back(s->radius());
        } else if (const auto* b = dynamic_cast<const BoxMesh*>(ob)) {
            d.kind = XRT_OBJ_BOX;
            d.first = (int32_t)(f_box.size() / 6);
            d.count = 1;
            for (int c = 0; c < 3; ++c) f_box.push_back(b->box().pMin[c]);
            for (int c = 0; c < 3; ++c) f_box.push_back(b->box().pMax[c]);
        } else {
            return XRT_ERR_UNSUPPORTED;
        }
        f_objects.push_back(d);
    }
    out->n_objects = (uint32_t)f_objects.size();
    out->objects = f_objects.data();
    out->n_tris = (uint32_t)(f_triv.size() / 9);
    out->tri_v = f_triv.data();
    out->tri_n = f_trin.data();
    out->n_spheres = (uint32_t)(f_sph.size() / 4);
    out->spheres = f_sph.data();
    out->n_boxes = (uint32_t)(f_box.size() / 6);
    out->boxes = f_box.data();
    out->n_lights = (uint32_t)f_lights.size();
    out->lights = f_lights.data();
    return XRT_OK;
}
