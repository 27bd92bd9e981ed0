// ref_kats.cpp — known-answer vectors from the REFERENCE's own code, compiled in place.
//
// TEST INFRASTRUCTURE ONLY.  Built by `make -C oracle ref` from
//   /root/reference/Src/geometry.cpp, /root/reference/Src/sampler.cpp and this driver,
// which includes the reference headers geometry.h, sampler.h, ray.h, primitive.h,
// material.h and medium.h unmodified (-I /root/reference/Src).  Only the compile
// definitions of Src/cmakelists.txt:57-65 (kEpsilon, kInfinity) and `-include cfloat`
// (for FLT_EPSILON / FLT_MAX, which the MSVC headers of the original build make visible
// transitively) are added.  No reference source is copied; no stand-in headers are used.
// Translation units that need spdlog / OpenCV / OpenVDB / tinyobjloader (camera.h,
// light.*, primitive.cpp, scene.*, integrator.h, renderer.*, medium.cpp, grid.h) are
// NOT buildable here and are not used.
//
// Output: one JSON object on stdout; every float is emitted as its uint32 bit pattern.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "geometry.h"
#include "material.h"
#include "medium.h"
#include "primitive.h"
#include "ray.h"
#include "sampler.h"

namespace {

uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// deterministic input generator (xorshift32) — inputs are emitted with the outputs
struct Gen {
    uint32_t s;
    explicit Gen(uint32_t seed) : s(seed) {}
    uint32_t next() {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        return s;
    }
    float uni(float a, float b) { return a + (b - a) * (float)(next() >> 8) * (1.0f / 16777216.0f); }
    Vec3f vec(float a, float b) {
        float x = uni(a, b), y = uni(a, b), z = uni(a, b);
        return Vec3f(x, y, z);
    }
};

struct Out {
    std::string s;
    bool first = true;
    void key(const char* k) {
        s += first ? "" : ",\n";
        first = false;
        s += "\"";
        s += k;
        s += "\": ";
    }
    void arr(const std::vector<uint32_t>& v) {
        s += "[";
        for (size_t i = 0; i < v.size(); ++i) {
            if (i) s += ",";
            s += std::to_string(v[i]);
        }
        s += "]";
    }
};

void push3(std::vector<uint32_t>& v, const Vec3f& a) {
    v.push_back(bits(a[0]));
    v.push_back(bits(a[1]));
    v.push_back(bits(a[2]));
}

}  // namespace

int main() {
    Out o;
    o.s = "{\n";

    // 1. UniformSampler streams (Src/sampler.h:37-50, 25): seeds and 2000 draws each,
    //    plus draws 100000..100099 of seed 7 (several twists deep).
    {
        const uint32_t seeds[] = {0u, 1u, 255u, 65535u, 479999u, 2073599u, 4294967295u};
        std::vector<uint32_t> sv, dv;
        for (uint32_t sd : seeds) {
            UniformSampler smp;
            smp.setSeed(sd);
            sv.push_back(sd);
            for (int k = 0; k < 2000; ++k) dv.push_back(bits(smp.getNext1D()));
        }
        o.key("rng_seeds"); o.arr(sv);
        o.key("rng_draws_2000"); o.arr(dv);
        UniformSampler smp;
        smp.setSeed(7);
        for (int k = 0; k < 100000; ++k) smp.getNext1D();
        std::vector<uint32_t> deep;
        for (int k = 0; k < 100; ++k) deep.push_back(bits(smp.getNext1D()));
        o.key("rng_seed7_skip100000"); o.arr(deep);
        // getNext2D order (Src/sampler.h:49): Vec2f(dis(gen), dis(gen))
        UniformSampler s2;
        s2.setSeed(12345);
        std::vector<uint32_t> v2;
        for (int k = 0; k < 64; ++k) {
            Vec2f u = s2.getNext2D();
            v2.push_back(bits(u[0]));
            v2.push_back(bits(u[1]));
        }
        o.key("rng_seed12345_next2d"); o.arr(v2);
    }

    // 2. normalize + orthonormalBasis (Src/geometry.cpp:13-16, 43-49)
    {
        Gen g(0x1234567u);
        std::vector<uint32_t> in, nrm, t, b;
        for (int k = 0; k < 512; ++k) {
            Vec3f v = g.vec(-3.0f, 3.0f);
            if (k % 7 == 0) v[2] = 0.0f;  // copysign(1, +0) branch
            push3(in, v);
            Vec3f n = normalize(v);
            push3(nrm, n);
            Vec3f tt, bb;
            orthonormalBasis(n, tt, bb);
            push3(t, tt);
            push3(b, bb);
        }
        o.key("onb_in"); o.arr(in);
        o.key("onb_normalized"); o.arr(nrm);
        o.key("onb_t"); o.arr(t);
        o.key("onb_b"); o.arr(b);
    }

    // 3. Lambert::sampleDir (Src/material.h:55-73) — SurfaceInfo with ng and the ONB of ng
    {
        Gen g(0xBADC0DEu);
        Lambert lam(Vec3f(0.5f, 0.25f, 1.0f));
        UniformSampler smp;
        smp.setSeed(2024);
        std::vector<uint32_t> in, wi, pdfs;
        for (int k = 0; k < 512; ++k) {
            SurfaceInfo si;
            si.ng = normalize(g.vec(-1.0f, 1.0f));
            orthonormalBasis(si.ng, si.dpdu, si.dpdv);
            push3(in, si.ng);
            push3(in, si.dpdu);
            push3(in, si.dpdv);
            float pdf = 0.0f;
            Vec3f w = lam.sampleDir(si, smp, pdf);
            push3(wi, w);
            pdfs.push_back(bits(pdf));
        }
        o.key("lambert_seed"); o.arr({2024u});
        o.key("lambert_in"); o.arr(in);
        o.key("lambert_wi"); o.arr(wi);
        o.key("lambert_pdf"); o.arr(pdfs);
    }

    // 4. Sphere::intersect / occluded (Src/primitive.h:106-156): rays aimed near spheres
    {
        Gen g(0x5EEDu);
        std::vector<uint32_t> in, hit, out, occ;
        for (int k = 0; k < 1024; ++k) {
            Vec3f c = g.vec(-20.0f, 20.0f);
            float r = g.uni(0.1f, 5.0f);
            Vec3f orig = g.vec(-30.0f, 30.0f);
            if (k % 5 == 0) orig = c + g.vec(-0.5f, 0.5f) * r;  // start inside
            Vec3f target = c + g.vec(-1.5f, 1.5f) * r;
            Vec3f dir = normalize(target - orig);
            if (k % 3 == 0) dir = dir * g.uni(0.5f, 2.0f);     // non-unit direction
            float tmax = g.uni(0.0f, 60.0f);
            push3(in, orig);
            push3(in, dir);
            push3(in, c);
            in.push_back(bits(r));
            in.push_back(bits(tmax));
            Sphere sp(c, r, nullptr, nullptr);
            Ray ray(orig, dir);
            IntersectInfo info;
            bool h = sp.intersect(ray, info);
            hit.push_back(h ? 1u : 0u);
            out.push_back(bits(info.t));
            push3(out, info.surfaceInfo.position);
            push3(out, info.surfaceInfo.ng);
            occ.push_back(sp.occluded(ray, tmax) ? 1u : 0u);
        }
        o.key("sphere_in"); o.arr(in);
        o.key("sphere_hit"); o.arr(hit);
        o.key("sphere_out"); o.arr(out);
        o.key("sphere_occluded"); o.arr(occ);
    }

    // 5. BoxMesh::intersect (Src/primitive.h:243-264)
    {
        Gen g(0xB0B0u);
        std::vector<uint32_t> in, hit, out;
        for (int k = 0; k < 1024; ++k) {
            Vec3f a = g.vec(-10.0f, 10.0f), b = g.vec(-10.0f, 10.0f);
            AABB box{vmin(a, b), vmax(a, b)};
            Vec3f orig = g.vec(-20.0f, 20.0f);
            Vec3f dir = normalize(g.vec(-1.0f, 1.0f));
            if (k % 9 == 0) dir[k % 3] = 0.0f;  // axis-parallel: 1/0 = inf slabs
            push3(in, orig);
            push3(in, dir);
            push3(in, box.pMin);
            push3(in, box.pMax);
            BoxMesh bm(box, nullptr);
            IntersectInfo info;
            bool h = bm.intersect(Ray(orig, dir), info);
            hit.push_back(h ? 1u : 0u);
            out.push_back(bits(info.t));
            out.push_back(bits(info.t1));
        }
        o.key("box_in"); o.arr(in);
        o.key("box_hit"); o.arr(hit);
        o.key("box_out"); o.arr(out);
    }

    // 6. HenyeyGreenstein::sampleDirection / evaluate (Src/medium.h:21-68)
    {
        const float gs[] = {0.0f, 0.0005f, 0.5f, -0.3f, 0.85f};
        Gen g(0x4E4Eu);
        std::vector<uint32_t> gv, in, wi, val;
        for (float gg : gs) {
            HenyeyGreenstein hg(gg);
            UniformSampler smp;
            smp.setSeed(99);
            gv.push_back(bits(gg));
            for (int k = 0; k < 256; ++k) {
                Vec3f wo = normalize(g.vec(-1.0f, 1.0f));
                push3(in, wo);
                Vec3f w;
                float v = hg.sampleDirection(wo, smp, w);
                push3(wi, w);
                val.push_back(bits(v));
            }
        }
        o.key("hg_g"); o.arr(gv);
        o.key("hg_seed"); o.arr({99u});
        o.key("hg_wo"); o.arr(in);
        o.key("hg_wi"); o.arr(wi);
        o.key("hg_eval"); o.arr(val);
    }

    // 7. Medium::sampleWavelength (Src/medium.h:102-115) + DiscreteEmpiricalDistribution1D
    {
        Gen g(0xC0C0u);
        UniformSampler smp;
        smp.setSeed(4242);
        std::vector<uint32_t> in, ch, pmf;
        for (int k = 0; k < 1024; ++k) {
            Vec3f thr = g.vec(0.0f, 2.0f), alb = g.vec(0.0f, 1.0f);
            if (k % 11 == 0) thr[k % 3] = 0.0f;
            push3(in, thr);
            push3(in, alb);
            Vec3f p;
            ch.push_back(Medium::sampleWavelength(thr, alb, smp, p));
            push3(pmf, p);
        }
        o.key("wl_seed"); o.arr({4242u});
        o.key("wl_in"); o.arr(in);
        o.key("wl_channel"); o.arr(ch);
        o.key("wl_pmf"); o.arr(pmf);
    }

    // 8. The pinhole camera's ray direction, PinholeCamera::sampleRay's expression
    //    (Src/camera.h:52-55) evaluated with the reference's own Matrix44f, multDirMatrix
    //    (geometry.h:653-669) and normalize (geometry.cpp:13-16): camera.h itself includes
    //    spdlog and is not buildable here, so only its one-line expression is repeated.
    //    Cameras: the Cornell c2w (Src/examples/cornellbox.cpp:29), the C3/C5 translations,
    //    and random rotation-like matrices.  Also Matrix44f::multDirMatrix (member).
    {
        Gen g(0xCA3E4Au);
        std::vector<uint32_t> mats, in, dirs, mem;
        std::vector<Matrix44f> ms = {Matrix44f(-1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, -1.0, 0, 278, 274.4, -750.0, 1),
                                     Matrix44f(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 4, 8, 1),
                                     Matrix44f(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 63.5f, 63.5f, 345.1f, 1)};
        for (int k = 0; k < 5; ++k) {
            Matrix44f m;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) m[r][c] = g.uni(-1.0f, 1.0f);
            for (int c = 0; c < 3; ++c) m[3][c] = g.uni(-500.0f, 500.0f);
            ms.push_back(m);
        }
        const float scales[] = {0.57735026f, 0.41421357f, 1.0f};
        const float aspects[] = {4.0f / 3.0f, 16.0f / 9.0f, 1.0f};
        int mi = 0;
        for (const Matrix44f& m : ms) {
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) mats.push_back(bits(m[r][c]));
            for (int k = 0; k < 128; ++k) {
                const float u = g.uni(0.0f, 1.0f), v = g.uni(0.0f, 1.0f);
                const float scale = scales[(mi + k) % 3], aspect = aspects[(mi + 2 * k) % 3];
                in.push_back(bits(u));
                in.push_back(bits(v));
                in.push_back(bits(scale));
                in.push_back(bits(aspect));
                const Vec3f dir((2 * u - 1) * scale, (1 - 2 * v) * scale / aspect, -1);
                push3(dirs, normalize(multDirMatrix(dir, m)));
                Vec3f dm;
                m.multDirMatrix(dir, dm);
                push3(mem, dm);
            }
            ++mi;
        }
        o.key("cam_c2w"); o.arr(mats);
        o.key("cam_in"); o.arr(in);
        o.key("cam_dir"); o.arr(dirs);
        o.key("cam_multdir_member"); o.arr(mem);
    }

    // 9. Lambert::evaluateBxDF and sampleBxDF (Src/material.h:39-53): the BSDF value
    //    albedo / PI and the sampled direction + pdf through the Material interface
    {
        Gen g(0x1A3B5u);
        UniformSampler smp;
        smp.setSeed(777);
        std::vector<uint32_t> in, f, wi, pdfs, ev;
        for (int k = 0; k < 256; ++k) {
            const Vec3f albedo = g.vec(0.0f, 1.0f);
            SurfaceInfo si;
            si.ng = normalize(g.vec(-1.0f, 1.0f));
            orthonormalBasis(si.ng, si.dpdu, si.dpdv);
            const Vec3f wo = normalize(g.vec(-1.0f, 1.0f));
            push3(in, albedo);
            push3(in, si.ng);
            push3(in, si.dpdu);
            push3(in, si.dpdv);
            push3(in, wo);
            Lambert lam(albedo);
            const Material& mat = lam;
            Vec3f w;
            float pdf = 0.0f;
            push3(f, mat.sampleBxDF(wo, si, smp, w, pdf));
            push3(wi, w);
            pdfs.push_back(bits(pdf));
            push3(ev, mat.evaluateBxDF(wo, w, si));
        }
        o.key("bxdf_seed"); o.arr({777u});
        o.key("bxdf_in"); o.arr(in);
        o.key("bxdf_f"); o.arr(f);
        o.key("bxdf_wi"); o.arr(wi);
        o.key("bxdf_pdf"); o.arr(pdfs);
        o.key("bxdf_eval"); o.arr(ev);
    }

    // 10. Host-side geometry of the drop-in API (include/xrt/geometry.h): Matrix44f::inverse
    //     (Gauss-Jordan, Src/geometry.h:509-590), operator* and transposed (:314-425) on the
    //     cameras above, random affine and random dense matrices and one singular matrix;
    //     worldToLocal / localToWorld (:686-701) in frames from orthonormalBasis.
    {
        Gen g(0xC0FFEEu);
        std::vector<Matrix44f> ms = {Matrix44f(-1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, -1.0, 0, 278, 274.4, -750.0, 1),
                                     Matrix44f(1, 2, 3, 4, 2, 4, 6, 8, 0, 1, 0, 0, 0, 0, 1, 1)};   // singular
        for (int k = 0; k < 40; ++k) {
            Matrix44f m;
            const bool affine = k < 20;
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) m[i][j] = (affine && j == 3) ? (i == 3 ? 1.0f : 0.0f) : g.uni(-2.0f, 2.0f);
            if (affine)
                for (int j = 0; j < 3; ++j) m[3][j] = g.uni(-500.0f, 500.0f);
            ms.push_back(m);
        }
        std::vector<uint32_t> mats, inv, prod, tr;
        for (size_t q = 0; q < ms.size(); ++q) {
            const Matrix44f& m = ms[q];
            const Matrix44f& n = ms[(q + 1) % ms.size()];
            const Matrix44f mi = m.inverse(), mn = m * n, mt = m.transposed();
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    mats.push_back(bits(m[i][j]));
                    inv.push_back(bits(mi[i][j]));
                    prod.push_back(bits(mn[i][j]));
                    tr.push_back(bits(mt[i][j]));
                }
        }
        o.key("m44_in"); o.arr(mats);
        o.key("m44_inverse"); o.arr(inv);
        o.key("m44_mul_next"); o.arr(prod);
        o.key("m44_transposed"); o.arr(tr);
        std::vector<uint32_t> in, w2l, l2w;
        for (int k = 0; k < 256; ++k) {
            const Vec3f n = normalize(g.vec(-1.0f, 1.0f));
            Vec3f t, b;
            orthonormalBasis(n, t, b);
            const Vec3f v = g.vec(-3.0f, 3.0f);
            push3(in, v);
            push3(in, t);
            push3(in, n);
            push3(in, b);
            push3(w2l, worldToLocal(v, t, n, b));
            push3(l2w, localToWorld(v, t, n, b));
        }
        o.key("frame_in"); o.arr(in);
        o.key("frame_w2l"); o.arr(w2l);
        o.key("frame_l2w"); o.arr(l2w);
    }

    // 11. SphereLight::sample built with AREA_SAMPLING (Src/light.h:131-135,185-191) and its
    //     UniformSampleSphere (Src/light.cpp:99-105): light.h includes spdlog and is not
    //     buildable here, so the sampling expression is repeated with the reference's own
    //     Vec3f, length/dot and UniformSampler — and, to pin GCC's draw order, the call keeps
    //     its shape: a const member taking (const float& r1, const float& r2), called with two
    //     getNext1D() operands.
    {
        struct AreaProbe {
            Vec3f center;
            float radius;
            Vec3f dirOnSphere(const float& r1, const float& r2) const {
                float z = 1.f - 2.f * r1;
                float sin_theta = std::sqrt(1 - z * z);
                float phi = 2 * PI * r2;
                return {std::cos(phi) * sin_theta, std::sin(phi) * sin_theta, z};
            }
            Vec3f sample(const Vec3f& position, Vec3f& wi, float& pdf, float& tmax, Sampler& s) const {
                Vec3f n = dirOnSphere(s.getNext1D(), s.getNext1D());
                Vec3f p = center + n * radius;
                Vec3f d = p - position;
                tmax = length(d);
                float d_dot_n = dot(d, n);
                if (d_dot_n >= 0) return Vec3f(0.0f);
                wi = d / tmax;
                pdf = (2.f * tmax * tmax * tmax) / std::abs(d_dot_n);
                return Vec3f(1.0f);
            }
        };
        Gen g(0xA2EAu);
        UniformSampler smp;
        smp.setSeed(31337);
        std::vector<uint32_t> in, out;
        for (int k = 0; k < 512; ++k) {
            AreaProbe L{g.vec(-20.0f, 20.0f), g.uni(0.2f, 6.0f)};
            Vec3f pos = g.vec(-30.0f, 30.0f);
            push3(in, L.center);
            in.push_back(bits(L.radius));
            push3(in, pos);
            Vec3f wi(0.0f);
            float pdf = 0.0f, tmax = 0.0f;
            Vec3f le = L.sample(pos, wi, pdf, tmax, smp);
            push3(out, wi);
            out.push_back(bits(pdf));
            out.push_back(bits(tmax));
            out.push_back(le[0] != 0.0f ? 1u : 0u);
        }
        o.key("sphere_area_seed"); o.arr({31337u});
        o.key("sphere_area_in"); o.arr(in);
        o.key("sphere_area_out"); o.arr(out);
    }

    o.s += "\n}\n";
    std::fputs(o.s.c_str(), stdout);
    return 0;
}
