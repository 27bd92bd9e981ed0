/*
 * oracle.c — CPU restatement of xRayTracer's path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Every function cites the reference
 * file:line it restates.  Floating-point evaluation follows the reference as compiled by
 * GCC 11 on x86-64 (SSE, no FMA contraction: build with -ffp-contract=off):
 *   - Vec3 operators evaluate component-wise, left to right (Src/geometry.h:174-261);
 *   - unqualified sqrt(float) in primitive.h resolves to ::sqrt(double) (probe in
 *     oracle/Makefile `overloads` target), std::sqrt/cos/sin/log/exp(float) to the float
 *     libm functions;
 *   - GCC evaluates call arguments right to left, which fixes the draw order of
 *     QuadLight::sample (light.cpp:61), TriangleLight::sample (light.cpp:23) and
 *     getNext2D (sampler.h:49).
 * Transcendentals come from the host glibc libm, exactly as the reference gets them.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- constants ---- */
/* Src/geometry.h:10-23 */
#define PI_F ((float)3.14159265359)
static const float PI_MUL_2 = 2.0f * (float)3.14159265359;
static const float PI_MUL_4_INV = 1.0f / (4.0f * (float)3.14159265359);
#define RAY_EPS 1e-3f
#define K_EPS FLT_EPSILON  /* kEpsilon = FLT_EPSILON (Src/cmakelists.txt:57-65) */
#define K_INF FLT_MAX      /* kInfinity = FLT_MAX */

/* ---------------------------------------------------------------- mt19937 ---- */
/* libstdc++ mersenne_twister_engine<uint_fast32_t, 32, 624, 397, 31, 0x9908b0df, 11,
 * 0xffffffff, 7, 0x9d2c5680, 15, 0xefc60000, 18, 1812433253>::seed / _M_gen_rand /
 * operator() — the engine behind Sampler::gen (Src/sampler.h:16, 25). */
void orc_mt_seed(orc_mt* m, uint32_t seed) {
    m->x[0] = seed;
    for (uint32_t i = 1; i < 624; ++i)
        m->x[i] = 1812433253u * (m->x[i - 1] ^ (m->x[i - 1] >> 30)) + i;
    m->p = 624;
    m->draws = 0;
}

static void mt_twist(orc_mt* m) {
    const uint32_t up = 0x80000000u, lo = 0x7fffffffu;
    uint32_t k;
    for (k = 0; k < 227; ++k) {
        uint32_t y = (m->x[k] & up) | (m->x[k + 1] & lo);
        m->x[k] = m->x[k + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    for (; k < 623; ++k) {
        uint32_t y = (m->x[k] & up) | (m->x[k + 1] & lo);
        m->x[k] = m->x[k - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    uint32_t y = (m->x[623] & up) | (m->x[0] & lo);
    m->x[623] = m->x[396] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    m->p = 0;
}

uint32_t orc_mt_next(orc_mt* m) {
    if (m->p >= 624) mt_twist(m);
    uint32_t z = m->x[m->p++];
    z ^= (z >> 11);
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= (z >> 18);
    return z;
}

/* uniform_real_distribution<float>(0,1)(gen) = generate_canonical<float,24>(gen)*1+0:
 * (float)x / 2^32, and nextafter(1,0) if that rounds to 1. */
float orc_draw(orc_mt* m) {
    m->draws++;
    float f = (float)orc_mt_next(m) / 4294967296.0f;
    if (f >= 1.0f) f = nextafterf(1.0f, 0.0f);
    return f;
}

void orc_draws(uint32_t seed, uint32_t skip, uint32_t n, float* out) {
    orc_mt m;
    orc_mt_seed(&m, seed);
    for (uint32_t i = 0; i < skip; ++i) (void)orc_draw(&m);
    for (uint32_t i = 0; i < n; ++i) out[i] = orc_draw(&m);
}

/* ---------------------------------------------------------------- Vec3f ---- */
typedef struct { float x, y, z; } v3;
static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline void st3(float* p, v3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
static inline float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
/* Src/geometry.h:174-236 */
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vmuls(v3 a, float k) { return mk(a.x * k, a.y * k, a.z * k); }
static inline v3 vdivs(v3 a, float k) { return mk(a.x / k, a.y / k, a.z / k); }
static inline v3 vdivv(v3 a, v3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 vneg(v3 a) { return mk(-a.x, -a.y, -a.z); }
/* Src/geometry.h:250-261 */
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Src/geometry.cpp:3-16: length = std::sqrt(dot), normalize = v / length (3 divides) */
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
static inline v3 vnormalize(v3 a) { return vdivs(a, vlength(a)); }
/* std::min / std::max(a, b) = (b < a) ? b : a  /  (a < b) ? b : a */
static inline float smin(float a, float b) { return (b < a) ? b : a; }
static inline float smax(float a, float b) { return (a < b) ? b : a; }
/* Src/geometry.cpp:43-49 (the active #else branch) */
static void onb(v3 n, v3* t, v3* b) {
    float sign = copysignf(1.0f, n.z);
    const float a = -1.0f / (sign + n.z);
    const float c = n.x * n.y * a;
    *t = mk(1.0f + sign * n.x * n.x * a, sign * c, -sign * n.x);
    *b = mk(c, sign + n.y * n.y * a, -n.y);
}
/* Src/geometry.h:693-701 */
static inline v3 local_to_world(v3 v, v3 lx, v3 ly, v3 lz) {
    return mk(v.x * lx.x + v.y * ly.x + v.z * lz.x, v.x * lx.y + v.y * ly.y + v.z * lz.y,
              v.x * lx.z + v.y * ly.z + v.z * lz.z);
}
static inline v3 vexp(v3 a) { return mk(expf(a.x), expf(a.y), expf(a.z)); } /* geometry.cpp:18-21 */
static inline v3 ray_at(v3 o, v3 d, float t) { return vadd(o, vmuls(d, t)); } /* ray.h:20 */

/* ---------------------------------------------------------------- scene ---- */
typedef struct {
    float t1, t;
    v3 pos, ng, ns, dpdu, dpdv;
    int hit; /* object index, -1 = none (IntersectInfo::hitObject) */
    int prim; /* the triangle (within its mesh) that last wrote barycentric, -1 = none */
    float bu, bv; /* SurfaceInfo::barycentric */
} hinfo;

static inline void hinfo_init(hinfo* h) {
    memset(h, 0, sizeof(*h));
    h->t1 = K_INF;
    h->t = K_INF;
    h->hit = -1;
    h->prim = -1;
}

typedef struct {
    const xrt_scene_desc* S;
    const xrt_medium_desc* M;
    float majorant, inv_majorant; /* HeterogeneousMedium ctor (medium.cpp:12-16) */
} scene_ctx;

/* Mesh::rayTriangleIntersect, no CULLING (Src/primitive.cpp:140-168) */
static int ray_tri(v3 orig, v3 dir, v3 v0, v3 v1, v3 v2, float* t, float* u, float* v) {
    v3 v0v1 = vsub(v1, v0);
    v3 v0v2 = vsub(v2, v0);
    v3 pvec = vcross(dir, v0v2);
    float det = vdot(v0v1, pvec);
    if (fabsf(det) < K_EPS) return 0;
    float invDet = 1 / det;
    v3 tvec = vsub(orig, v0);
    *u = vdot(tvec, pvec) * invDet;
    if (*u < 0 || *u > 1) return 0;
    v3 qvec = vcross(tvec, v0v1);
    *v = vdot(dir, qvec) * invDet;
    if (*v < 0 || *u + *v > 1) return 0;
    *t = vdot(v0v2, qvec) * invDet;
    return *t > K_EPS;
}

static inline v3 tri_vert(const xrt_scene_desc* S, int tri, int k) { return ld3(S->tri_v + (size_t)tri * 9 + k * 3); }
static inline v3 tri_nrm(const xrt_scene_desc* S, int tri, int k) { return ld3(S->tri_n + (size_t)tri * 9 + k * 3); }

/* Mesh::intersect (Src/primitive.cpp:83-116) */
static int mesh_intersect(const xrt_scene_desc* S, int obj, v3 o, v3 d, hinfo* info, uint64_t* tests) {
    const xrt_object* ob = &S->objects[obj];
    int isect = 0;
    for (int i = ob->first; i < ob->first + ob->count; ++i) {
        float t = 0.0f, u = 0.0f, v = 0.0f;
        v3 a = tri_vert(S, i, 0), b = tri_vert(S, i, 1), c = tri_vert(S, i, 2);
        (*tests)++;
        if (ray_tri(o, d, a, b, c, &t, &u, &v)) {
            isect = 1;
            if (t < info->t) {
                info->t = t;
                info->pos = ray_at(o, d, t);
                info->ng = vnormalize(vcross(vsub(b, a), vsub(c, a)));
                float w = 1.0f - u - v;
                info->ns = vadd(vadd(vmuls(tri_nrm(S, i, 0), w), vmuls(tri_nrm(S, i, 1), u)),
                                vmuls(tri_nrm(S, i, 2), v));
                onb(info->ns, &info->dpdu, &info->dpdv);
                info->hit = obj;
                info->prim = i - ob->first, info->bu = u, info->bv = v;
            }
        }
    }
    return isect;
}

/* Mesh::occluded (Src/primitive.cpp:118-138) */
static int mesh_occluded(const xrt_scene_desc* S, int obj, v3 o, v3 d, float tmax, uint64_t* tests) {
    const xrt_object* ob = &S->objects[obj];
    for (int i = ob->first; i < ob->first + ob->count; ++i) {
        float t = 0.0f, u = 0.0f, v = 0.0f;
        (*tests)++;
        int rst = ray_tri(o, d, tri_vert(S, i, 0), tri_vert(S, i, 1), tri_vert(S, i, 2), &t, &u, &v);
        if (rst && t < tmax) return 1;
    }
    return 0;
}

/* Sphere::solveQuadratic (Src/primitive.h:161-177): the -0.5*(...) terms are double and
 * the unqualified sqrt(float) is ::sqrt(double). */
static int solve_quadratic(float a, float b, float c, float* x0, float* x1) {
    float discr = b * b - 4 * a * c;
    if (discr < 0) return 0;
    else if (discr == 0) {
        *x0 = *x1 = (float)(-0.5 * (double)b / (double)a);
    } else {
        float q = (b > 0) ? (float)(-0.5 * ((double)b + sqrt((double)discr)))
                          : (float)(-0.5 * ((double)b - sqrt((double)discr)));
        *x0 = q / a;
        *x1 = c / q;
    }
    return 1;
}

/* Sphere::doIntersect (Src/primitive.h:133-156) */
static int sphere_do_intersect(v3 orig, v3 dir, v3 center, float r2, float* tnear) {
    float t0, t1;
    v3 L = vsub(orig, center);
    float a = vdot(dir, dir);
    float b = 2 * vdot(dir, L);
    float c = vdot(L, L) - r2;
    if (!solve_quadratic(a, b, c, &t0, &t1)) return 0;
    if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
    if (t0 < 0) {
        t0 = t1;
        if (t0 < 0) return 0;
    }
    *tnear = t0;
    return 1;
}

/* Sphere::intersect (Src/primitive.h:106-124); dpdu/dpdv are never set by a sphere */
static int sphere_intersect(v3 center, float radius, int obj, v3 o, v3 d, hinfo* info) {
    float t = 0.0f;
    if (!sphere_do_intersect(o, d, center, radius * radius, &t)) return 0;
    if (t < info->t) {
        info->t = t;
        info->pos = ray_at(o, d, t);
        info->ng = vnormalize(vsub(ray_at(o, d, t), center));
        info->ns = info->ng;
        info->hit = obj;
    }
    return 1;
}

/* BoxMesh::intersect (Src/primitive.h:243-264): overwrites unconditionally */
static int box_intersect(v3 pmin, v3 pmax, int obj, v3 o, v3 d, hinfo* info) {
    v3 dinv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    v3 ttop = vmul(dinv, vsub(pmax, o));
    v3 tbot = vmul(dinv, vsub(pmin, o));
    v3 tmin = mk(smin(ttop.x, tbot.x), smin(ttop.y, tbot.y), smin(ttop.z, tbot.z));
    v3 tmax = mk(smax(ttop.x, tbot.x), smax(ttop.y, tbot.y), smax(ttop.z, tbot.z));
    float t0 = smax(smax(tmin.x, tmin.y), tmin.z);
    float t1 = smin(smin(tmax.x, tmax.y), tmax.z);
    if (t0 > t1 || t1 <= 0.0f) return 0;
    t0 = smax(t0, 0.0f);
    info->hit = obj;
    info->t = t0;
    info->t1 = t1;
    return 1;
}

/* Scene::intersect (Src/scene.cpp:190-200): every object in m_objects order */
static int scene_intersect(const xrt_scene_desc* S, v3 o, v3 d, hinfo* info, uint64_t* tests) {
    int any = 0;
    for (uint32_t k = 0; k < S->n_objects; ++k) {
        const xrt_object* ob = &S->objects[k];
        int r = 0;
        if (ob->kind == XRT_OBJ_MESH) r = mesh_intersect(S, (int)k, o, d, info, tests);
        else if (ob->kind == XRT_OBJ_SPHERE) {
            const float* sp = S->spheres + (size_t)ob->first * 4;
            r = sphere_intersect(ld3(sp), sp[3], (int)k, o, d, info);
        } else if (ob->kind == XRT_OBJ_BOX) {
            const float* bx = S->boxes + (size_t)ob->first * 6;
            r = box_intersect(ld3(bx), ld3(bx + 3), (int)k, o, d, info);
        }
        if (r) any = 1;
    }
    return any;
}

/* Scene::occluded (Src/scene.cpp:202-211): objects without an area light, early exit */
static int scene_occluded(const xrt_scene_desc* S, v3 o, v3 d, float tmax, uint64_t* tests) {
    for (uint32_t k = 0; k < S->n_objects; ++k) {
        const xrt_object* ob = &S->objects[k];
        if (ob->light >= 0) continue;
        if (ob->kind == XRT_OBJ_MESH) {
            if (mesh_occluded(S, (int)k, o, d, tmax, tests)) return 1;
        } else if (ob->kind == XRT_OBJ_SPHERE) {
            const float* sp = S->spheres + (size_t)ob->first * 4;
            float t = 0.0f;
            /* Sphere::occluded (Src/primitive.h:126-130) */
            if (sphere_do_intersect(o, d, ld3(sp), sp[3] * sp[3], &t) && t < tmax) return 1;
        } else if (ob->kind == XRT_OBJ_BOX) {
            return 1; /* BoxMesh::occluded returns true (Src/primitive.h:266-268) */
        }
    }
    return 0;
}

/* ---------------------------------------------------------------- lights ---- */
/* AreaLight::Le (Src/light.h:62-69): one-sided */
static inline v3 light_Le(const xrt_light* l, v3 ns, v3 wi) {
    if (vdot(wi, ns) < 0) return ld3(l->Le);
    return mk(0, 0, 0);
}

/* Returns L; writes wi, pdf, tmax exactly as the reference's sample() would (pdf is left
 * untouched on the back-facing early return). */
static v3 light_sample(const xrt_light* l, v3 position, v3* wi, float* pdf, float* tmax, orc_mt* rng) {
    if (l->kind == XRT_LIGHT_QUAD) {
        /* QuadLight::sample (Src/light.cpp:59-68); GCC evaluates the second getNext1D()
         * operand first, so the first draw scales e2 and the second e1. */
        v3 v0 = ld3(l->v0), v1 = ld3(l->v1), v2 = ld3(l->v2);
        v3 e1 = vsub(v1, v0), e2 = vsub(v2, v0), Ng = vcross(e1, e2);
        float ra = orc_draw(rng);
        float rb = orc_draw(rng);
        v3 d = vsub(vadd(vadd(v0, vmuls(e1, rb)), vmuls(e2, ra)), position);
        *tmax = vlength(d);
        float dn = vdot(d, Ng);
        if (dn >= 0) return mk(0, 0, 0);
        *wi = vdivs(d, *tmax);
        *pdf = (*tmax * *tmax * *tmax) / fabsf(dn);
        return ld3(l->Le);
    } else if (l->kind == XRT_LIGHT_TRIANGLE) {
        /* TriangleLight::sample (Src/light.cpp:21-30) + uniformSampleTriangle (:43-47):
         * arguments evaluated right to left -> first draw is v, second u. */
        v3 A = ld3(l->v0), B = ld3(l->v1), C = ld3(l->v2);
        v3 Ng = vcross(vsub(B, A), vsub(C, A));
        float vv = orc_draw(rng);
        float uu = orc_draw(rng);
        float su = sqrtf(uu);
        v3 p = vadd(vadd(C, vmuls(vsub(A, C), 1.f - su)), vmuls(vsub(B, C), vv * su));
        v3 d = vsub(p, position);
        *tmax = vlength(d);
        float dn = vdot(d, Ng);
        if (dn >= 0) return mk(0, 0, 0);
        *wi = vdivs(d, *tmax);
        *pdf = (2.f * *tmax * *tmax * *tmax) / fabsf(dn);
        return ld3(l->Le);
    } else if (l->kind == XRT_LIGHT_SPHERE_AREA) {
        /* SphereLight::sample with AREA_SAMPLING (Src/light.h:131-135,185-191) and
         * UniformSampleSphere (Src/light.cpp:99-105).  GCC evaluates the call's second
         * getNext1D() operand first: the first draw is r2 (phi), the second r1 (z). */
        v3 center = ld3(l->center);
        float r2 = orc_draw(rng);
        float r1 = orc_draw(rng);
        float z = 1.f - 2.f * r1;
        float sin_theta = sqrtf(1 - z * z);
        float phi = PI_MUL_2 * r2;
        v3 n = mk(cosf(phi) * sin_theta, sinf(phi) * sin_theta, z);
        v3 p = vadd(center, vmuls(n, l->radius));
        v3 d = vsub(p, position);
        *tmax = vlength(d);
        float dn = vdot(d, n);
        if (dn >= 0) return mk(0, 0, 0);
        *wi = vdivs(d, *tmax);
        *pdf = (2.f * *tmax * *tmax * *tmax) / fabsf(dn);
        return ld3(l->Le);
    } else {
        /* SphereLight::sample, default (cone) branch (Src/light.h:157-197) */
        v3 center = ld3(l->center);
        float radius = l->radius;
        v3 dz = vsub(center, position);
        float dz_len_2 = vdot(dz, dz);
        float dz_len = sqrtf(dz_len_2);
        dz = vdivv(dz, mk(-dz_len, -dz_len, -dz_len));
        v3 dx, dy;
        onb(dz, &dx, &dy);
        float sin_theta_max_2 = radius * radius / dz_len_2;
        float sin_theta_max = sqrtf(sin_theta_max_2);
        float cos_theta_max = sqrtf(smax(0.f, 1.f - sin_theta_max_2));
        float cos_theta = 1 + (cos_theta_max - 1) * orc_draw(rng);
        float sin_theta_2 = 1.f - cos_theta * cos_theta;
        float cos_alpha = sin_theta_2 / sin_theta_max +
                          cos_theta * sqrtf(smax(0.0f, 1 - sin_theta_2 / sin_theta_max_2));
        float sin_alpha = sqrtf(smax(0.0f, 1 - cos_alpha * cos_alpha));
        float phi = PI_MUL_2 * orc_draw(rng);
        v3 n = vadd(vadd(vmuls(dx, cosf(phi) * sin_alpha), vmuls(dy, sinf(phi) * sin_alpha)),
                    vmuls(dz, cos_alpha));
        v3 p = vadd(center, vmuls(n, radius));
        v3 d = vsub(p, position);
        *tmax = vlength(d);
        float dn = vdot(d, n);
        if (dn >= 0) return mk(0, 0, 0);
        *pdf = 1.f / (PI_MUL_2 * (1.f - cos_theta_max));
        *wi = vdivs(d, *tmax);
        return ld3(l->Le);
    }
}

/* ---------------------------------------------------------------- Lambert ---- */
/* Lambert::sampleDir + uniformSampleHemisphere (Src/material.h:55-73) */
static v3 lambert_sample_dir(v3 ng, v3 dpdu, v3 dpdv, orc_mt* rng, float* pdf) {
    float r1 = orc_draw(rng);
    float r2 = orc_draw(rng);
    *pdf = 1 / (2 * PI_F);
    float sinTheta = sqrtf(1 - r1 * r1);
    float phi = 2 * PI_F * r2;
    float x = sinTheta * cosf(phi);
    float z = sinTheta * sinf(phi);
    return local_to_world(mk(x, r1, z), dpdu, ng, dpdv);
}

/* Object::evaluateBxDF -> Lambert::evaluateBxDF = albedo / PI (Src/material.h:39-48) */
static inline v3 eval_bxdf(const xrt_object* ob) {
    if (ob->material != XRT_MAT_LAMBERT) return mk(0, 0, 0);
    return vdivs(ld3(ob->albedo), PI_F);
}

/* ---------------------------------------------------------------- medium ---- */
/* DensityGrid::getDensity = OpenVDB GridSampler<FloatGrid, BoxSampler>::wsSample
 * (Src/grid.h:71-77): world->index in double, floor, trilinear lerps
 * a + float((b - a) * w) nested z, y, x; background 0 outside the grid. */
static float grid_value(const xrt_medium_desc* M, int i, int j, int k) {
    if (i < 0 || j < 0 || k < 0 || i >= (int)M->nx || j >= (int)M->ny || k >= (int)M->nz) return 0.0f;
    return M->density[((size_t)k * M->ny + (size_t)j) * M->nx + (size_t)i];
}
static inline float vdb_lerp(float a, float b, double w) { return a + (float)((double)(b - a) * w); }
static float grid_density(const xrt_medium_desc* M, v3 p) {
    double inv = 1.0 / (double)M->voxel_size;
    double xi = ((double)p.x - (double)M->origin[0]) * inv;
    double yi = ((double)p.y - (double)M->origin[1]) * inv;
    double zi = ((double)p.z - (double)M->origin[2]) * inv;
    double fx = floor(xi), fy = floor(yi), fz = floor(zi);
    int i = (int)fx, j = (int)fy, k = (int)fz;
    double u = xi - fx, v = yi - fy, w = zi - fz;
    float d000 = grid_value(M, i, j, k), d001 = grid_value(M, i, j, k + 1);
    float d010 = grid_value(M, i, j + 1, k), d011 = grid_value(M, i, j + 1, k + 1);
    float d100 = grid_value(M, i + 1, j, k), d101 = grid_value(M, i + 1, j, k + 1);
    float d110 = grid_value(M, i + 1, j + 1, k), d111 = grid_value(M, i + 1, j + 1, k + 1);
    return vdb_lerp(vdb_lerp(vdb_lerp(d000, d001, w), vdb_lerp(d010, d011, w), v),
                    vdb_lerp(vdb_lerp(d100, d101, w), vdb_lerp(d110, d111, w), v), u);
}
/* HeterogeneousMedium::getDensity (Src/medium.cpp:24-27) */
static inline float medium_density(const xrt_medium_desc* M, v3 p) {
    return M->density_multiplier * grid_density(M, p);
}

/* Medium::sampleWavelength + DiscreteEmpiricalDistribution1D (Src/medium.h:102-115,
 * Src/sampler.h:53-94).  lower_bound past the end (u > cdf[3]) is undefined in the
 * reference (reads element 3 of a Vec3f); both our implementations clamp it to channel
 * 2 and count it (orc_stats.ub_channel). */
static uint32_t sample_wavelength(v3 thr, v3 albedo, orc_mt* rng, v3* pmf, uint64_t* ub) {
    v3 ta = vmul(thr, albedo);
    float vals[3] = {ta.x, ta.y, ta.z};
    float sum = 0;
    for (int i = 0; i < 3; ++i) sum += vals[i];
    float cdf[4];
    cdf[0] = 0;
    for (int i = 1; i < 4; ++i) cdf[i] = cdf[i - 1] + vals[i - 1] / sum;
    *pmf = mk(cdf[1] - cdf[0], cdf[2] - cdf[1], cdf[3] - cdf[2]);
    float u = orc_draw(rng);
    int x = 0;
    while (x < 4 && cdf[x] < u) ++x; /* std::lower_bound */
    if (x == 0) x++;
    if (x == 4) { x = 3; if (ub) (*ub)++; }
    return (uint32_t)(x - 1);
}

/* HenyeyGreenstein::evaluate / sampleDirection (Src/medium.h:29-67).  getNext2D returns
 * (second draw, first draw) under GCC. */
static float hg_evaluate(float g, v3 wo, v3 wi) {
    const float cosTheta = vdot(wo, wi);
    const float denom = 1 + g * g - 2 * g * cosTheta;
    return PI_MUL_4_INV * (1 - g * g) / (denom * sqrtf(denom));
}
static float hg_sample(float g, v3 wo, orc_mt* rng, v3* wi) {
    float d1 = orc_draw(rng);
    float d2 = orc_draw(rng);
    float u0 = d2, u1 = d1;
    float cosTheta;
    if (fabs((double)g) < 1e-3) {
        cosTheta = 2 * u0 - 1.0f;
    } else {
        const float sqrTerm = (1 - g * g) / (1 - g + 2 * g * u0);
        cosTheta = (1 + g * g - sqrTerm * sqrTerm) / (2 * g);
    }
    const float sinTheta = sqrtf(smax(1.0f - cosTheta * cosTheta, 0.0f));
    const float phi = 2 * PI_F * u1;
    const v3 wi_local = mk(cosf(phi) * sinTheta, cosTheta, sinf(phi) * sinTheta);
    v3 t, b;
    onb(wo, &t, &b);
    *wi = local_to_world(wi_local, t, wo, b);
    return hg_evaluate(g, wo, *wi);
}

static inline int isnan3(v3 a) { return isnan(a.x) || isnan(a.y) || isnan(a.z); }

/* HeterogeneousMedium::sampleMedium — delta tracking with spectral MIS
 * (Src/medium.cpp:45-133).  Returns 1 on a real scattering event. */
static int sample_medium(const scene_ctx* C, v3 ro, v3 rd, v3 rthr, const hinfo* info, orc_mt* rng,
                         v3* pos, v3* dir, v3* throughput, uint64_t* ub) {
    const xrt_medium_desc* M = C->M;
    const float majorant = C->majorant, invMajorant = C->inv_majorant;
    const v3 absorb = ld3(M->absorption), scatter = ld3(M->scattering);
    const v3 vmaj = mk(majorant, majorant, majorant);
    v3 tt = mk(1, 1, 1);
    float t = info->t;
    const float density0 = medium_density(M, ray_at(ro, rd, t));
    v3 sigma_a = vmuls(absorb, density0);
    for (;;) {
        v3 pmf;
        const uint32_t channel = sample_wavelength(vmul(rthr, tt), vmuls(vsub(vmaj, sigma_a), invMajorant), rng, &pmf, ub);
        const float s = -logf(smax(1.0f - orc_draw(rng), 0.0f)) * invMajorant;
        t += s;
        if (t > info->t1 - RAY_EPS) {
            *pos = ray_at(ro, rd, info->t1 + RAY_EPS);
            *dir = rd;
            const float dist = s - (t - (info->t1 - RAY_EPS));
            const v3 tr = vexp(vmuls(vneg(vmaj), dist));
            const v3 pdf = vmul(pmf, tr);
            tt = vmul(tt, vdivs(tr, pdf.x + pdf.y + pdf.z));
            *throughput = isnan3(tt) ? mk(0, 0, 0) : tt;
            return 0;
        }
        const float density = medium_density(M, ray_at(ro, rd, t));
        const v3 sigma_s = vmuls(scatter, density);
        sigma_a = vmuls(absorb, density);
        const v3 sigma_n = vsub(vsub(vmaj, sigma_a), sigma_s);
        const v3 P_s = vdivv(sigma_s, vadd(sigma_s, sigma_n));
        const v3 P_n = vdivv(sigma_n, vadd(sigma_s, sigma_n));
        if (orc_draw(rng) < comp(P_s, (int)channel)) {
            *pos = ray_at(ro, rd, t);
            hg_sample(M->g, rd, rng, dir);
            const v3 tr = vexp(vmuls(vneg(vmaj), s));
            const v3 pdf_distance = vmuls(tr, majorant);
            const v3 pdf = vmul(vmul(pmf, pdf_distance), P_s);
            tt = vmul(tt, vdivs(vmul(tr, sigma_s), pdf.x + pdf.y + pdf.z));
            *throughput = isnan3(tt) ? mk(0, 0, 0) : tt;
            return 1;
        }
        const v3 tr = vexp(vmuls(vneg(vmaj), s));
        const v3 pdf_distance = vmuls(tr, majorant);
        const v3 pdf = vmul(vmul(pmf, pdf_distance), P_n);
        tt = vmul(tt, vdivs(vmul(tr, sigma_n), pdf.x + pdf.y + pdf.z));
    }
}

/* Homogeneous media (Src/medium.h:122-277): one free-flight sample, analytic
 * transmittance exp(-sigma_t * t).  Returns 1 on a scattering event. */
static inline v3 analytic_tr(float t, v3 sigma_t) {   /* Medium::analyticTransmittance */
    return vexp(vmuls(vneg(sigma_t), t));
}
static int homog_sample_medium(const xrt_medium_desc* M, v3 ro, v3 rd, v3 rthr, const hinfo* info, orc_mt* rng,
                               v3* pos, v3* dir, v3* throughput, uint64_t* ub) {
    const v3 sa = ld3(M->absorption), ss = ld3(M->scattering), st = vadd(sa, ss);
    const float distToSurface = info->t1 - info->t;
    if (M->kind == XRT_MEDIUM_HOMOGENEOUS_MIS) {
        /* HomogeneousMediumMIS::sampleMedium (Src/medium.h:154-191) */
        v3 pmf;
        const uint32_t channel = sample_wavelength(rthr, vdivv(ss, st), rng, &pmf, ub);
        const float t = -logf(smax(1.0f - orc_draw(rng), 0.0f)) / comp(st, (int)channel);
        if (t > distToSurface - RAY_EPS) {
            *pos = ray_at(ro, rd, info->t1 + RAY_EPS);
            *dir = rd;
            const v3 tr = analytic_tr(distToSurface, st);
            const v3 pdf = vmul(pmf, tr);
            *throughput = vdivs(tr, pdf.x + pdf.y + pdf.z);
            return 0;
        }
        hg_sample(M->g, rd, rng, dir);
        *pos = ray_at(ro, rd, info->t + t);
        const v3 tr = analytic_tr(t, st);
        const v3 pdf = vmul(pmf, vmul(st, tr));
        *throughput = vdivs(vmul(tr, ss), pdf.x + pdf.y + pdf.z);
        return 1;
    }
    if (M->kind == XRT_MEDIUM_HOMOGENEOUS_ACHROMATIC) {
        /* HomogeneousMediumAchromatic::sampleMedium (Src/medium.h:201-229) */
        const float t = -logf(smax(1.0f - orc_draw(rng), 0.0f)) / st.x;
        if (t > distToSurface - RAY_EPS) {
            *pos = ray_at(ro, rd, info->t1 + RAY_EPS);
            *dir = rd;
            *throughput = mk(1.0f, 1.0f, 1.0f);
            return 0;
        }
        hg_sample(M->g, rd, rng, dir);
        *pos = ray_at(ro, rd, info->t + t);
        *throughput = vdivv(ss, st);
        return 1;
    }
    /* HomogeneousMediumNoMIS::sampleMedium (Src/medium.h:240-275) */
    int channel = (int)(3 * orc_draw(rng));
    if (channel == 3) channel--;
    const float pmf_wavelength = 1.0f / 3.0f;
    const float sc = comp(st, channel);
    const float t = -logf(smax(1.0f - orc_draw(rng), 0.0f)) / sc;
    const float pdf_distance = sc * expf(-sc * t);
    if (t > distToSurface - RAY_EPS) {
        *pos = ray_at(ro, rd, info->t1 + RAY_EPS);
        *dir = rd;
        const v3 tr = analytic_tr(distToSurface, st);
        const float p_surface = expf(-sc * distToSurface);
        *throughput = vdivs(vmuls(tr, 1.0f / 3.0f), pmf_wavelength * p_surface);
        return 0;
    }
    hg_sample(M->g, rd, rng, dir);
    *pos = ray_at(ro, rd, info->t + t);
    *throughput = vdivs(vmul(vmuls(analytic_tr(t, st), 1.0f / 3.0f), ss), pmf_wavelength * pdf_distance);
    return 1;
}

/* Object::sampleMedium -> the scene medium's sampleMedium */
static int medium_sample(const scene_ctx* C, v3 ro, v3 rd, v3 rthr, const hinfo* info, orc_mt* rng, v3* pos,
                         v3* dir, v3* throughput, uint64_t* ub) {
    if (C->M->kind != XRT_MEDIUM_HETEROGENEOUS)
        return homog_sample_medium(C->M, ro, rd, rthr, info, rng, pos, dir, throughput, ub);
    return sample_medium(C, ro, rd, rthr, info, rng, pos, dir, throughput, ub);
}

/* ---------------------------------------------------------------- integrators ---- */
typedef struct {
    uint64_t segments, shadow_rays, tri_tests, stalled, ub_channel;
} path_counters;

/* GIIntegrator::integrate (Src/integrator.h:205-287) */
static v3 integrate_gi(const scene_ctx* C, v3 ro, v3 rd, uint32_t max_depth, orc_mt* rng, path_counters* pc) {
    const xrt_scene_desc* S = C->S;
    v3 radiance = mk(0, 0, 0);
    v3 thr = mk(1, 1, 1);
    const v3 background = mk(0, 0, 0);
    uint32_t depth = 0;
    while (depth < max_depth) {
        hinfo info;
        hinfo_init(&info);
        pc->segments++;
        if (!scene_intersect(S, ro, rd, &info, &pc->tri_tests)) {
            radiance = vadd(radiance, vmul(thr, background));
            break;
        }
        if (depth > 0) {
            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
            if (orc_draw(rng) >= p) break;
            thr = vdivv(thr, mk(p, p, p));
        }
        const xrt_object* ob = &S->objects[info.hit];
        if (ob->light >= 0) {
            if (depth == 0) radiance = vadd(radiance, vmul(thr, light_Le(&S->lights[ob->light], info.ns, rd)));
            break;
        }
        v3 directL = mk(0, 0, 0);
        for (uint32_t li = 0; li < S->n_lights; ++li) {
            v3 L_light = mk(0, 0, 0);
            v3 wi = mk(0, 0, 0);
            float tmax = 0.0f, pdf = 0.0f;
            v3 L = light_sample(&S->lights[li], info.pos, &wi, &pdf, &tmax, rng);
            if (pdf == 0) continue;
            const float bias = 0.01f;
            pc->shadow_rays++;
            int vis = !scene_occluded(S, vadd(info.pos, vmuls(info.ng, bias)), wi, tmax - bias, &pc->tri_tests);
            float cosv = smax(0.0f, vdot(info.ng, wi));
            v3 fr = eval_bxdf(ob);
            L_light = vadd(L_light, vdivs(vmuls(vmul(vmuls(fr, (float)vis), L), cosv), pdf));
            directL = vadd(directL, L_light);
        }
        radiance = vadd(radiance, vmul(thr, directL));
        /* Object::sampleBxDF (primitive.cpp:35-40): no material -> 0, no draws */
        float pdf = 1.0f;
        v3 nextDir = mk(0, 0, 0);
        v3 fr = mk(0, 0, 0);
        if (ob->material == XRT_MAT_LAMBERT) {
            nextDir = lambert_sample_dir(info.ng, info.dpdu, info.dpdv, rng, &pdf);
            fr = eval_bxdf(ob);
        }
        float cosv = smax(.0f, vdot(nextDir, info.ng));
        const float bias = 0.01f;
        thr = vmul(thr, vdivs(vmuls(fr, cosv), pdf));
        ro = vadd(info.pos, vmuls(info.ng, bias));
        rd = nextDir;
        depth++;
    }
    return radiance;
}

/* IndirectIntegrator::integrate (Src/integrator.h:130-185): GIIntegrator's bounce loop with
 * no light sampling; an area light adds throughput * Le at every depth */
static v3 integrate_indirect(const scene_ctx* C, v3 ro, v3 rd, uint32_t max_depth, orc_mt* rng, path_counters* pc) {
    const xrt_scene_desc* S = C->S;
    v3 radiance = mk(0, 0, 0);
    v3 thr = mk(1, 1, 1);
    const v3 background = mk(0, 0, 0);
    uint32_t depth = 0;
    while (depth < max_depth) {
        hinfo info;
        hinfo_init(&info);
        pc->segments++;
        if (!scene_intersect(S, ro, rd, &info, &pc->tri_tests)) {
            radiance = vadd(radiance, vmul(thr, background));
            break;
        }
        if (depth > 0) {
            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
            if (orc_draw(rng) >= p) break;
            thr = vdivv(thr, mk(p, p, p));
        }
        const xrt_object* ob = &S->objects[info.hit];
        if (ob->light >= 0) {
            radiance = vadd(radiance, vmul(thr, light_Le(&S->lights[ob->light], info.ns, rd)));
            break;
        }
        float pdf = 1.0f;
        v3 nextDir = mk(0, 0, 0);
        v3 fr = mk(0, 0, 0);
        if (ob->material == XRT_MAT_LAMBERT) {
            nextDir = lambert_sample_dir(info.ng, info.dpdu, info.dpdv, rng, &pdf);
            fr = eval_bxdf(ob);
        }
        float cosv = smax(.0f, vdot(nextDir, info.ng));
        const float bias = 0.01f;
        thr = vmul(thr, vdivs(vmuls(fr, cosv), pdf));
        ro = vadd(info.pos, vmuls(info.ng, bias));
        rd = nextDir;
        depth++;
    }
    return radiance;
}

/* NormalIntegrator::integrate (Src/integrator.h:28-37): 0.5 * (ns + 1) on a hit, else 0.
 * (Everything after its first return is unreachable.) */
static v3 integrate_normal(const scene_ctx* C, v3 ro, v3 rd, path_counters* pc) {
    hinfo info;
    hinfo_init(&info);
    pc->segments++;
    if (scene_intersect(C->S, ro, rd, &info, &pc->tri_tests)) {
        const v3 a = mk(info.ns.x + 1.0f, info.ns.y + 1.0f, info.ns.z + 1.0f);
        return mk(0.5f * a.x, 0.5f * a.y, 0.5f * a.z);
    }
    return mk(0, 0, 0);
}

/* DirectIntegrator::integrate (Src/integrator.h:82-119) */
static v3 integrate_direct(const scene_ctx* C, v3 ro, v3 rd, orc_mt* rng, path_counters* pc) {
    const xrt_scene_desc* S = C->S;
    v3 radiance = mk(0.0f, 0.0f, 0.0f);
    hinfo info;
    hinfo_init(&info);
    pc->segments++;
    if (scene_intersect(S, ro, rd, &info, &pc->tri_tests)) {
        const xrt_object* ob = &S->objects[info.hit];
        if (ob->light >= 0) return light_Le(&S->lights[ob->light], info.ns, rd);
        for (uint32_t li = 0; li < S->n_lights; ++li) {
            v3 wi = mk(0, 0, 0);
            float tmax = 0.0f, pdf = 0.0f;
            v3 L = light_sample(&S->lights[li], info.pos, &wi, &pdf, &tmax, rng);
            if (pdf == 0) continue;
            const float bias = 0.01f;
            pc->shadow_rays++;
            int vis = !scene_occluded(S, vadd(info.pos, vmuls(info.ng, bias)), wi, tmax - bias, &pc->tri_tests);
            float cosv = smax(0.0f, vdot(info.ng, wi));
            v3 fr = eval_bxdf(ob);
            radiance = vadd(radiance, vdivs(vmuls(vmul(vmuls(fr, (float)vis), L), cosv), pdf));
        }
    } else {
        return mk((float)0.18, (float)0.18, (float)0.18);
    }
    return radiance;
}

/* VolumePathTracing::integrate (Src/integrator.h:409-473).  An object that is neither a
 * light nor a medium never advances the ray in the reference (an endless loop,
 * SURVEY §3.4); here the path stops and is counted in `stalled`. */
static v3 integrate_vpt(const scene_ctx* C, v3 ro, v3 rd, uint32_t max_depth, orc_mt* rng, path_counters* pc) {
    const xrt_scene_desc* S = C->S;
    v3 radiance = mk(0, 0, 0);
    v3 thr = mk(1, 1, 1);
    const v3 background = mk(0.0f, 0.0f, 0.0f);
    uint32_t depth = 0;
    while (depth < max_depth) {
        hinfo info;
        hinfo_init(&info);
        pc->segments++;
        if (!scene_intersect(S, ro, rd, &info, &pc->tri_tests)) {
            radiance = vadd(radiance, vmuls(vmul(thr, background), (float)(depth != 0)));
            break;
        }
        if (depth > 0) {
            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
            if (orc_draw(rng) >= p) break;
            thr = vdivv(thr, mk(p, p, p));
        }
        const xrt_object* ob = &S->objects[info.hit];
        if (ob->light >= 0) {
            radiance = vadd(radiance, vmul(thr, light_Le(&S->lights[ob->light], info.ns, rd)));
            break;
        }
        if (ob->medium >= 0 && C->M) {
            v3 pos, dir, tm;
            int scattered = medium_sample(C, ro, rd, thr, &info, rng, &pos, &dir, &tm, &pc->ub_channel);
            ro = pos;
            rd = dir;
            thr = vmul(thr, tm);
            if (scattered) depth++;
        } else {
            pc->stalled++;
            break;
        }
    }
    return radiance;
}

/* HeterogeneousMedium::ratioTrackingTransmittance (Src/medium.h:360-386) */
static v3 ratio_tracking(const scene_ctx* C, v3 p1, v3 p2, orc_mt* rng) {
    const xrt_medium_desc* M = C->M;
    const float majorant = C->majorant, invMajorant = C->inv_majorant;
    const v3 vmaj = mk(majorant, majorant, majorant);
    const float distToEnd = vlength(vsub(p1, p2));
    float t = 0;
    const v3 dn = vnormalize(vsub(p2, p1));
    v3 tr = mk(1, 1, 1);
    for (;;) {
        const float s = -logf(smax(1.0f - orc_draw(rng), 0.0f)) * invMajorant;
        t += s;
        if (t > distToEnd) break;
        const float density = medium_density(M, ray_at(p1, dn, t));
        const v3 sigma_n = vsub(vsub(vmaj, vmuls(ld3(M->absorption), density)), vmuls(ld3(M->scattering), density));
        tr = vmul(tr, vmuls(sigma_n, invMajorant));
    }
    return tr;
}

/* VolumePathTracingNEE::integrate (Src/integrator.h:489-584) with sampleDirectionToLight
 * (:586-602, Scene::sampleAreaLight Src/scene.cpp:182-188) and isVisible (:604-631):
 * the shadow ray takes the closest hit, a surface occludes, a medium attenuates by ratio
 * tracking between the hit's t and t1.  Objects with neither light nor medium stall the
 * path as in integrate_vpt. */
static v3 integrate_vpt_nee(const scene_ctx* C, v3 ro, v3 rd, uint32_t max_depth, orc_mt* rng, path_counters* pc) {
    const xrt_scene_desc* S = C->S;
    v3 radiance = mk(0, 0, 0);
    v3 thr = mk(1, 1, 1);
    const v3 background = mk(0.0f, 0.0f, 0.0f);
    uint32_t depth = 0;
    while (depth < max_depth) {
        hinfo info;
        hinfo_init(&info);
        pc->segments++;
        if (!scene_intersect(S, ro, rd, &info, &pc->tri_tests)) {
            radiance = vadd(radiance, vmuls(vmul(thr, background), (float)(depth != 0)));
            break;
        }
        if (depth > 0) {
            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
            if (orc_draw(rng) >= p) break;
            thr = vdivv(thr, mk(p, p, p));
        }
        const xrt_object* ob = &S->objects[info.hit];
        if (ob->light >= 0) {
            if (depth == 0) radiance = vadd(radiance, vmul(thr, light_Le(&S->lights[ob->light], info.ns, rd)));
            break;
        }
        if (ob->medium >= 0 && C->M) {
            v3 pos, dir, tm;
            const int scattered = medium_sample(C, ro, rd, thr, &info, rng, &pos, &dir, &tm, &pc->ub_channel);
            if (scattered) {
                /* light index: (unsigned)(size * u), clamped; pdf 1 / size */
                unsigned li = (unsigned)((float)S->n_lights * orc_draw(rng));
                if (li == S->n_lights) li--;
                const float choose = 1.0f / (float)S->n_lights;
                v3 wl = mk(0, 0, 0);
                float lpdf = 0.0f, dist = 0.0f;
                const v3 Le = light_sample(&S->lights[li], pos, &wl, &lpdf, &dist, rng);
                const float pdf_dir = choose * lpdf;
                if (pdf_dir > 0.0f) {
                    v3 transmittance = mk(1, 1, 1);
                    int visible = 1;
                    hinfo sh;
                    hinfo_init(&sh);
                    pc->shadow_rays++;
                    if (scene_intersect(S, pos, wl, &sh, &pc->tri_tests)) {
                        const xrt_object* so = &S->objects[sh.hit];
                        if (so->material != XRT_MAT_NONE) {
                            visible = 0;
                        } else if (so->medium >= 0) {
                            const v3 p1 = ray_at(pos, wl, sh.t), p2 = ray_at(pos, wl, sh.t1);
                            /* Medium::transmittance: ratio tracking (heterogeneous) or
                             * analyticTransmittance(length(p1 - p2), sigma_t) (Src/medium.h:133-137) */
                            transmittance = vmul(transmittance,
                                                 C->M->kind == XRT_MEDIUM_HETEROGENEOUS
                                                     ? ratio_tracking(C, p1, p2, rng)
                                                     : analytic_tr(vlength(vsub(p1, p2)),
                                                                   vadd(ld3(C->M->absorption), ld3(C->M->scattering))));
                        }
                    }
                    if (visible) {
                        const float f = hg_evaluate(C->M->g, rd, wl);
                        const v3 Ls = vdivs(vmul(vmuls(transmittance, f), Le), pdf_dir);
                        radiance = vadd(radiance, vmul(vmul(thr, tm), Ls));
                    }
                }
            }
            ro = pos;
            rd = dir;
            thr = vmul(thr, tm);
            if (scattered) depth++;
        } else {
            pc->stalled++;
            break;
        }
    }
    return radiance;
}

/* ---------------------------------------------------------------- renderer ---- */
static int setup_ctx(scene_ctx* C, const xrt_scene_desc* S, const xrt_medium_desc* M) {
    C->S = S;
    C->M = M;
    C->majorant = 0.0f;
    C->inv_majorant = 0.0f;
    if (M && M->kind == XRT_MEDIUM_HETEROGENEOUS) {
        /* HeterogeneousMedium ctor (Src/medium.cpp:5-17) */
        const float max_density = M->density_multiplier * M->max_density;
        const v3 m = vadd(vmuls(ld3(M->absorption), max_density), vmuls(ld3(M->scattering), max_density));
        C->majorant = smax(m.x, smax(m.y, m.z));
        C->inv_majorant = 1.0f / C->majorant;
    }
    return 0;
}

/* PinholeCamera::sampleRay (Src/camera.h:49-60) with multDirMatrix (geometry.h:653-669) */
static void camera_ray(const orc_camera* cam, float u, float v, v3* o, v3* d) {
    const float* x = cam->c2w;
    v3 dir = mk((2 * u - 1) * cam->scale, (1 - 2 * v) * cam->scale / cam->aspect, -1);
    v3 w = mk(dir.x * x[0] + dir.y * x[4] + dir.z * x[8], dir.x * x[1] + dir.y * x[5] + dir.z * x[9],
              dir.x * x[2] + dir.y * x[6] + dir.z * x[10]);
    *d = vnormalize(w);
    *o = mk(x[12], x[13], x[14]);
}

static v3 integrate(const scene_ctx* C, const xrt_render_params* p, v3 ro, v3 rd, orc_mt* rng, path_counters* pc) {
    if (p->integrator == XRT_INTEGRATOR_DIRECT) return integrate_direct(C, ro, rd, rng, pc);
    if (p->integrator == XRT_INTEGRATOR_VPT) return integrate_vpt(C, ro, rd, p->max_depth, rng, pc);
    if (p->integrator == XRT_INTEGRATOR_INDIRECT) return integrate_indirect(C, ro, rd, p->max_depth, rng, pc);
    if (p->integrator == XRT_INTEGRATOR_NORMAL) return integrate_normal(C, ro, rd, pc);
    if (p->integrator == XRT_INTEGRATOR_VPT_NEE) return integrate_vpt_nee(C, ro, rd, p->max_depth, rng, pc);
    return integrate_gi(C, ro, rd, p->max_depth, rng, pc);
}

/* NormalRenderer::doRender (Src/renderer.cpp:29-81) for one pixel; optional per-sample
 * records.  Returns the accumulated (not yet divided) pixel sum. */
static v3 do_render_pixel(const scene_ctx* C, const orc_camera* cam, const xrt_render_params* p,
                          uint32_t i, uint32_t j, path_counters* pc, uint64_t* draws, uint64_t* rejected,
                          float* rec_rad, uint32_t* rec_draws, uint32_t* rec_segs, v3 acc) {
    const uint32_t width = p->width, height = p->height;
    orc_mt rng;
    orc_mt_seed(&rng, j + width * i);
    for (uint32_t k = 0; k < p->spp; ++k) {
        uint64_t d0 = rng.draws, s0 = pc->segments;
        const float u = ((float)(int)j + orc_draw(&rng)) / (float)width;
        const float v = ((float)(int)i + orc_draw(&rng)) / (float)height;
        v3 ro, rd;
        camera_ray(cam, u, v, &ro, &rd);
        const float pdf = 1.0f;
        const v3 radiance = vdivs(integrate(C, p, ro, rd, &rng, pc), pdf);
        if (rec_rad) {
            st3(rec_rad + (size_t)k * 3, radiance);
            rec_draws[k] = (uint32_t)(rng.draws - d0);
            rec_segs[k] = (uint32_t)(pc->segments - s0);
        }
        if (isnan(radiance.x) || isnan(radiance.y) || isnan(radiance.z)) { (*rejected)++; continue; }
        if (isinf(radiance.x) || isinf(radiance.y) || isinf(radiance.z)) { (*rejected)++; continue; }
        if (radiance.x < 0 || radiance.y < 0 || radiance.z < 0) { (*rejected)++; continue; }
        acc = vadd(acc, radiance); /* Image::addPixel (Src/image.h:46-50) */
    }
    *draws += rng.draws;
    return acc;
}

static int check_params(const xrt_scene_desc* S, const xrt_render_params* p, const xrt_medium_desc* M) {
    if (!S || !p || p->width == 0 || p->height == 0 || p->shard_count == 0 || p->shard_index >= p->shard_count) return -1;
    if ((p->integrator == XRT_INTEGRATOR_VPT || p->integrator == XRT_INTEGRATOR_VPT_NEE) && !M) return -1;
    return 0;
}

int orc_render(const xrt_scene_desc* S, const orc_camera* cam, const xrt_medium_desc* M,
               const xrt_render_params* p, float* rgb_out, int nthreads, orc_stats* st) {
    if (check_params(S, p, M)) return XRT_ERR_INVALID;
    scene_ctx C;
    setup_ctx(&C, S, M);
    /* XRT_FLAG_ACCUMULATE: the reference's Image is filled in place — addPixel adds every
     * sample to what the pixel already holds (Src/renderer.cpp:75, image.h:46-50) */
    const int accumulate = (p->flags & XRT_FLAG_ACCUMULATE) != 0;
    if (!accumulate) memset(rgb_out, 0, sizeof(float) * 3 * (size_t)p->width * p->height);
    uint64_t segs = 0, shadows = 0, draws = 0, rejected = 0, tests = 0, stalled = 0, ub = 0, samples = 0;
    const int64_t rows = p->height;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : segs, shadows, draws, rejected, tests, stalled, ub, samples)
#endif
    for (int64_t ii = 0; ii < rows; ++ii) {
        const uint32_t i = (uint32_t)ii;
        if (i % p->shard_count != p->shard_index) continue;
        path_counters pc = {0, 0, 0, 0, 0};
        for (uint32_t j = 0; j < p->width; ++j) {
            float* px = rgb_out + ((size_t)j + (size_t)p->width * i) * 3;
            const v3 acc0 = accumulate ? mk(px[0], px[1], px[2]) : mk(0, 0, 0);
            v3 acc = do_render_pixel(&C, cam, p, i, j, &pc, &draws, &rejected, NULL, NULL, NULL, acc0);
            /* Image::operator/= (Src/image.h:69-78) with Vec3f(n_samples) */
            const float n = (float)p->spp;
            st3(px, vdivv(acc, mk(n, n, n)));
            samples += p->spp;
        }
        segs += pc.segments;
        shadows += pc.shadow_rays;
        tests += pc.tri_tests;
        stalled += pc.stalled;
        ub += pc.ub_channel;
    }
    if (st) {
        st->samples = samples; st->segments = segs; st->shadow_rays = shadows; st->draws = draws;
        st->rejected = rejected; st->tri_tests = tests; st->stalled = stalled; st->ub_channel = ub;
    }
    return XRT_OK;
}

int orc_trace_pixels(const xrt_scene_desc* S, const orc_camera* cam, const xrt_medium_desc* M,
                     const xrt_render_params* p, const uint32_t* pix_i, const uint32_t* pix_j, uint32_t n,
                     float* rad, uint32_t* draws, uint32_t* segs) {
    if (check_params(S, p, M)) return XRT_ERR_INVALID;
    scene_ctx C;
    setup_ctx(&C, S, M);
    for (uint32_t q = 0; q < n; ++q) {
        path_counters pc = {0, 0, 0, 0, 0};
        uint64_t dr = 0, rj = 0;
        (void)do_render_pixel(&C, cam, p, pix_i[q], pix_j[q], &pc, &dr, &rj, rad + (size_t)q * p->spp * 3,
                              draws + (size_t)q * p->spp, segs + (size_t)q * p->spp, mk(0, 0, 0));
    }
    return XRT_OK;
}

/* Scene::intersect on a fresh IntersectInfo / Scene::occluded (Src/scene.cpp:190-211) for n
 * rays {o, d} — the checker of xrt_query */
int orc_query(const xrt_scene_desc* S, uint32_t n, const float* rays, const float* tmax, int mode, xrt_hit* out) {
    uint64_t tests = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const float* r = rays + 6 * (size_t)i;
        const v3 o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
        xrt_hit* q = &out[i];
        memset(q, 0, sizeof(*q));
        q->object = -1, q->primitive = -1, q->t = K_INF, q->t1 = K_INF;
        if (mode == XRT_QUERY_OCCLUDED) {
            q->hit = scene_occluded(S, o, d, tmax ? tmax[i] : K_INF, &tests);
            continue;
        }
        hinfo h;
        hinfo_init(&h);
        q->hit = scene_intersect(S, o, d, &h, &tests);
        if (h.hit < 0) continue;
        q->object = h.hit, q->primitive = h.prim, q->t = h.t, q->t1 = h.t1;
        st3(q->position, h.pos), st3(q->ng, h.ng), st3(q->ns, h.ns), st3(q->dpdu, h.dpdu), st3(q->dpdv, h.dpdv);
        if (h.prim >= 0) q->barycentric[0] = h.bu, q->barycentric[1] = h.bv;
    }
    return XRT_OK;
}

/* ---------------------------------------------------------------- KATs ---- */
void orc_kat_normalize(const float* v, float* out) { st3(out, vnormalize(ld3(v))); }
void orc_kat_onb(const float* n, float* t, float* b) {
    v3 tt, bb;
    onb(ld3(n), &tt, &bb);
    st3(t, tt);
    st3(b, bb);
}
void orc_kat_lambert(orc_mt* m, const float* ng, const float* dpdu, const float* dpdv, float* wi, float* pdf) {
    st3(wi, lambert_sample_dir(ld3(ng), ld3(dpdu), ld3(dpdv), m, pdf));
}
void orc_kat_lambert_bxdf(orc_mt* m, const float* albedo, const float* ng, const float* dpdu, const float* dpdv,
                          float* f, float* wi, float* pdf) {
    xrt_object ob;
    memset(&ob, 0, sizeof(ob));
    ob.material = XRT_MAT_LAMBERT;
    ob.albedo[0] = albedo[0], ob.albedo[1] = albedo[1], ob.albedo[2] = albedo[2];
    st3(wi, lambert_sample_dir(ld3(ng), ld3(dpdu), ld3(dpdv), m, pdf));
    st3(f, eval_bxdf(&ob));
}
void orc_kat_camera(const orc_camera* cam, float u, float v, float* o, float* d) {
    v3 ro, rd;
    camera_ray(cam, u, v, &ro, &rd);
    st3(o, ro);
    st3(d, rd);
}
int orc_kat_ray_tri(const float* o, const float* d, const float* v0, const float* v1, const float* v2, float* tuv) {
    float t = 0, u = 0, v = 0;
    int r = ray_tri(ld3(o), ld3(d), ld3(v0), ld3(v1), ld3(v2), &t, &u, &v);
    tuv[0] = t; tuv[1] = u; tuv[2] = v;
    return r;
}
int orc_kat_sphere(const float* o, const float* d, const float* c, float r, float* out) {
    hinfo h;
    hinfo_init(&h);
    int res = sphere_intersect(ld3(c), r, 0, ld3(o), ld3(d), &h);
    out[0] = h.t;
    st3(out + 1, h.pos);
    st3(out + 4, h.ng);
    return res;
}
int orc_kat_sphere_occluded(const float* o, const float* d, const float* c, float r, float tmax) {
    float t = 0.0f;
    return sphere_do_intersect(ld3(o), ld3(d), ld3(c), r * r, &t) && t < tmax;
}
int orc_kat_box(const float* o, const float* d, const float* pmin, const float* pmax, float* out) {
    hinfo h;
    hinfo_init(&h);
    int r = box_intersect(ld3(pmin), ld3(pmax), 0, ld3(o), ld3(d), &h);
    out[0] = h.t;
    out[1] = h.t1;
    return r;
}
float orc_kat_hg(orc_mt* m, float g, const float* wo, float* wi) {
    v3 w;
    float r = hg_sample(g, ld3(wo), m, &w);
    st3(wi, w);
    return r;
}
uint32_t orc_kat_wavelength(orc_mt* m, const float* thr, const float* albedo, float* pmf) {
    v3 pm;
    uint32_t c = sample_wavelength(ld3(thr), ld3(albedo), m, &pm, NULL);
    st3(pmf, pm);
    return c;
}
void orc_kat_light(orc_mt* m, const xrt_light* l, const float* pos, float* out) {
    v3 wi = mk(0, 0, 0);
    float pdf = 0.0f, tmax = 0.0f;
    v3 L = light_sample(l, ld3(pos), &wi, &pdf, &tmax, m);
    st3(out, wi);
    out[3] = pdf;
    out[4] = tmax;
    st3(out + 5, L);
}

/* host glibc logf/expf over an array (the checker for the device restatement) */
void orc_libm_logexpf(const float* x, uint32_t n, float* lg, float* ex) {
    for (uint32_t i = 0; i < n; ++i) {
        lg[i] = logf(x[i]);
        ex[i] = expf(x[i]);
    }
}

/* host glibc sinf/cosf over an array (the checker for the device restatement) */
void orc_libm_sincosf(const float* x, uint32_t n, float* s, float* c) {
    for (uint32_t i = 0; i < n; ++i) {
        s[i] = sinf(x[i]);
        c[i] = cosf(x[i]);
    }
}

/* host libm powf (checker for the device restatement) */
void orc_libm_powf(const float* x, uint32_t n, float y, float* out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = powf(x[i], y);
}

/* Image::gammaCorrection (Src/image.h:80-90) then writePPM's per-channel value
 * std::clamp(static_cast<uint32_t>(255.0f * c), 0u, 255u) (:92-114) over n floats */
void orc_tonemap(const float* rgb, uint32_t n, float gamma, uint8_t* out) {
    for (uint32_t i = 0; i < n; ++i) {
        const float c = powf(rgb[i], 1.0f / gamma);
        uint32_t u = (uint32_t)(255.0f * c);
        out[i] = (uint8_t)(u > 255u ? 255u : u);
    }
}

