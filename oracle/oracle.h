/*
 * oracle.h — CPU restatement of xRayTracer's path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libxrt_hip.so, xraytracer_amd/)
 * links, loads or calls this code.  It is used by tests/ as the parity checker, by
 * __graft_entry__.smoke() as the checker, and by bench.py as the timed CPU baseline
 * (cpu_baseline.kind = "port").
 *
 * Pinning: the building blocks (mt19937 stream, normalize/ONB, Lambert::sampleDir,
 * Sphere/BoxMesh intersection, HenyeyGreenstein, sampleWavelength) are checked against
 * golden vectors produced by the reference's own sources compiled in place
 * (oracle/_ref, recipe oracle/Makefile, fixtures tests/golden/ref_kats.json).  The
 * parts whose reference translation units cannot be built here (camera.h, light.*,
 * primitive.cpp, integrator.h, renderer.cpp, scene.cpp all include spdlog / OpenCV /
 * OpenVDB / tinyobjloader, none of which exist in this image) are restated from the
 * source text with file:line citations and are "parity unpinned" beyond those KATs.
 * See DESIGN.md §Oracle.
 */
#ifndef XRT_ORACLE_H
#define XRT_ORACLE_H

#include <stdint.h>
#include "../include/xrt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* libstdc++ std::mt19937 (used by Sampler, Src/sampler.h:16) */
typedef struct {
    uint32_t x[624];
    uint32_t p;
    uint64_t draws;
} orc_mt;

void orc_mt_seed(orc_mt* m, uint32_t seed);
uint32_t orc_mt_next(orc_mt* m);
/* UniformSampler::getNext1D (Src/sampler.h:49): uniform_real_distribution<float>(0,1) */
float orc_draw(orc_mt* m);
/* draws n values for `seed` after skipping `skip` draws */
void orc_draws(uint32_t seed, uint32_t skip, uint32_t n, float* out);

typedef struct {
    float c2w[16];   /* row-major Matrix44f */
    float scale;     /* PinholeCamera::scale */
    float aspect;    /* Camera::aspect_ratio */
} orc_camera;

typedef struct {
    uint64_t samples, segments, shadow_rays, draws, rejected, tri_tests, stalled, ub_channel;
} orc_stats;

/* NormalRenderer::render / ParallelRenderer::render: fills rgb_out[H][W][3] for the rows
 * of shard (p->shard_index, p->shard_count); other rows are left at 0.
 * medium may be NULL unless the scene has a medium box.  nthreads <= 0: all cores. */
int orc_render(const xrt_scene_desc* scene, const orc_camera* cam, const xrt_medium_desc* medium,
               const xrt_render_params* p, float* rgb_out, int nthreads, orc_stats* st);

/* Per-sample record for a list of pixels (i = row, j = col):
 * rad[(n*spp + k)*3 + c], draws[n*spp + k], segs[n*spp + k] (Scene::intersect calls) */
int orc_trace_pixels(const xrt_scene_desc* scene, const orc_camera* cam,
                     const xrt_medium_desc* medium, const xrt_render_params* p,
                     const uint32_t* pix_i, const uint32_t* pix_j, uint32_t n,
                     float* rad, uint32_t* draws, uint32_t* segs);

/* Scene::intersect (fresh IntersectInfo) / Scene::occluded for n rays {o, d}: the checker
 * of xrt_query, same record layout */
int orc_query(const xrt_scene_desc* scene, uint32_t n, const float* rays, const float* tmax, int mode, xrt_hit* out);

/* ---- building-block KATs (each mirrors one reference function) ---------------------- */
void orc_kat_normalize(const float* v, float* out);                     /* geometry.cpp:13-16 */
void orc_kat_onb(const float* n, float* t, float* b);                     /* geometry.cpp:43-49 */
/* Lambert::sampleDir with SurfaceInfo{ng, dpdu, dpdv} (material.h:55-73): consumes 2 draws */
void orc_kat_lambert(orc_mt* m, const float* ng, const float* dpdu, const float* dpdv,
                     float* wi, float* pdf);
/* Lambert::sampleBxDF + evaluateBxDF (material.h:39-53): f = albedo / PI, 2 draws */
void orc_kat_lambert_bxdf(orc_mt* m, const float* albedo, const float* ng, const float* dpdu, const float* dpdv,
                          float* f, float* wi, float* pdf);
/* PinholeCamera::sampleRay (camera.h:49-60) for sensor coordinates (u, v) */
void orc_kat_camera(const orc_camera* cam, float u, float v, float* o, float* d);
/* Mesh::rayTriangleIntersect (primitive.cpp:140-168): returns hit, writes t,u,v */
int orc_kat_ray_tri(const float* o, const float* d, const float* v0, const float* v1,
                    const float* v2, float* tuv);
/* Sphere::intersect on a fresh IntersectInfo (primitive.h:106-124); out: t, pos, ng */
int orc_kat_sphere(const float* o, const float* d, const float* c, float r, float* out);
int orc_kat_sphere_occluded(const float* o, const float* d, const float* c, float r, float tmax);
/* BoxMesh::intersect (primitive.h:243-264); out: t, t1 */
int orc_kat_box(const float* o, const float* d, const float* pmin, const float* pmax, float* out);
/* HenyeyGreenstein::sampleDirection (medium.h:37-67): 2 draws; returns evaluate() */
float orc_kat_hg(orc_mt* m, float g, const float* wo, float* wi);
/* Medium::sampleWavelength (medium.h:102-115): 1 draw */
uint32_t orc_kat_wavelength(orc_mt* m, const float* thr, const float* albedo, float* pmf);
/* QuadLight::sample (light.cpp:59-68) / TriangleLight::sample (light.cpp:21-30) /
 * SphereLight::sample default branch (light.h:157-197).  out: wi[3], pdf, tmax, L[3] */
void orc_kat_light(orc_mt* m, const xrt_light* l, const float* pos, float* out);

/* host libm sinf/cosf (checker for the device restatement) */
void orc_libm_sincosf(const float* x, uint32_t n, float* s, float* c);
void orc_libm_logexpf(const float* x, uint32_t n, float* lg, float* ex);
void orc_libm_powf(const float* x, uint32_t n, float y, float* out);
/* Image::gammaCorrection + writePPM quantisation (Src/image.h:80-114), n floats -> n bytes */
void orc_tonemap(const float* rgb, uint32_t n, float gamma, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
