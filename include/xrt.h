/*
 * xrt.h — C ABI of libxrt_hip.so, the MI355X (gfx950) path-tracing backend that sits
 * behind the reference's Renderer::render() (Src/renderer.h:15).
 *
 * The reference has no FFI: its plugin surface is the C++ virtual class
 *   virtual void Renderer::render(const Scene&, Sampler::SamplerType, Image&) const = 0;
 * (Src/renderer.h:8-20).  A renderer that replaces NormalRenderer / ParallelRenderer
 * (Src/renderer.cpp:8-27, 83-99) needs exactly four things from the caller's objects:
 *   - the scene's objects in Scene::m_objects iteration order (Src/scene.h:45, scene.cpp:190-211),
 *   - the area lights in Scene::m_areaLights order             (Src/scene.h:44, scene.cpp:166-188),
 *   - the pinhole camera (c2w, scale, aspect)                   (Src/camera.h:10-11,37-60),
 *   - the integrator kind and its max depth                     (Src/integrator.h:198-291,76-120,401-478),
 * and it must fill an Image of W*H float3 in place with the per-pixel sample mean
 * (Src/renderer.cpp:29-81,98; Src/image.h:46-78).  Every entry point below maps onto
 * one of those steps.  The C++ HipRenderer (include/xrt/renderer.h) is the
 * reference-side binding; INTEGRATION.md shows it.
 *
 * Conventions: plain C types only; the caller owns all host memory and the library
 * copies what it needs; status 0 = XRT_OK, negative = error (xrt_last_error gives
 * text); no C++ exception crosses this boundary.  A context is used by one host thread.
 * Multi-GPU, two ways: one process per GPU with one context each, rendering row shards
 * (shard_index / shard_count) and reducing the framebuffers over RCCL (the bench); or one
 * process with one context over several GPUs (xrt_create_multi), which shards and
 * assembles the frame itself (ParallelRenderer over the node, Src/renderer.cpp:83-99).
 */
#ifndef XRT_H
#define XRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XRT_ABI_VERSION 12

/* ---- status codes ---------------------------------------------------------------- */
enum {
    XRT_OK = 0,
    XRT_ERR_INVALID = -1,     /* bad argument / inconsistent scene */
    XRT_ERR_HIP = -2,         /* HIP runtime error (no GPU, launch failure, fault) */
    XRT_ERR_STATE = -3,       /* call order: e.g. render before upload */
    XRT_ERR_OOM = -4,         /* device allocation failed */
    XRT_ERR_UNSUPPORTED = -5, /* feature outside the supported set */
    XRT_ERR_IO = -6           /* file could not be read / parsed (Scene::loadObj exit(1)) */
};

/* ---- scene description (flattened Scene) ------------------------------------------ */
enum { XRT_OBJ_MESH = 0, XRT_OBJ_SPHERE = 1, XRT_OBJ_BOX = 2 };
/* XRT_LIGHT_SPHERE: SphereLight::sample's default (cone) branch (Src/light.h:157-197);
 * XRT_LIGHT_SPHERE_AREA: the same light built with AREA_SAMPLING (Src/light.h:131-135,185-191:
 * a uniform point on the sphere, UniformSampleSphere Src/light.cpp:99-105, pdf 2 tmax^3/|d.n|) */
enum { XRT_LIGHT_QUAD = 0, XRT_LIGHT_TRIANGLE = 1, XRT_LIGHT_SPHERE = 2, XRT_LIGHT_SPHERE_AREA = 3 };
enum { XRT_MAT_NONE = 0, XRT_MAT_LAMBERT = 1 };

/* One Object (Src/primitive.h:40-95) in Scene::m_objects iteration order. */
typedef struct {
    int32_t kind;       /* XRT_OBJ_*                                                     */
    int32_t first;      /* first primitive in the kind's array (tris / spheres / boxes)  */
    int32_t count;      /* number of primitives (mesh: triangles; sphere/box: 1)         */
    int32_t material;   /* XRT_MAT_* (Object::m_material != nullptr)                     */
    float albedo[3];    /* Lambert::m_albedo (Src/material.h:76)                         */
    int32_t light;      /* index into lights[] or -1 (Object::m_areaLight)               */
    int32_t medium;     /* 0 = the scene medium, -1 = none (Object::m_medium)            */
} xrt_object;

/* One AreaLight (Src/light.h:54-210) in Scene::m_areaLights order, world space. */
typedef struct {
    int32_t kind;       /* XRT_LIGHT_*                                                   */
    float v0[3];        /* quad / triangle vertices after multVecMatrix(l2w)             */
    float v1[3];
    float v2[3];
    float center[3];    /* sphere light                                                  */
    float radius;
    float Le[3];        /* AreaLight::Le_                                                */
} xrt_light;

typedef struct {
    uint32_t n_objects;
    const xrt_object* objects;
    uint32_t n_tris;
    const float* tri_v;      /* [n_tris][3][3] vertices (Primitive::m_vertices)       */
    const float* tri_n;      /* [n_tris][3][3] vertex normals (Primitive::m_normals)  */
    uint32_t n_spheres;
    const float* spheres;    /* [n_spheres][4] center.xyz, radius                      */
    uint32_t n_boxes;
    const float* boxes;      /* [n_boxes][6] pMin.xyz, pMax.xyz (AABB)                 */
    uint32_t n_lights;
    const xrt_light* lights;
} xrt_scene_desc;

/* The scene medium.  kind XRT_MEDIUM_HETEROGENEOUS: HeterogeneousMedium over a dense
 * density grid standing in for DensityGrid (Src/grid.h:9-15): OpenVDB
 * BoxSampler::wsSample semantics — world -> index by (p - origin) / voxel_size, voxel
 * centres at integer index coordinates, trilinear, background 0 outside the data.
 * The homogeneous kinds (Src/medium.h:122-277) use absorption / scattering as sigma_a /
 * sigma_s (Achromatic: channel 0 of each), bbox as the medium box and g; the grid fields
 * (nx..voxel_size, max_density, density_multiplier) are ignored and density may be NULL. */
enum {
    XRT_MEDIUM_HETEROGENEOUS = 0,          /* HeterogeneousMedium (delta / ratio tracking)  */
    XRT_MEDIUM_HOMOGENEOUS_MIS = 1,        /* HomogeneousMediumMIS (Src/medium.h:148-192)   */
    XRT_MEDIUM_HOMOGENEOUS_ACHROMATIC = 2, /* HomogeneousMediumAchromatic (:195-231)        */
    XRT_MEDIUM_HOMOGENEOUS_NOMIS = 3       /* HomogeneousMediumNoMIS (:234-277)             */
};
typedef struct {
    uint32_t nx, ny, nz;
    const float* density;    /* [nz][ny][nx]                                           */
    float origin[3];         /* world position of index (0,0,0)                         */
    float voxel_size;
    float bbox_min[3];       /* DensityGrid::getBounds() (world)                        */
    float bbox_max[3];
    float max_density;       /* DensityGrid::getMaxDensity()                            */
    float g;                 /* HenyeyGreenstein g                                      */
    float absorption[3];     /* HeterogeneousMedium::absorptionColor                    */
    float scattering[3];     /* HeterogeneousMedium::scatteringColor                    */
    float density_multiplier;
    int32_t kind;            /* XRT_MEDIUM_* (0 when zero-initialised: heterogeneous)   */
} xrt_medium_desc;

/* ---- render parameters --------------------------------------------------------------- */
enum {
    XRT_INTEGRATOR_GI = 0,        /* GIIntegrator(maxDepth)            Src/integrator.h:198-291 */
    XRT_INTEGRATOR_DIRECT = 1,    /* DirectIntegrator                  Src/integrator.h:76-120  */
    XRT_INTEGRATOR_VPT = 2,       /* VolumePathTracing(maxDepth)       Src/integrator.h:401-478 */
    XRT_INTEGRATOR_INDIRECT = 3,  /* IndirectIntegrator(maxDepth)      Src/integrator.h:122-190 */
    XRT_INTEGRATOR_NORMAL = 4,    /* NormalIntegrator (shading normal) Src/integrator.h:22-74   */
    XRT_INTEGRATOR_VPT_NEE = 5    /* VolumePathTracingNEE(maxDepth)    Src/integrator.h:481-636 */
};
enum {
    XRT_FLAG_TIMING = 1u,      /* time every kernel with HIP events (xrt_stats.kernel_ms)     */
    XRT_FLAG_WAVEFRONT = 2u,   /* force the multi-pass schedule (k_shade + k_trace) even when
                                  the scene fits the fused LDS-resident schedule (k_step)     */
    XRT_FLAG_NO_MERGED = 4u,   /* triangle scenes: per-segment cooperative traces (k_step_tri)
                                  instead of the merged shadow + extension traces             */
    XRT_FLAG_NO_GROUP = 8u,    /* merged schedule with 16/32 slots per wave: spread the traces
                                  over idle lanes (pair passes) instead of 4/2-lane groups    */
    XRT_FLAG_DEEP_SINGLE = 32u, /* two-level traces: walk the BVH with one lane per queued ray  */
    XRT_FLAG_DEEP_QUAD = 64u,   /* ... with four lanes per ray (the default); results never
                                   depend on either                                            */
    XRT_FLAG_NO_PIXEL = 128u,   /* Direct / Normal: the per-slot fused schedule (k_step) instead
                                   of pixel-parallel sample chains (k_pixel); same results     */
    XRT_FLAG_NO_SPEC = 256u,    /* GI, one light, small triangle scenes: the merged schedule's
                                   16-slot launches start every sample beside its predecessor's
                                   last trace (k_step_spec, the default); this flag keeps them on
                                   k_step_merged — same results                                */
    XRT_FLAG_ACCUMULATE = 16u  /* Renderer::render's in-place contract (Src/renderer.cpp:75,98):
                                  each owned pixel starts from the value already in the output
                                  buffer (Image::addPixel adds to it in sample order), then
                                  /= spp; pixels of other shards are left untouched.  Without
                                  the flag the buffer is overwritten (zeros outside the shard). */
};

typedef struct {
    int32_t integrator;      /* XRT_INTEGRATOR_*                                        */
    uint32_t max_depth;      /* GIIntegrator / VolumePathTracing m_maxDepth             */
    uint32_t width, height;  /* Image size                                              */
    uint32_t spp;            /* NormalRenderer::n_samples                               */
    uint32_t shard_index;    /* this rank owns image rows y with y % shard_count == idx */
    uint32_t shard_count;    /* 1 = whole image                                         */
    uint32_t flags;          /* XRT_FLAG_*                                              */
    /* launch geometry of the merged schedule; 0 = chosen by the library from the shard's
     * slot count.  Results never depend on these (tests render every layout). */
    uint32_t slots_per_wave;    /* 0, 4, 8, 16, 32 or 64 path slots per 64-lane wave     */
    uint32_t visits_per_launch; /* 0 or 1..128 path segments per slot per step launch    */
} xrt_render_params;

/* kernel families timed in xrt_stats: XRT_K_TRACE is the wavefront trace (for two-level
 * scenes its phase A, the small objects), XRT_K_DEEP the BVH walk of the rays phase A queued */
enum {
    XRT_K_SEED = 0, XRT_K_TRACE = 1, XRT_K_SHADE = 2, XRT_K_FINISH = 3, XRT_K_STEP = 4, XRT_K_REFILL = 5,
    XRT_K_DEEP = 6, XRT_K_COUNT = 7
};

/* device schedules: multi-pass wavefront (k_shade + k_trace), fused per-slot k_step with
 * the scene in LDS, its triangle-scene form with cooperative (ray, triangle) traces, that
 * form with one merged trace (shadow rays + next extension ray) per segment, the merged
 * form for two-level scenes (small objects in LDS, a big mesh's BVH walked by the wave), and
 * for the one-trace integrators (Direct, Normal) pixel-parallel sample chains: one wave per
 * pixel evaluates 64 candidate samples at once and keeps those on the pixel's chain (k_pixel;
 * timed as XRT_K_STEP) */
enum {
    XRT_SCHED_WAVEFRONT = 0, XRT_SCHED_STEP = 1, XRT_SCHED_STEP_TRI = 2, XRT_SCHED_STEP_MERGED = 3,
    XRT_SCHED_STEP_BVH = 4, XRT_SCHED_PIXEL = 5
};

typedef struct {
    double wall_ms;              /* host wall clock of the render call (upload excluded) */
    double kernel_ms[XRT_K_COUNT];   /* summed HIP-event time per kernel (XRT_FLAG_TIMING) */
    uint64_t launches[XRT_K_COUNT];  /* launches per kernel                                */
    uint64_t samples;            /* pixels * spp rendered by this shard                    */
    uint64_t segments;           /* Scene::intersect calls (extension rays traced)         */
    uint64_t shadow_rays;        /* Scene::occluded calls                                  */
    uint64_t draws;              /* RNG draws (Sampler::getNext1D)                         */
    uint64_t rejected;           /* samples dropped by the NaN/Inf/negative check          */
    uint64_t iterations;         /* trace+shade pass pairs, or k_step rounds               */
    uint64_t path_slots;         /* slots in flight (pixels of this shard)                 */
    uint64_t schedule;           /* XRT_SCHED_* the render ran                             */
    uint64_t stalled;            /* paths stopped by the VPT no-progress guard             */
    /* launch geometry the render ran with (merged schedules; 0 otherwise) */
    uint32_t slots_per_wave;     /* path slots per wave of the first step launch            */
    uint32_t group_lanes;        /* lanes sharing one slot's traces (1 = pair passes)      */
    uint32_t partitions;         /* live-list partitions                                   */
    uint32_t visits_per_launch;  /* path segments per slot per step launch                 */
    uint64_t rng_twists;         /* mt19937 blocks generated (624 words each) over all slots,
                                    including each slot's first: rng_twists - path_slots is
                                    the number of ring refills done while paths were live  */
    uint64_t layout_launches[5]; /* merged schedules: step launches per slots-per-wave layout
                                    64, 32, 16, 8, 4 (the layout is re-chosen every launch
                                    from the live count)                                   */
    /* pixel-parallel chains (XRT_SCHED_PIXEL): which of k_pixel's paths ran */
    uint64_t pix_windows;        /* candidate windows evaluated (64 offsets each)           */
    uint64_t pix_stride4;        /* ... of them at stride 4 (after a window of surface hits) */
    uint64_t pix_frustum;        /* pixels whose camera rays tested a camera-frustum list   */
    uint64_t pix_frustum_overflow; /* pixels whose frustum list overflowed (BVH walks)      */
    uint64_t pix_shadow_list;    /* pixels whose shadow rays tested an occluder list        */
    uint64_t pix_shadow_overflow;  /* pixels whose occluder list overflowed (BVH walks)     */
    uint64_t pix_flushes;        /* deferred-shading queue flushes                          */
    uint64_t spec_launches;      /* merged schedule: step launches with speculative starts  */
} xrt_stats;

/* ---- context ----------------------------------------------------------------------- */
typedef struct xrt_ctx xrt_ctx;

int  xrt_abi_version(void);
/* device = HIP device ordinal (one process per GPU: LOCAL_RANK) */
int  xrt_create(int device, xrt_ctx** out);
/* One context over n_devices GPUs (HIP ordinals; a device may be listed twice, e.g. to
 * exercise the multi-GPU path on one GPU).  Every call fans out to all of them; a render
 * gives device i the interleaved rows y % (n * shard_count) == shard_index + shard_count * i
 * (one host thread and HIP stream per device, concurrently) and assembles the frame on
 * devices[0] with one strided peer copy per device — bit-identical to a one-GPU render.
 * xrt_render_device* take a device pointer on devices[0]. */
int  xrt_create_multi(const int* devices, int n_devices, xrt_ctx** out);
int  xrt_device_count(const xrt_ctx* ctx);   /* GPUs a context renders on */
void xrt_destroy(xrt_ctx* ctx);
const char* xrt_last_error(const xrt_ctx* ctx);   /* ctx may be NULL (create failure) */

int  xrt_upload_scene(xrt_ctx* ctx, const xrt_scene_desc* scene);
/* Camera::camera2world (row-major, row-vector convention, Src/geometry.h:486-498),
 * PinholeCamera::scale = tan(0.5*deg2rad(FOV)) and aspect_ratio (Src/camera.h:37-47) */
int  xrt_set_camera(xrt_ctx* ctx, const float c2w[16], float scale, float aspect);
int  xrt_set_medium(xrt_ctx* ctx, const xrt_medium_desc* medium);
/* Sparse heterogeneous density in leaf bricks (the layout NanoVDB / OpenVDB give a grid:
 * 8^3-voxel leaves, Src/examples/nanovdb_convert.cpp, Src/grid.h:22-83).  The grid's
 * index space [0, nx) x [0, ny) x [0, nz) is cut into XRT_BRICK^3 bricks;
 * table[(bz * nby + by) * nbx + bx] is the brick's index in `bricks` or -1 (inactive:
 * background 0, as OpenVDB's BoxSampler reads it).  bricks[b] holds XRT_BRICK^3 floats in
 * [z][y][x] order.  Sampling is the same trilinear BoxSampler as the dense grid, so a brick
 * grid renders bit-identically to the dense grid it was cut from.  medium->density is
 * ignored; every other field of xrt_medium_desc keeps its meaning. */
#define XRT_BRICK 8
typedef struct {
    uint32_t nbx, nby, nbz;      /* bricks per axis: ceil(n / XRT_BRICK)                    */
    const int32_t* table;        /* [nbz][nby][nbx] brick index or -1                        */
    uint32_t n_bricks;
    const float* bricks;         /* [n_bricks][XRT_BRICK^3]                                  */
} xrt_brick_grid;
int  xrt_set_medium_bricks(xrt_ctx* ctx, const xrt_medium_desc* medium, const xrt_brick_grid* grid);

/* Render into caller-owned HOST memory rgb_out[height][width][3] (Image::pixels order
 * j + width*i).  Pixels outside this shard are written as 0.  Blocks until done. */
int  xrt_render(xrt_ctx* ctx, const xrt_render_params* p, float* rgb_out, xrt_stats* st);
/* Same, writing into a DEVICE pointer on this context's GPU (e.g. a torch tensor), so a
 * multi-GPU caller can reduce framebuffers over RCCL without a host round trip.
 * Ordering: the render starts only after all work previously queued on the device has
 * finished (a device-wide wait), so it never overwrites d_rgb_out while a collective or
 * copy issued by the caller still reads it.  Returns after the image is complete. */
int  xrt_render_device(xrt_ctx* ctx, const xrt_render_params* p, float* d_rgb_out, xrt_stats* st);
/* As xrt_render_device, but waits only for the work queued so far on `hip_stream` (a
 * hipStream_t of this context's GPU, e.g. torch.cuda.current_stream().cuda_stream; NULL =
 * the legacy default stream) before touching d_rgb_out. */
int  xrt_render_device_after(xrt_ctx* ctx, const xrt_render_params* p, float* d_rgb_out, void* hip_stream,
                             xrt_stats* st);

/* ---- ray queries: Scene::intersect / Scene::occluded (Src/scene.cpp:190-211) ---------- */
/* One IntersectInfo (Src/ray.h:23-39) as Scene::intersect leaves a fresh one. */
typedef struct {
    int32_t hit;             /* the query's return value                                   */
    int32_t object;          /* hitObject: index in iteration order (-1: none)             */
    int32_t primitive;       /* mesh hits: the object's triangle that set surfaceInfo, else -1 */
    float t;                 /* IntersectInfo::t  (kInfinity = FLT_MAX when nothing wrote it) */
    float t1;                /* IntersectInfo::t1 (medium boxes)                           */
    float position[3], ng[3], ns[3], dpdu[3], dpdv[3];   /* SurfaceInfo                  */
    float barycentric[2];    /* SurfaceInfo::barycentric (u, v) of that triangle           */
} xrt_hit;
enum { XRT_QUERY_INTERSECT = 0, XRT_QUERY_OCCLUDED = 1 };
/* n rays rays[i] = {ox, oy, oz, dx, dy, dz} against the uploaded scene, on the GPU with the
 * render's own trace kernels: XRT_QUERY_INTERSECT fills out[i] like Scene::intersect on a
 * fresh IntersectInfo; XRT_QUERY_OCCLUDED sets out[i].hit = Scene::occluded(ray, tmax[i])
 * (tmax NULL: FLT_MAX) and leaves the other fields zero.  Blocks until done. */
int  xrt_query(xrt_ctx* ctx, uint32_t n, const float* rays, const float* tmax, int32_t mode, xrt_hit* out);

/* Output stage: Image::gammaCorrection(gamma) then writePPM's 8-bit quantisation
 * (Src/image.h:80-114) on the device, for n_pixels float3 pixels: d_rgb is a DEVICE
 * pointer on this context's GPU, or NULL for the framebuffer of the last xrt_render;
 * rgb8_out is caller-owned HOST memory of 3 * n_pixels bytes (the R G B values writePPM
 * prints, in pixel order). */
int  xrt_tonemap(xrt_ctx* ctx, const float* d_rgb, uint32_t n_pixels, float gamma, uint8_t* rgb8_out);

/* ---- host scene layer (C facade over the C++ Scene API; no GPU needed) ------------- */
typedef struct xrt_hscene xrt_hscene;
xrt_hscene* xrt_hscene_create(void);
void xrt_hscene_destroy(xrt_hscene* s);
const char* xrt_hscene_last_error(const xrt_hscene* s);
/* Scene::loadObj (Src/scene.cpp:46-154): OBJ/MTL with tinyobjloader-v2 semantics */
int xrt_hscene_load_obj(xrt_hscene* s, const char* path);
/* Scene::addObj(name, make_unique<Mesh>(prims, Lambert(albedo))); tri_n may be NULL
 * (face normals, as loadObj does when the OBJ has no vn) */
int xrt_hscene_add_mesh(xrt_hscene* s, const char* name, const float* tri_v, const float* tri_n,
                        uint32_t n_tris, const float albedo[3]);
/* SphereMesh(center, radius, nTheta, nPhi, Lambert(albedo)) (Src/primitive.cpp:170-205) */
int xrt_hscene_add_sphere_mesh(xrt_hscene* s, const char* name, const float center[3], float radius,
                               int n_theta, int n_phi, const float albedo[3]);
/* Sphere(center, radius, Lambert(albedo)) (Src/primitive.h:97-184) */
int xrt_hscene_add_sphere(xrt_hscene* s, const char* name, const float center[3], float radius,
                          const float albedo[3]);
/* Scene::addAreaLight(name, QuadLight/TriangleLight/SphereLight(..., Matrix44f(), Le)) */
int xrt_hscene_add_quad_light(xrt_hscene* s, const char* name, const float v0[3], const float v1[3],
                              const float v2[3], const float Le[3]);
int xrt_hscene_add_triangle_light(xrt_hscene* s, const char* name, const float v0[3],
                                  const float v1[3], const float v2[3], const float Le[3]);
int xrt_hscene_add_sphere_light(xrt_hscene* s, const char* name, const float center[3], float radius,
                                const float Le[3]);
/* the same SphereLight as the reference compiled with AREA_SAMPLING (XRT_LIGHT_SPHERE_AREA) */
int xrt_hscene_add_sphere_light_area(xrt_hscene* s, const char* name, const float center[3], float radius,
                                     const float Le[3]);
/* Scene::addObj(name, medium->makeObject()): a BoxMesh over the medium's bounds */
int xrt_hscene_add_medium_box(xrt_hscene* s, const char* name, const float pmin[3], const float pmax[3]);
/* Flatten in unordered_map iteration order.  Pointers stay valid until the next
 * mutation or destroy. */
int xrt_hscene_flatten(xrt_hscene* s, xrt_scene_desc* out);
/* Name of the i-th object in iteration order (NULL if out of range). */
const char* xrt_hscene_object_name(const xrt_hscene* s, uint32_t i);

/* PinholeCamera(aspect, c2w, FOV) -> scale = tan(0.5f*deg2rad(FOV)) (Src/camera.h:45) */
float xrt_pinhole_scale(float fov_deg);

/* ---- device self-tests (used by tests/, never by render) ------------------------- */
/* libstdc++ mt19937 + generate_canonical<float,24> draws for seeds[i], n draws each,
 * taken at stream offset `skip`: out[i*n + k] */
int xrt_test_rng(xrt_ctx* ctx, const uint32_t* seeds, uint32_t n_seeds, uint32_t skip, uint32_t n,
                 float* out);
/* glibc-sinf/cosf restatement on device over x[i]: out[2i] = sinf, out[2i+1] = cosf */
int xrt_test_trig(xrt_ctx* ctx, const float* x, uint32_t n, float* out);
/* exhaustive: count φ = 2π·r over every reachable draw value r where the device
 * restatement differs from the host values supplied by the caller in chunks. */
int xrt_test_trig_draw_domain(xrt_ctx* ctx, uint32_t first_bits, uint32_t count, float* out_sin,
                              float* out_cos, float* out_r);
/* glibc-logf/expf restatement on device over x[i]: out[2i] = logf, out[2i+1] = expf */
int xrt_test_logexp(xrt_ctx* ctx, const float* x, uint32_t n, float* out);
/* glibc-powf restatement on device: out[i] = powf(x[i], y) */
int xrt_test_powf(xrt_ctx* ctx, const float* x, uint32_t n, float y, float* out);
/* every 32-bit input: mode 0 checks the device's fast correctly rounded reciprocal against
 * 1.0f / b, mode 1 its division by the constant c (rc = 1.0f / c) against x / c; returns the
 * mismatch count and up to 16 mismatching inputs (0xffffffff = unused) */
int xrt_test_fastdiv(xrt_ctx* ctx, uint32_t mode, float c, float rc, uint64_t* n_bad, uint32_t* first_bad16);

#ifdef __cplusplus
}
#endif
#endif /* XRT_H */
