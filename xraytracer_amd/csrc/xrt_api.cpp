// xrt_api.cpp — the C ABI of include/xrt.h: device context, scene upload, and the
// wavefront pass schedule that replaces NormalRenderer::render / ParallelRenderer::render
// (Src/renderer.cpp:8-27, 83-99).
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <cfloat>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "bvh.h"
#include "launch.h"
#include "wavefront.h"
#include "xrt.h"
#include "xrt/geometry.h"

using namespace xrt;

static constexpr float kPiF = 3.14159265359;   // Src/geometry.h:10 (float PI), = device_math.h kPI

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct xrt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // scene
    std::vector<DevBuf*> scene_bufs;
    DevBuf tri, tri_ng, tri_nrm, sph, sph_obj, box, objs, lights, segs, density, obj_box, obj_plane, bvh_node,
        bvh_tri, snode, ssph, sbk, sblk, stri, sbox, splane, bvh4;
    KParams base{};
    StepObjs step_objs{};   // kernel-argument object records of the merged-trace schedule
    StepObjs sstep{};       // two-level trace: the small objects' records (KParams::sstep)
    bool has_scene = false, has_camera = false, has_medium = false;
    // slots
    size_t cap_slots = 0;
    DevBuf ray_o, ray_d, thr, rad, thr_prev, hit, hit2, hit3, sh_o, sh_d, sh_c, med, med2, nee;
    DevBuf state, sample_k, depth, occ, rng_c, rng_g, ring, c_seg, c_shadow, c_rej, c_stall, lists, deep, camlist;
    DevBuf counts, stats, fb, scratch, kparams;
    size_t cap_fb = 0;
    uint32_t* h_poll = nullptr;  // pinned
    std::vector<hipEvent_t> events;
    hipEvent_t poll_ev[8] = {};  // live-count polls of render_impl (created once)
    hipEvent_t wait_ev = nullptr;   // xrt_render_device_after: the caller stream's position
    // multi-GPU context (xrt_create_multi): one sub-context per device, each rendering an
    // interleaved row shard; the frame is assembled in subs[0]'s framebuffer
    std::vector<xrt_ctx*> subs;
    // ray queries (xrt_query): per object, its first triangle in the device arrays (-1: not
    // a mesh), and the query's own buffers
    std::vector<int> obj_tri_first;
    DevBuf q_rays, q_tmax, q_out;
    DevBuf brick_table, brick_data;   // sparse medium (xrt_set_medium_bricks)
    DevBuf corners;                   // dense medium: per-cell corner values (DMedium::corners)
    DevBuf stage;              // multi: device-output staging on subs[0] (accumulate from a device image)
};

namespace {

int set_err(xrt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_err(xrt_ctx* c, hipError_t e, const char* what) {
    return set_err(c, XRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(ctx, expr)                                    \
    do {                                                     \
        hipError_t e_ = (expr);                              \
        if (e_ != hipSuccess) return hip_err(ctx, e_, #expr); \
    } while (0)

void free_buf(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

int ensure(xrt_ctx* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return XRT_OK;
    free_buf(b);
    if (bytes == 0) return XRT_OK;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) {
        b.p = nullptr;
        return set_err(c, XRT_ERR_OOM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
    }
    b.bytes = bytes;
    return XRT_OK;
}

int upload(xrt_ctx* c, DevBuf& b, const void* src, size_t bytes) {
    int rc = ensure(c, b, std::max<size_t>(bytes, 16));
    if (rc) return rc;
    if (bytes) HIPCHK(c, hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
    return XRT_OK;
}

template <typename T>
T* as(DevBuf& b) {
    return reinterpret_cast<T*>(b.p);
}

uint32_t shard_rows(uint32_t h, uint32_t idx, uint32_t n) { return idx < h ? (h - idx + n - 1) / n : 0; }

// two-level trace queues (KParams::deep): per partition part_cap extension-ray entries, then
// the shadow rays from entry part_cap on — part_cap per light of the trace kernel, which is
// instantiated for at least one light (an occluded query on a light-less scene queues its
// rays as shadow rays of light 0) — then kMaxParts counts, fetch counters and shadow counts
int setup_deep(xrt_ctx* c, KParams& P) {
    P.deep = nullptr, P.deep_count = nullptr, P.deep_cap = 0;
    if (!P.two_level) return XRT_OK;
    P.deep_cap = P.part_cap * (1u + (uint32_t)std::max(1, P.n_lights));
    const size_t words = (size_t)P.n_part * P.deep_cap + 3 * kMaxParts;   // queues, counts, fetch counters
    const int rc = ensure(c, c->deep, words * 4);
    if (rc) return rc;
    P.deep = as<uint32_t>(c->deep);
    P.deep_count = P.deep + (size_t)P.n_part * P.deep_cap;
    return XRT_OK;
}

// Is the device's div_const(x, c, RN(1/c)) — q = x * rc, q + (x - c q) * rc with two fmas —
// equal to the IEEE quotient x / c for every x it is used on?  Within div_const's window
// (x exponent 25..248) the computation scales exactly with x's exponent (a residual small
// enough to be subnormal is far below ulp(q) / 2 and cannot change the result), so one
// binade decides it: all 2^23 mantissas of x in [1, 2) are compared with the host's IEEE
// division (SSE, correctly rounded).  c is limited to [2^-4, 2^20] so the window's quotients
// stay normal.  About 10 ms per divisor on 8 threads.  Results are cached process-wide
// (all contexts, including the sub-contexts of xrt_create_multi, share one table under a
// mutex, so a multi-GPU render proves each divisor once), and the check uses at most as many
// threads as the process's CPU affinity mask allows (capped at 8).
bool cdiv_exact(xrt_ctx*, float d) {
    if (!(d >= 0x1p-4f && d <= 0x1p20f)) return false;
    uint32_t key;
    std::memcpy(&key, &d, 4);
    static std::mutex mu;
    static std::unordered_map<uint32_t, bool> cache;
    std::lock_guard<std::mutex> lock(mu);   // held during the check: concurrent callers wait for it
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    const float rc = 1.0f / d;
    int nthreads = 1;
    {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        if (sched_getaffinity(0, sizeof(cs), &cs) == 0) nthreads = CPU_COUNT(&cs);
        nthreads = std::max(1, std::min(nthreads, 8));
    }
    std::vector<char> part(nthreads, 1);
    auto work = [&](int t) {
        bool ok = true;
        for (uint32_t m = (uint32_t)t; m < (1u << 23) && ok; m += (uint32_t)nthreads) {
            const uint32_t xb = 0x3f800000u | m;
            float x;
            std::memcpy(&x, &xb, 4);
            const float q = x * rc;
            ok = std::fma(std::fma(-d, q, x), rc, q) == x / d;
        }
        part[t] = ok;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
    work(0);
    bool ok = true;
    for (auto& t : th) t.join();
    for (char p : part) ok &= p != 0;
    cache[key] = ok;
    return ok;
}

// A triangle of an object lying in the plane x_a = c (e1_a = e2_a = 0 exactly) qualifies for
// the exact plane cull (DObjPlane, plane_away in step_tri.hip) when the
// Moller-Trumbore det and t numerator keep the sign of their exact values: with p, q the
// other two axes, both reduce to (d_a resp. o_a - c) * (e1_p e2_q - e1_q e2_p), each product
// rounded twice and the difference once, so |A - B| must exceed a few ulps of |A| + |B|.
// Nonzero edge components within [1e-6, 1e5] keep every product in the normal range for
// |d_a| >= 1e-20 and |o_a - c| >= 1e-25, and below those |det| resp. |t| stays under
// FLT_EPSILON, so the test rejects without the sign argument.
bool plane_tri_ok(const float* e1, const float* e2, int a) {
    if (e1[a] != 0.0f || e2[a] != 0.0f) return false;
    const int p = (a + 1) % 3, q = (a + 2) % 3;
    for (float x : {e1[p], e1[q], e2[p], e2[q]})
        if (x != 0.0f && !(std::fabs(x) >= 1e-6f && std::fabs(x) <= 1e5f)) return false;
    const double A = (double)e1[p] * e2[q], B = (double)e1[q] * e2[p];
    return std::fabs(A - B) > 1e-4 * (std::fabs(A) + std::fabs(B));
}


}  // namespace

extern "C" {

int xrt_abi_version(void) { return XRT_ABI_VERSION; }

int xrt_create(int device, xrt_ctx** out) {
    if (!out) return XRT_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return XRT_ERR_HIP;
    if (device < 0 || device >= n) return XRT_ERR_INVALID;
    xrt_ctx* c = new xrt_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&c->h_poll, 8 * kMaxParts * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->wait_ev, hipEventDisableTiming) != hipSuccess) {
        xrt_destroy(c);
        return XRT_ERR_HIP;
    }
    for (hipEvent_t& e : c->poll_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            xrt_destroy(c);
            return XRT_ERR_HIP;
        }
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess || lds <= 0) {
        xrt_destroy(c);
        return XRT_ERR_HIP;
    }
    c->base.lds_max = (uint32_t)lds;
    *out = c;
    return XRT_OK;
}

void xrt_destroy(xrt_ctx* c) {
    if (!c) return;
    for (xrt_ctx* s : c->subs) xrt_destroy(s);
    c->subs.clear();
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    DevBuf* all[] = {&c->tri, &c->tri_ng, &c->tri_nrm, &c->sph, &c->sph_obj, &c->box, &c->objs, &c->lights,
                     &c->segs, &c->density, &c->obj_box, &c->obj_plane, &c->bvh_node, &c->bvh_tri, &c->snode, &c->ssph, &c->sbk, &c->sblk, &c->ray_o, &c->ray_d, &c->thr, &c->rad, &c->thr_prev, &c->hit,
                     &c->hit2, &c->hit3, &c->sh_o, &c->sh_d, &c->sh_c, &c->med, &c->med2, &c->nee, &c->state,
                     &c->sample_k, &c->depth, &c->occ, &c->rng_c, &c->rng_g, &c->ring, &c->c_seg, &c->c_shadow,
                     &c->c_rej, &c->c_stall, &c->lists, &c->counts, &c->stats, &c->fb, &c->scratch, &c->kparams};
    for (DevBuf* b : all) free_buf(*b);
    free_buf(c->stri), free_buf(c->sbox), free_buf(c->splane), free_buf(c->bvh4), free_buf(c->deep);
    free_buf(c->stage), free_buf(c->q_rays), free_buf(c->q_tmax), free_buf(c->q_out);
    free_buf(c->brick_table), free_buf(c->brick_data), free_buf(c->corners), free_buf(c->camlist);
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->poll_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->wait_ev) (void)hipEventDestroy(c->wait_ev);
    if (c->h_poll) (void)hipHostFree(c->h_poll);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* xrt_last_error(const xrt_ctx* c) { return c ? c->err.c_str() : "no context (xrt_create failed: no HIP device?)"; }

// Flattened Scene -> device layout.  Primitives are re-packed in object iteration order,
// so the linear scan order equals Scene::intersect's order (Src/scene.cpp:190-200).
static int upload_scene_one(xrt_ctx* c, const xrt_scene_desc* s) {
    if (!c || !s) return XRT_ERR_INVALID;
    // a failed upload (OOM, bad range) must not leave the previous scene's freed buffers
    // behind a valid-looking context: renders are refused until an upload completes
    c->has_scene = false;
    HIPCHK(c, hipSetDevice(c->device));
    if (s->n_lights > (uint32_t)kMaxLights)
        return set_err(c, XRT_ERR_UNSUPPORTED, "more than " + std::to_string(kMaxLights) + " area lights");
    if ((s->n_objects && !s->objects) || (s->n_lights && !s->lights))
        return set_err(c, XRT_ERR_INVALID, "null scene arrays");
    std::vector<f4> tri, tri_ng, tri_nrm, sph, box;
    std::vector<int> sph_obj;
    std::vector<DObj> objs;
    std::vector<DSeg> segs;
    std::vector<int> tri_first(s->n_objects, -1);
    std::vector<DObjPlane> planes(s->n_objects, DObjPlane{-1, 0.0f});
    auto V = [](const float* p) { return Vec3f(p[0], p[1], p[2]); };
    auto F4 = [](const Vec3f& v, float w) { return f4{v[0], v[1], v[2], w}; };
    auto bits = [](int x) { float f; std::memcpy(&f, &x, 4); return f; };
    double emax = 0.0;   // largest |e1| |e2| of a triangle (bounds |det| of every ray test)
    for (uint32_t k = 0; k < s->n_objects; ++k) {
        const xrt_object& o = s->objects[k];
        if (o.light >= (int)s->n_lights || o.count < 0 || o.first < 0)
            return set_err(c, XRT_ERR_INVALID, "object " + std::to_string(k) + ": bad light index or range");
        DObj d{};
        d.kind = o.kind, d.material = o.material, d.light = o.light, d.medium = o.medium;
        for (int q = 0; q < 3; ++q) d.fr[q] = o.material == 1 ? o.albedo[q] / kPiF : 0.0f;
        objs.push_back(d);
        const bool occluder = o.light < 0;  // Scene::occluded skips area-light objects
        int kind = -1, first = 0;
        uint32_t axes = 0;   // meshes: DObjPlane candidates
        if (o.kind == XRT_OBJ_MESH) {
            if ((uint64_t)o.first + o.count > s->n_tris || (o.count && (!s->tri_v || !s->tri_n)))
                return set_err(c, XRT_ERR_INVALID, "mesh range out of bounds");
            kind = SEG_TRI;
            first = (int)(tri.size() / 3);
            tri_first[k] = first;
            axes = o.count > 0 ? 7u : 0u;   // axes on which every vertex so far shares v[0]'s coordinate
            const float* vfirst = s->tri_v + 9 * (size_t)o.first;
            for (int t = o.first; t < o.first + o.count; ++t) {
                const float* v = s->tri_v + 9 * (size_t)t;
                const float* n = s->tri_n + 9 * (size_t)t;
                const Vec3f v0 = V(v), v1 = V(v + 3), v2 = V(v + 6);
                const Vec3f e1 = v1 - v0, e2 = v2 - v0;     // Src/primitive.cpp:142-143
                emax = std::max(emax, std::sqrt((double)dot(e1, e1) * (double)dot(e2, e2)));
                for (int a = 0; a < 3; ++a)
                    if (!(v[a] == vfirst[a] && v[3 + a] == vfirst[a] && v[6 + a] == vfirst[a]) ||
                        !plane_tri_ok(e1.getPtr(), e2.getPtr(), a))
                        axes &= ~(1u << a);
                tri.push_back(F4(v0, bits((int)k)));
                tri.push_back(F4(e1, occluder ? 1.0f : 0.0f));
                tri.push_back(F4(e2, 0.0f));
                tri_ng.push_back(F4(normalize(cross(e1, e2)), 0.0f));   // Src/primitive.cpp:106
                tri_nrm.push_back(F4(V(n), 0.0f));
                tri_nrm.push_back(F4(V(n + 3), 0.0f));
                tri_nrm.push_back(F4(V(n + 6), 0.0f));
            }
        } else if (o.kind == XRT_OBJ_SPHERE) {
            if ((uint64_t)o.first + o.count > s->n_spheres || !s->spheres)
                return set_err(c, XRT_ERR_INVALID, "sphere range out of bounds");
            kind = SEG_SPHERE;
            first = (int)sph.size();
            for (int t = o.first; t < o.first + o.count; ++t) {
                const float* p = s->spheres + 4 * (size_t)t;
                sph.push_back(f4{p[0], p[1], p[2], p[3]});
                sph_obj.push_back((int)k | (occluder ? (1 << 30) : 0));
            }
        } else if (o.kind == XRT_OBJ_BOX) {
            if ((uint64_t)o.first + o.count > s->n_boxes || !s->boxes)
                return set_err(c, XRT_ERR_INVALID, "box range out of bounds");
            kind = SEG_BOX;
            first = (int)(box.size() / 2);
            for (int t = o.first; t < o.first + o.count; ++t) {
                const float* p = s->boxes + 6 * (size_t)t;
                box.push_back(f4{p[0], p[1], p[2], bits((int)k)});
                box.push_back(f4{p[3], p[4], p[5], 0.0f});
            }
        } else {
            return set_err(c, XRT_ERR_INVALID, "unknown object kind");
        }
        if (kind == SEG_TRI && o.count > 0) {
            for (int a = 0; a < 3; ++a)
                if ((axes >> a) & 1u) {
                    planes[k] = DObjPlane{a, s->tri_v[9 * (size_t)o.first + a]};
                    break;
                }
        }
        if (o.count == 0) continue;
        if (!segs.empty() && segs.back().kind == kind && segs.back().first + segs.back().count == first)
            segs.back().count += o.count;
        else
            segs.push_back(DSeg{kind, first, o.count, 0});
    }
    std::vector<DLight> lights;
    for (uint32_t l = 0; l < s->n_lights; ++l) {
        const xrt_light& L = s->lights[l];
        if (L.kind < XRT_LIGHT_QUAD || L.kind > XRT_LIGHT_SPHERE_AREA)
            return set_err(c, XRT_ERR_INVALID, "light " + std::to_string(l) + ": unknown kind");
        DLight d{};
        d.kind = L.kind;
        const Vec3f v0 = V(L.v0), v1 = V(L.v1), v2 = V(L.v2);
        const Vec3f e1 = v1 - v0, e2 = v2 - v0, Ng = cross(e1, e2);   // QuadLight/TriangleLight ctor
        for (int q = 0; q < 3; ++q) {
            d.v0[q] = v0[q], d.v1[q] = v1[q], d.v2[q] = v2[q];
            d.e1[q] = e1[q], d.e2[q] = e2[q], d.Ng[q] = Ng[q];
            d.center[q] = L.center[q], d.Le[q] = L.Le[q];
        }
        d.radius = L.radius;
        lights.push_back(d);
    }
    int rc;
    if ((rc = upload(c, c->tri, tri.data(), tri.size() * sizeof(f4))) ||
        (rc = upload(c, c->tri_ng, tri_ng.data(), tri_ng.size() * sizeof(f4))) ||
        (rc = upload(c, c->tri_nrm, tri_nrm.data(), tri_nrm.size() * sizeof(f4))) ||
        (rc = upload(c, c->sph, sph.data(), sph.size() * sizeof(f4))) ||
        (rc = upload(c, c->sph_obj, sph_obj.data(), sph_obj.size() * sizeof(int))) ||
        (rc = upload(c, c->box, box.data(), box.size() * sizeof(f4))) ||
        (rc = upload(c, c->objs, objs.data(), objs.size() * sizeof(DObj))) ||
        (rc = upload(c, c->lights, lights.data(), lights.size() * sizeof(DLight))) ||
        (rc = upload(c, c->segs, segs.data(), segs.size() * sizeof(DSeg))))
        return rc;
    KParams& P = c->base;
    P.tri = as<f4>(c->tri), P.tri_ng = as<f4>(c->tri_ng), P.tri_nrm = as<f4>(c->tri_nrm);
    P.sph = as<f4>(c->sph), P.sph_obj = as<int>(c->sph_obj), P.box = as<f4>(c->box);
    P.objs = as<DObj>(c->objs), P.lights = as<DLight>(c->lights), P.segs = as<DSeg>(c->segs);
    P.n_segs = (int)segs.size(), P.n_lights = (int)lights.size();
    P.n_tris = (int)(tri.size() / 3), P.n_sph = (int)sph.size(), P.n_box = (int)(box.size() / 2);
    bool only_tri = true, only_sph = true;
    for (const DSeg& g : segs) only_tri &= g.kind == SEG_TRI, only_sph &= g.kind == SEG_SPHERE;
    P.scene_kind = (only_tri || segs.empty()) ? SCN_TRI : (only_sph ? SCN_SPHERE : SCN_MIXED);
    // small triangle scenes: per-object culling boxes for k_trace_small.  Margin: 1e-3 of
    // the scene diagonal + 1e-3, orders of magnitude above the float error of a
    // Moller-Trumbore hit position, so culling never removes a hit the linear scan accepts.
    P.small_tri = 0;
    P.n_objs = (int)objs.size();
    // |det| = |e1 . (d x e2)| <= |e1| |e2| |d| with |d| = 1 (+ a few ulp) for every traced ray,
    // so below 2^120 every finite det is either < kEPSILON (rejected whatever 1/det is) or in
    // rcp_newton's exact range: ray_tri_nb then skips the IEEE fallback (det_bounded).
    P.det_bounded = emax < 0x1p120 ? 1 : 0;   // NaN / inf edges: false
    if (P.scene_kind == SCN_TRI && P.n_tris <= kSmallTris && P.n_objs <= kSmallObjs && P.n_tris > 0) {
        float lo[3] = {3e38f, 3e38f, 3e38f}, hi[3] = {-3e38f, -3e38f, -3e38f};
        std::vector<DObjBox> boxes(objs.size());
        int tri_first = 0;
        for (size_t k = 0; k < objs.size(); ++k) {
            DObjBox& b = boxes[k];
            const int cnt = s->objects[k].count;
            b.first = tri_first;
            b.count_occ = cnt | (objs[k].light < 0 ? (int)0x80000000 : 0);
            for (int q = 0; q < 3; ++q) b.bmin[q] = 3e38f, b.bmax[q] = -3e38f;
            for (int t = tri_first; t < tri_first + cnt; ++t) {
                const f4 v0 = tri[3 * t], e1 = tri[3 * t + 1], e2 = tri[3 * t + 2];
                const float vs[3][3] = {{v0.x, v0.y, v0.z}, {v0.x + e1.x, v0.y + e1.y, v0.z + e1.z},
                                        {v0.x + e2.x, v0.y + e2.y, v0.z + e2.z}};
                for (int a = 0; a < 3; ++a)
                    for (int q = 0; q < 3; ++q) b.bmin[q] = std::min(b.bmin[q], vs[a][q]), b.bmax[q] = std::max(b.bmax[q], vs[a][q]);
            }
            for (int q = 0; q < 3; ++q) lo[q] = std::min(lo[q], b.bmin[q]), hi[q] = std::max(hi[q], b.bmax[q]);
            tri_first += cnt;
        }
        const float diag = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                     (hi[2] - lo[2]) * (hi[2] - lo[2]));
        const float margin = 1e-3f * diag + 1e-3f;
        for (DObjBox& b : boxes)
            for (int q = 0; q < 3; ++q) b.bmin[q] -= margin, b.bmax[q] += margin;
        if ((rc = upload(c, c->obj_box, boxes.data(), boxes.size() * sizeof(DObjBox))) ||
            (rc = upload(c, c->obj_plane, planes.data(), planes.size() * sizeof(DObjPlane))))
            return rc;
        P.obj_box = as<DObjBox>(c->obj_box);
        P.obj_plane = as<DObjPlane>(c->obj_plane);
        if (boxes.size() <= (size_t)kMergedMaxObjs)
            build_step_objs(boxes.data(), planes.data(), (int)boxes.size(), c->step_objs);
        P.small_tri = 1;
    }
    // large triangle scenes: a BVH for the wavefront trace (C4's 51k-triangle sphere mesh).
    // Margin: 1e-4 of the scene diagonal + 1e-4, above the float error of a Moller-Trumbore
    // hit position, so box tests never drop a hit the linear scan accepts.
    P.bvh_node = nullptr, P.bvh_tri = nullptr, P.bvh_stack = 0, P.bvh_nodes = 0;
    P.stri = nullptr, P.sbox = nullptr, P.splane = nullptr, P.n_stri = 0, P.n_sobj = 0, P.two_level = 0;
    P.sstep = nullptr, P.bvh4 = nullptr, P.bvh4_nodes = 0, P.bvh4_stack = 0, P.deep_quad = 0;
    if (P.scene_kind == SCN_TRI && !P.small_tri && P.n_tris > 0 && !exp_env("XRT_NO_BVH")) {
        // two-level split: mesh objects of more than kLargeObjTris triangles go into the BVH,
        // the rest (if any, and if they fit the LDS scan) are scanned directly
        std::vector<uint32_t> big;   // original indices of the BVH's triangles
        std::vector<DObjBox> sboxes;
        std::vector<DObjPlane> splanes;
        std::vector<f4> stri;
        {
            int t0 = 0;
            for (size_t k = 0; k < objs.size(); ++k) {
                const int cnt = s->objects[k].count;
                if (cnt > kLargeObjTris) {
                    for (int t = t0; t < t0 + cnt; ++t) big.push_back((uint32_t)t);
                } else if (cnt > 0) {
                    DObjBox b;
                    b.first = (int)(stri.size() / 3);
                    b.count_occ = cnt | (objs[k].light < 0 ? (int)0x80000000 : 0);
                    for (int t = t0; t < t0 + cnt; ++t) {
                        stri.push_back(tri[3 * t]), stri.push_back(tri[3 * t + 1]), stri.push_back(tri[3 * t + 2]);
                        stri.back().w = bits(t);
                    }
                    sboxes.push_back(b);
                    splanes.push_back(planes[k]);
                }
                t0 += cnt;
            }
        }
        const bool two = !big.empty() && !sboxes.empty() && stri.size() / 3 <= (size_t)kSmallTris &&
                         sboxes.size() <= (size_t)kSmallObjs && !exp_env("XRT_NO_TWO_LEVEL");
        if (!two) {
            big.resize(P.n_tris);
            for (size_t t = 0; t < big.size(); ++t) big[t] = (uint32_t)t;
        }
        // A triangle with an exactly zero edge vector (two equal vertices, e.g. half of a
        // SphereMesh's pole cells) is rejected by every Moller-Trumbore test: e1 = 0 makes
        // det = e1 . pvec an exact 0, e2 = 0 makes pvec = d x e2 an exact 0 (a NaN direction
        // fails t > eps instead) — so it is left out of the BVH, where its box would overlap
        // every other pole triangle's.
        {
            auto zero = [](const f4& e) { return e.x == 0.0f && e.y == 0.0f && e.z == 0.0f; };
            size_t w = 0;
            for (size_t i = 0; i < big.size(); ++i)
                if (!zero(tri[3 * big[i] + 1]) && !zero(tri[3 * big[i] + 2])) big[w++] = big[i];
            if (w > 0) big.resize(w);
        }
        const size_t nt = big.size();
        std::vector<float> mn(3 * nt), mx(3 * nt);
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        auto tri_box = [&](size_t t, float* bmn, float* bmx) {
            const f4 v0 = tri[3 * t], e1 = tri[3 * t + 1], e2 = tri[3 * t + 2];
            const float vs[3][3] = {{v0.x, v0.y, v0.z}, {v0.x + e1.x, v0.y + e1.y, v0.z + e1.z},
                                    {v0.x + e2.x, v0.y + e2.y, v0.z + e2.z}};
            for (int q = 0; q < 3; ++q) {
                bmn[q] = std::min({vs[0][q], vs[1][q], vs[2][q]});
                bmx[q] = std::max({vs[0][q], vs[1][q], vs[2][q]});
                lo[q] = std::min(lo[q], bmn[q]), hi[q] = std::max(hi[q], bmx[q]);
            }
        };
        for (size_t i = 0; i < nt; ++i) tri_box(big[i], &mn[3 * i], &mx[3 * i]);
        if (two) {   // small objects' boxes (the scene diagonal covers them too)
            for (DObjBox& b : sboxes) {
                for (int q = 0; q < 3; ++q) b.bmin[q] = 3e38f, b.bmax[q] = -3e38f;
                for (int i = b.first; i < b.first + (b.count_occ & 0x7fffffff); ++i) {
                    float bmn[3], bmx[3];
                    tri_box((size_t)__builtin_bit_cast(int, stri[3 * i + 2].w), bmn, bmx);
                    for (int q = 0; q < 3; ++q) b.bmin[q] = std::min(b.bmin[q], bmn[q]), b.bmax[q] = std::max(b.bmax[q], bmx[q]);
                }
            }
        }
        const float diag = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                     (hi[2] - lo[2]) * (hi[2] - lo[2]));
        if (two) {
            // culling margin of the small-scene scan (1e-3 of the diagonal + 1e-3, see above)
            const float margin = 1e-3f * diag + 1e-3f;
            for (DObjBox& b : sboxes)
                for (int q = 0; q < 3; ++q) b.bmin[q] -= margin, b.bmax[q] += margin;
            if ((rc = upload(c, c->stri, stri.data(), stri.size() * sizeof(f4))) ||
                (rc = upload(c, c->sbox, sboxes.data(), sboxes.size() * sizeof(DObjBox))) ||
                (rc = upload(c, c->splane, splanes.data(), splanes.size() * sizeof(DObjPlane))))
                return rc;
            P.stri = as<f4>(c->stri), P.sbox = as<DObjBox>(c->sbox), P.splane = as<DObjPlane>(c->splane);
            P.n_stri = (int)(stri.size() / 3), P.n_sobj = (int)sboxes.size(), P.two_level = 1;
            if (sboxes.size() <= (size_t)kMergedMaxObjs) {   // phase A as cooperative pair passes
                build_step_objs(sboxes.data(), splanes.data(), (int)sboxes.size(), c->sstep);
                P.sstep = P.det_bounded ? &c->sstep : nullptr;   // k_trace_2a_coop: ray_tri_nb
            }
        }
        const BvhBuild B = build_bvh(mn.data(), mx.data(), (uint32_t)nt, kBvhLeafTri, 1e-4f * diag + 1e-4f, kBvhMaxDepth);
        if (B.depth >= kBvhStack) return set_err(c, XRT_ERR_UNSUPPORTED, "BVH deeper than the traversal stack");
        std::vector<f4> btri(3 * nt);
        for (size_t i = 0; i < nt; ++i) {
            const uint32_t t = big[B.order[i]];
            btri[3 * i] = tri[3 * t], btri[3 * i + 1] = tri[3 * t + 1], btri[3 * i + 2] = tri[3 * t + 2];
            btri[3 * i + 2].w = bits((int)t);
        }
        if ((rc = upload(c, c->bvh_node, B.nodes.data(), B.nodes.size() * sizeof(BvhNode))) ||
            (rc = upload(c, c->bvh_tri, btri.data(), btri.size() * sizeof(f4))))
            return rc;
        P.bvh_node = as<f4>(c->bvh_node), P.bvh_tri = as<f4>(c->bvh_tri);
        P.bvh_stack = B.depth + 1;
        P.bvh_nodes = (int)B.nodes.size();
        if (P.two_level) {   // the deep rays walk the 4-wide form
            int d4 = 0;
            const std::vector<Bvh4Node> b4 = collapse_bvh4(B, d4);
            if (3 * d4 + 1 > kBvh4Stack) return set_err(c, XRT_ERR_UNSUPPORTED, "4-wide BVH deeper than the traversal stack");
            if ((rc = upload(c, c->bvh4, b4.data(), b4.size() * sizeof(Bvh4Node)))) return rc;
            P.bvh4 = as<f4>(c->bvh4), P.bvh4_nodes = (int)b4.size(), P.bvh4_stack = 3 * d4 + 1;
        }
    }
    // sphere scenes (C3's 1001 spheres): a threaded BVH for the fused schedule's traces.
    // Sphere boxes: center +- radius, padded by 1e-4 of the scene diagonal + 1e-4 —
    // far above the float error of Sphere::intersect's hit point (and of its
    // near-tangent discriminant), so a box test never drops a hit the linear scan accepts.
    P.snode = nullptr, P.ssph = nullptr, P.sbk = nullptr, P.sblk = nullptr, P.n_snode = 0, P.sph_pad = 0.0f;
    if (P.scene_kind == SCN_SPHERE && P.n_sph >= kSphBvhMin && !exp_env("XRT_NO_BVH")) {
        const size_t ns = (size_t)P.n_sph;
        std::vector<float> mn(3 * ns), mx(3 * ns);
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t k = 0; k < ns; ++k) {
            const float cc[3] = {sph[k].x, sph[k].y, sph[k].z}, r = std::fabs(sph[k].w);
            for (int q = 0; q < 3; ++q) {
                mn[3 * k + q] = cc[q] - r, mx[3 * k + q] = cc[q] + r;
                lo[q] = std::min(lo[q], mn[3 * k + q]), hi[q] = std::max(hi[q], mx[3 * k + q]);
            }
        }
        const float diag = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                     (hi[2] - lo[2]) * (hi[2] - lo[2]));
        P.sph_pad = 1e-4f * diag + 1e-4f;
        const BvhBuild B = build_bvh(mn.data(), mx.data(), (uint32_t)ns, kBvhLeaf, P.sph_pad, kBvhMaxDepth);
        const std::vector<SkipNode> T = thread_bvh(B);
        std::vector<f4> bs(ns);
        std::vector<int> bk(ns);
        for (size_t i = 0; i < ns; ++i) {
            const uint32_t k = B.order[i];
            bs[i] = sph[k];
            bk[i] = (int)k | (sph_obj[k] & (1 << 30));
        }
        // a ball around every 64 consecutive spheres of the leaf order (spatially coherent
        // blocks): it contains each member's ball of radius |r| + sph_pad, so the pixel
        // schedule's list scans skip a block whose ball misses the region (pixel.hip)
        std::vector<f4> blk((ns + 63) / 64);
        for (size_t b = 0; b < blk.size(); ++b) {
            const size_t i0 = 64 * b, i1 = std::min(ns, i0 + 64);
            double lo3[3] = {1e300, 1e300, 1e300}, hi3[3] = {-1e300, -1e300, -1e300};
            for (size_t i = i0; i < i1; ++i)
                for (int q = 0; q < 3; ++q) {
                    const double cq = q == 0 ? bs[i].x : q == 1 ? bs[i].y : bs[i].z;
                    lo3[q] = std::min(lo3[q], cq), hi3[q] = std::max(hi3[q], cq);
                }
            const double C[3] = {0.5 * (lo3[0] + hi3[0]), 0.5 * (lo3[1] + hi3[1]), 0.5 * (lo3[2] + hi3[2])};
            const float Cf[3] = {(float)C[0], (float)C[1], (float)C[2]};
            double R = 0.0;
            for (size_t i = i0; i < i1; ++i) {
                const double dx = (double)bs[i].x - Cf[0], dy = (double)bs[i].y - Cf[1], dz = (double)bs[i].z - Cf[2];
                R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + std::fabs((double)bs[i].w));
            }
            blk[b] = f4{Cf[0], Cf[1], Cf[2], (float)(R * (1.0 + 1e-5)) + P.sph_pad};
        }
        if ((rc = upload(c, c->snode, T.data(), T.size() * sizeof(SkipNode))) ||
            (rc = upload(c, c->ssph, bs.data(), bs.size() * sizeof(f4))) ||
            (rc = upload(c, c->sbk, bk.data(), bk.size() * sizeof(int))) ||
            (rc = upload(c, c->sblk, blk.data(), blk.size() * sizeof(f4))))
            return rc;
        P.snode = as<f4>(c->snode), P.ssph = as<f4>(c->ssph), P.sbk = as<int>(c->sbk);
        P.sblk = as<f4>(c->sblk);
        P.n_snode = (int)T.size();
    }
    c->obj_tri_first = std::move(tri_first);
    c->has_scene = true;
    return XRT_OK;
}

static int set_camera_one(xrt_ctx* c, const float c2w[16], float scale, float aspect) {
    if (!c || !c2w) return XRT_ERR_INVALID;
    std::memcpy(c->base.c2w, c2w, sizeof(float) * 16);
    c->base.scale = scale;
    c->base.aspect = aspect;
    c->has_camera = true;
    return XRT_OK;
}

static int set_medium_grid(xrt_ctx* c, const xrt_medium_desc* m);

static int set_medium_one(xrt_ctx* c, const xrt_medium_desc* m) {
    if (!c || !m) return XRT_ERR_INVALID;
    if (m->kind != XRT_MEDIUM_HETEROGENEOUS) {
        // HomogeneousMedium{MIS, Achromatic, NoMIS} (Src/medium.h:122-277): sigma_t = a + s
        if (m->kind > XRT_MEDIUM_HOMOGENEOUS_NOMIS || m->kind < 0) return set_err(c, XRT_ERR_INVALID, "bad medium kind");
        DMedium& D = c->base.medium;
        D = DMedium{};
        D.kind = m->kind;
        D.g = m->g;
        const Vec3f a(m->absorption[0], m->absorption[1], m->absorption[2]);
        const Vec3f sc(m->scattering[0], m->scattering[1], m->scattering[2]);
        const Vec3f t = a + sc;
        for (int q = 0; q < 3; ++q) D.absorption[q] = a[q], D.scattering[q] = sc[q], D.sigma_t[q] = t[q];
        c->has_medium = true;
        return XRT_OK;
    }
    if (!m->density || !m->nx || !m->ny || !m->nz) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t n = (size_t)m->nx * m->ny * m->nz;
    int rc = upload(c, c->density, m->density, n * sizeof(float));
    if (rc) return rc;
    DMedium& D = c->base.medium;
    D = DMedium{};
    D.density = as<float>(c->density);
    // the per-cell corner layout (8x the grid's bytes; skipped above 2 GiB).  It is only an
    // acceleration: when the host copy or the device buffer cannot be had, the medium reads
    // the dense grid's rows instead (D.corners = null), with identical results.
    const size_t cx = m->nx - 1, cy = m->ny - 1, cz = m->nz - 1, cells = cx * cy * cz;
    free_buf(c->corners);
    if (XRT_CORNER_GRID && cells && cells * 32 <= (size_t(2) << 30)) {
        std::vector<float> cor;
        try {
            cor.resize(cells * 8);
        } catch (const std::bad_alloc&) {
            cor.clear();
        }
        if (!cor.empty()) {
            const float* g = m->density;
            const size_t sy = m->nx, sz = (size_t)m->nx * m->ny;
            for (size_t k = 0; k < cz; ++k)
                for (size_t j = 0; j < cy; ++j)
                    for (size_t i = 0; i < cx; ++i) {
                        const float* b = g + k * sz + j * sy + i;
                        float* o = cor.data() + 8 * ((k * cy + j) * cx + i);
                        o[0] = b[0], o[1] = b[sz], o[2] = b[sy], o[3] = b[sy + sz];
                        o[4] = b[1], o[5] = b[1 + sz], o[6] = b[1 + sy], o[7] = b[1 + sy + sz];
                    }
            if (upload(c, c->corners, cor.data(), cor.size() * sizeof(float)) == XRT_OK) {
                D.corners = as<float>(c->corners);
            } else {
                free_buf(c->corners);
                (void)hipGetLastError();
                c->err.clear();
            }
        }
    }
    return set_medium_grid(c, m);
}

// the grid-independent part of a heterogeneous medium (dense or bricks)
static int set_medium_grid(xrt_ctx* c, const xrt_medium_desc* m) {
    DMedium& D = c->base.medium;
    D.nx = (int)m->nx, D.ny = (int)m->ny, D.nz = (int)m->nz;
    for (int q = 0; q < 3; ++q) {
        D.origin[q] = m->origin[q];
        D.absorption[q] = m->absorption[q];
        D.scattering[q] = m->scattering[q];
    }
    D.voxel_size = m->voxel_size;
    D.inv_voxel = 1.0 / (double)m->voxel_size;
    D.multiplier = m->density_multiplier;
    D.g = m->g;
    D.kind = XRT_MEDIUM_HETEROGENEOUS;
    // HeterogeneousMedium ctor (Src/medium.cpp:5-17)
    const float max_density = m->density_multiplier * m->max_density;
    const Vec3f a(m->absorption[0], m->absorption[1], m->absorption[2]);
    const Vec3f sc(m->scattering[0], m->scattering[1], m->scattering[2]);
    const Vec3f mm = a * max_density + sc * max_density;
    D.majorant = std::max(mm[0], std::max(mm[1], mm[2]));
    D.inv_majorant = 1.0f / D.majorant;
    c->has_medium = true;
    return XRT_OK;
}

// Sparse heterogeneous density in XRT_BRICK^3 leaf bricks (the NanoVDB / OpenVDB leaf
// layout): the same trilinear BoxSampler as the dense grid, reading voxels through the brick
// table (medium_density), so inactive regions cost no memory.
static int set_medium_bricks_one(xrt_ctx* c, const xrt_medium_desc* m, const xrt_brick_grid* g) {
    if (!c || !m || !g) return XRT_ERR_INVALID;
    if (m->kind != XRT_MEDIUM_HETEROGENEOUS) return set_err(c, XRT_ERR_INVALID, "brick grids are heterogeneous media");
    if (!m->nx || !m->ny || !m->nz || !g->table || (g->n_bricks && !g->bricks) || g->nbx != (m->nx + 7) / 8 ||
        g->nby != (m->ny + 7) / 8 || g->nbz != (m->nz + 7) / 8)
        return set_err(c, XRT_ERR_INVALID, "brick table dimensions do not match the grid (ceil(n / 8) per axis)");
    const size_t nt = (size_t)g->nbx * g->nby * g->nbz;
    for (size_t i = 0; i < nt; ++i)
        if (g->table[i] < -1 || g->table[i] >= (int32_t)g->n_bricks)
            return set_err(c, XRT_ERR_INVALID, "brick table entry out of range");
    HIPCHK(c, hipSetDevice(c->device));
    int rc;
    if ((rc = upload(c, c->brick_table, g->table, nt * sizeof(int32_t))) ||
        (rc = upload(c, c->brick_data, g->bricks, (size_t)g->n_bricks * 512 * sizeof(float))))
        return rc;
    DMedium& D = c->base.medium;
    D = DMedium{};
    D.brick_table = as<int>(c->brick_table);
    D.bricks = as<float>(c->brick_data);
    D.nbx = (int)g->nbx, D.nby = (int)g->nby, D.nbz = (int)g->nbz;
    return set_medium_grid(c, m);
}

int xrt_set_medium_bricks(xrt_ctx* c, const xrt_medium_desc* m, const xrt_brick_grid* g) {
    if (!c || c->subs.empty()) return set_medium_bricks_one(c, m, g);
    for (xrt_ctx* d : c->subs) {
        const int rc = set_medium_bricks_one(d, m, g);
        if (rc) return set_err(c, rc, "xrt_set_medium_bricks on device " + std::to_string(d->device) + ": " + d->err);
    }
    return XRT_OK;
}

// wait: 0 = none (host output: the library owns the framebuffer), 1 = the whole device
// (xrt_render_device), 2 = the caller's stream `wait_stream` (xrt_render_device_after)
static int render_impl(xrt_ctx* c, const xrt_render_params* p, float* d_out, float* h_out, xrt_stats* st,
                       int wait = 0, hipStream_t wait_stream = nullptr) {
    const auto t_start = std::chrono::steady_clock::now();
    if (!c || !p) return XRT_ERR_INVALID;
    if (!c->has_scene || !c->has_camera) return set_err(c, XRT_ERR_STATE, "upload a scene and set a camera first");
    if (p->width == 0 || p->height == 0 || p->shard_count == 0 || p->shard_index >= p->shard_count)
        return set_err(c, XRT_ERR_INVALID, "bad image size or shard");
    if (p->integrator < XRT_INTEGRATOR_GI || p->integrator > XRT_INTEGRATOR_VPT_NEE)
        return set_err(c, XRT_ERR_INVALID, "unknown integrator");
    const bool volumetric = p->integrator == XRT_INTEGRATOR_VPT || p->integrator == XRT_INTEGRATOR_VPT_NEE;
    if (volumetric && !c->has_medium)
        return set_err(c, XRT_ERR_STATE, "VolumePathTracing needs xrt_set_medium first");
    if (p->integrator == XRT_INTEGRATOR_VPT_NEE && c->base.n_lights == 0)
        return set_err(c, XRT_ERR_STATE, "VolumePathTracingNEE needs an area light");
    if (p->slots_per_wave != 0 && p->slots_per_wave != 4 && p->slots_per_wave != 8 && p->slots_per_wave != 16 &&
        p->slots_per_wave != 32 && p->slots_per_wave != 64)
        return set_err(c, XRT_ERR_INVALID, "slots_per_wave must be 0, 4, 8, 16, 32 or 64");
    if (p->visits_per_launch > 128) return set_err(c, XRT_ERR_INVALID, "visits_per_launch must be 0..128");
    HIPCHK(c, hipSetDevice(c->device));
    if (wait == 1) {
        HIPCHK(c, hipDeviceSynchronize());
    } else if (wait == 2) {
        HIPCHK(c, hipEventRecord(c->wait_ev, wait_stream));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->wait_ev, 0));
    }
    const uint32_t rows = shard_rows(p->height, p->shard_index, p->shard_count);
    const size_t n = (size_t)rows * p->width;
    const size_t npix = (size_t)p->width * p->height;
    int rc;
    if (n == 0) {
        // a shard that owns no rows (shard_index >= height): an all-zero framebuffer
        float* fb0 = d_out;
        if (!fb0) {
            if ((rc = ensure(c, c->fb, npix * 3 * sizeof(float)))) return rc;
            fb0 = as<float>(c->fb);
        }
        if (p->flags & XRT_FLAG_ACCUMULATE) return XRT_OK;   // nothing owned, nothing touched
        HIPCHK(c, hipMemsetAsync(fb0, 0, npix * 3 * sizeof(float), c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (h_out) HIPCHK(c, hipMemcpy(h_out, fb0, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
        if (st) {
            std::memset(st, 0, sizeof(*st));
            st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        }
        return XRT_OK;
    }
    if (n > c->cap_slots) {
        const size_t L = kMaxLights;
        if ((rc = ensure(c, c->ray_o, n * 16)) || (rc = ensure(c, c->ray_d, n * 16)) || (rc = ensure(c, c->thr, n * 16)) ||
            (rc = ensure(c, c->rad, n * 16)) || (rc = ensure(c, c->thr_prev, n * 16)) || (rc = ensure(c, c->hit, n * 16)) ||
            (rc = ensure(c, c->hit2, n * 16)) || (rc = ensure(c, c->hit3, n * 16)) ||
            (rc = ensure(c, c->sh_o, L * n * 16)) || (rc = ensure(c, c->sh_d, L * n * 16)) ||
            (rc = ensure(c, c->sh_c, L * n * 16)) || (rc = ensure(c, c->med, n * 16)) || (rc = ensure(c, c->med2, n * 16)) ||
            (rc = ensure(c, c->nee, 4 * n * 16)) ||
            (rc = ensure(c, c->state, n * 4)) || (rc = ensure(c, c->sample_k, n * 4)) || (rc = ensure(c, c->depth, n * 4)) ||
            (rc = ensure(c, c->occ, n * 4)) || (rc = ensure(c, c->rng_c, n * 4)) || (rc = ensure(c, c->rng_g, n * 4)) ||
            (rc = ensure(c, c->ring, n * kRing * 4)) || (rc = ensure(c, c->c_seg, n * 4)) ||
            (rc = ensure(c, c->c_shadow, n * 4)) || (rc = ensure(c, c->c_rej, n * 4)) || (rc = ensure(c, c->c_stall, n * 4)) ||
            (rc = ensure(c, c->lists, 3 * (n + kMaxParts) * 4)))   // two live lists + the refill list
            return rc;
        c->cap_slots = n;
    }
    if ((rc = ensure(c, c->counts, 5 * kMaxParts * 4)) || (rc = ensure(c, c->stats, 512))) return rc;
    float* fb = d_out;
    if (!fb) {
        if ((rc = ensure(c, c->fb, npix * 3 * sizeof(float)))) return rc;
        fb = as<float>(c->fb);
    }
    KParams P = c->base;
    P.integrator = p->integrator;
    P.max_depth = p->max_depth, P.width = p->width, P.height = p->height, P.spp = p->spp;
    P.fw = (float)p->width, P.fh = (float)p->height, P.rw = 1.0f / P.fw, P.rh = 1.0f / P.fh;
    P.raspect = 1.0f / P.aspect;
    P.cdiv = (cdiv_exact(c, P.fw) ? 1u : 0u) | (cdiv_exact(c, P.fh) ? 2u : 0u) | (cdiv_exact(c, P.aspect) ? 4u : 0u);
    P.shard_index = p->shard_index, P.shard_count = p->shard_count, P.n_slots = (uint32_t)n;
    P.spw_req = p->slots_per_wave, P.rflags = p->flags;
    // two-level traces: the BVH walk takes four lanes per queued ray (k_trace_deep4q, every
    // size: its lanes keep their own best hits) unless the caller asks for one
    {
        const char* dq = exp_env("XRT_DEEP_QUAD");
        P.deep_quad = dq ? std::atoi(dq) : (p->flags & XRT_FLAG_DEEP_SINGLE) ? 0 : 1;
    }
    // Schedule, decided once (the partition count below depends on it): the fused k_step
    // (scene resident in LDS, kStepVisits path segments per slot per launch, in-kernel
    // compaction and refill requests) when the scene fits, in its merged-trace form for small
    // triangle scenes; else the multi-pass wavefront (k_shade, then k_trace streaming the
    // scene through LDS tiles; k_shade refills its slots' rings in-line).
    // Two-level scenes (C4) take the merged kernel with the wave's own BVH walk.
    const bool bvh = !(p->flags & (XRT_FLAG_WAVEFRONT | XRT_FLAG_NO_MERGED)) && use_step_bvh(P);
    // Direct / Normal over an LDS-resident scene: pixel-parallel sample chains (pixel.hip) —
    // one k_pixel launch between k_seed and k_finish, no live lists, no refill launch
    const bool pixel = !bvh && !(p->flags & (XRT_FLAG_WAVEFRONT | XRT_FLAG_NO_PIXEL)) && use_pixel(P);
    const bool fused = bvh || (!(p->flags & XRT_FLAG_WAVEFRONT) && step_lds_bytes(P) != 0);
    const bool merged = bvh || (fused && !(p->flags & XRT_FLAG_NO_MERGED) && use_step_merged(P));
    // speculative sample starts for the merged schedule's 16-slot launches (spec.hip)
    const bool spec = merged && !bvh && !(p->flags & XRT_FLAG_NO_SPEC) && use_step_spec(P);
    // live-list partitions (a multiple of the 8 XCDs): every wave appends to its partition's
    // counters once per launch, so more partitions mean less atomic contention (64 -> 256:
    // C4 -14%, C2 -4.5%).  The merged schedule (64 segments per launch) is fastest with
    // >= 2048 slots per partition (at most 256), the per-segment ones with >= 512 (at most
    // kMaxParts): C3 -8%, C4 -4% over 256
    {
        const bool merged_sched = merged;
        const size_t cap = merged_sched ? 256 : kMaxParts, per = merged_sched ? 2048 : kPartMinSlots;
        uint32_t np = (uint32_t)std::min<size_t>(cap, std::max<size_t>(1, n / per));
        if (np >= 8) np &= ~7u;
        P.n_part = np;
        P.part_cap = (uint32_t)((n + np - 1) / np);
    }
    const size_t lcap = (size_t)P.n_part * P.part_cap;
    P.ray_o = as<f4>(c->ray_o), P.ray_d = as<f4>(c->ray_d), P.thr = as<f4>(c->thr), P.rad = as<f4>(c->rad);
    P.thr_prev = as<f4>(c->thr_prev), P.hit = as<f4>(c->hit), P.hit2 = as<f4>(c->hit2), P.hit3 = as<f4>(c->hit3);
    P.sh_o = as<f4>(c->sh_o), P.sh_d = as<f4>(c->sh_d), P.sh_c = as<f4>(c->sh_c);
    P.med = as<f4>(c->med), P.med2 = as<f4>(c->med2), P.nee = as<f4>(c->nee);
    P.state = as<uint32_t>(c->state), P.sample_k = as<uint32_t>(c->sample_k), P.depth = as<uint32_t>(c->depth);
    P.occ = as<uint32_t>(c->occ), P.rng_c = as<uint32_t>(c->rng_c), P.rng_g = as<uint32_t>(c->rng_g);
    P.ring = as<uint32_t>(c->ring);
    P.c_seg = as<uint32_t>(c->c_seg), P.c_shadow = as<uint32_t>(c->c_shadow), P.c_rej = as<uint32_t>(c->c_rej);
    P.c_stall = as<uint32_t>(c->c_stall);
    P.fb = fb;
    P.stats = as<unsigned long long>(c->stats);
    if ((rc = setup_deep(c, P))) return rc;

    uint32_t* lists[2] = {as<uint32_t>(c->lists), as<uint32_t>(c->lists) + lcap};
    P.req = as<uint32_t>(c->lists) + 2 * lcap;
    // counter arrays of kMaxParts words: live[0..2] (rotating), then refill[0..1]
    uint32_t* cbase = as<uint32_t>(c->counts);
    auto counts_at = [&](uint64_t j) { return cbase + (size_t)j * kMaxParts; };
    uint32_t* req_counts = cbase + 3 * kMaxParts;
    const bool timing = (p->flags & XRT_FLAG_TIMING) != 0;
    xrt_stats S;
    std::memset(&S, 0, sizeof(S));
    S.path_slots = n;
    S.samples = (uint64_t)n * p->spp;
    std::vector<std::pair<int, size_t>> ev_use;   // (kernel id, first event index)
    size_t ev_next = 0;
    auto ev_pair = [&](int kid) -> size_t {
        while (c->events.size() < ev_next + 2) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return (size_t)-1;
            c->events.push_back(e);
        }
        const size_t i = ev_next;
        ev_next += 2;
        ev_use.push_back({kid, i});
        return i;
    };
    auto launch = [&](int kid, auto&& fn) -> hipError_t {
        size_t e = timing ? ev_pair(kid) : (size_t)-1;
        if (e != (size_t)-1) (void)hipEventRecord(c->events[e], c->stream);
        hipError_t err = fn();
        if (e != (size_t)-1) (void)hipEventRecord(c->events[e + 1], c->stream);
        S.launches[kid]++;
        return err;
    };

    if (!(p->flags & XRT_FLAG_ACCUMULATE))
        HIPCHK(c, hipMemsetAsync(fb, 0, npix * 3 * sizeof(float), c->stream));
    else if (h_out)   // the caller's Image is the accumulator (Src/renderer.cpp:75)
        HIPCHK(c, hipMemcpyAsync(fb, h_out, npix * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(P.stats, 0, 512, c->stream));
    HIPCHK(c, launch(XRT_K_SEED, [&] { return launch_seed(P, lists[0], counts_at(0), counts_at(1), req_counts, c->stream); }));
    // the pixels' camera-ray triangle lists (small triangle scenes on the merged schedule:
    // k_step_spec's candidates, and with XRT_MERGED_CAMLIST the merged kernel's camera rays),
    // once per render, timed with the seeding; built before the first launch that reads them
    P.camlist = nullptr;
    bool camlist_pending = false;
    if (merged && !bvh && P.n_tris <= 64 && !exp_env("XRT_NO_CAMLIST")) {
        if ((rc = ensure(c, c->camlist, n * sizeof(uint4)))) return rc;
        P.camlist = as<uint4>(c->camlist);
        camlist_pending = true;
    }
    auto build_camlist = [&]() -> hipError_t {
        camlist_pending = false;
        return launch(XRT_K_SEED, [&] { return launch_camlist(P, c->stream); });
    };
    if (camlist_pending && XRT_MERGED_CAMLIST) HIPCHK(c, build_camlist());
    if (pixel) {
        // every pixel of the shard in one persistent launch; the pixel counter is a stats word
        // (zeroed with them above)
        uint32_t* work = reinterpret_cast<uint32_t*>(P.stats + kStatsWork);
        hipError_t e = launch(XRT_K_STEP, [&] { return launch_pixel(P, work, c->stream); });
        if (e != hipSuccess) return hip_err(c, e, "k_pixel");
    }
    // refill epochs: shading launches of epoch e append to req_counts[e & 1]; k_refill(e)
    // consumes it and clears req_counts[(e + 1) & 1] for epoch e + 1.  Epoch 0 is the
    // first twist of every slot, requested by k_seed.
    uint64_t epoch = 0;
    bool merged_refill = false;   // set once the merged schedule is chosen (below)
    auto refill = [&]() -> hipError_t {
        const int a = (int)(epoch & 1), b = a ^ 1;
        ++epoch;
        return launch(XRT_K_REFILL, [&] {
            if (merged_refill)
                return launch_refill_merged(P, req_counts + a * kMaxParts, req_counts + b * kMaxParts, c->stream);
            return launch_refill(P, req_counts + a * kMaxParts, req_counts + b * kMaxParts, c->stream);
        });
    };
    if (!pixel) HIPCHK(c, refill());

    const uint32_t blocks = P.n_part * ((P.part_cap + 255) / 256);   // one entry per thread
    // GI/Direct: at most max_depth + 1 shade passes per sample; VPT walks are unbounded
    // (null collisions, suspensions), so only the live-slot poll ends the loop there.
    const uint64_t cap_iters = volumetric ? (uint64_t)p->spp * 100000ull + 1000000ull
                                          : (uint64_t)p->spp * (p->max_depth + 2) + 16;
    // asynchronous termination polling: every kPoll iterations copy the live-slot count to
    // pinned memory; block on a poll only when the host runs kAhead iterations ahead.
    constexpr uint64_t kPoll = 16, kAhead = 64;
    struct Poll { uint64_t it; hipEvent_t ev; int slot; };
    std::vector<Poll> polls;
    hipEvent_t* poll_ev = c->poll_ev;
    uint64_t it = 0;
    int poll_slot = 0;
    bool done = pixel;   // the pixel schedule has no step loop
    // k_step rotates three live counters: round i reads counts[i%3], appends to
    // counts[(i+1)%3] and clears counts[(i+2)%3] for round i+1 (every step kernel twists its
    // slots' rings in-line at the end of the launch: no k_refill after the seeding one).
    // segments per slot per step launch: kMergedVisits / kStepVisits unless the caller
    // sets visits_per_launch (results do not depend on it)
    const uint32_t merged_visits =
        merged ? std::min<uint32_t>(kMergedVisits, (kMT - step_merged_draws(P)) / step_merged_draws(P)) : 0;
    const char* ev = exp_env("XRT_VISITS");   // experiment builds only
    const uint32_t step_visits = ev                    ? (uint32_t)std::atoi(ev)
                                 : p->visits_per_launch ? p->visits_per_launch
                                 : merged               ? merged_visits
                                 : (volumetric && kVptEvents) ? kVptEventVisits
                                                        : kStepVisits;
    merged_refill = merged;
    // a slot's ring is twisted at the end of a launch when fewer words are left than the next
    // launch can draw: the merged kernel draws at most step_merged_draws per segment and
    // checks it; k_step / k_step_tri check kRngVisit per visit
    // k_step_spec reads up to kSpecDraws words past the cursor per visit: fewer visits per launch
    // (with XRT_SPEC_TWIST it twists in-loop instead: XRT_SPEC_VISITS visits unless the caller sets them)
    const uint32_t spec_visits = !spec ? 0
                                 : XRT_SPEC_TWIST ? ((ev || p->visits_per_launch) ? step_visits : XRT_SPEC_VISITS)
                                                  : std::min<uint32_t>(step_visits, (kMT - kSpecDraws) / kSpecDraws);
    P.rng_keep = spec && !XRT_SPEC_TWIST
                     ? std::max(step_visits * step_merged_draws(P) + step_merged_draws(P), spec_visits * kSpecDraws + kSpecDraws)
                 : merged                      ? step_visits * step_merged_draws(P) + step_merged_draws(P)
                 : (volumetric && kVptEvents) ? step_visits * kVptEventDraws + kRngVisit
                                              : step_visits * kVisitDraws + kRngVisit;
    if (!pixel && P.rng_keep > kMT) return set_err(c, XRT_ERR_INVALID, "visits_per_launch too large for the RNG ring");
    // device copy of the (now final) parameters for kernels that read them from memory
    if ((rc = ensure(c, c->kparams, sizeof(KParams)))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->kparams.p, &P, sizeof(KParams), hipMemcpyHostToDevice, c->stream));
    const KParams* dP = as<KParams>(c->kparams);
    // the merged schedule polls every launch and runs at most 3 launches ahead of the last
    // retired poll, so its per-launch layout (below) follows the live count closely
    const uint64_t poll_every = merged ? 1 : fused ? 4 : kPoll, ahead = merged ? 3 : fused ? 16 : kAhead;
    // merged schedule: the slots-per-wave layout is chosen from the shard's slot count (full
    // waves for a whole frame, 2 or 4 lanes per slot for small pixel shards); switching it
    // as the live count drops measured slower.  Every layout gives identical
    // results.
    // The merged schedule re-chooses the layout every launch from the live count of the last
    // retired poll (an upper bound: paths only finish), so a frame's tail, where few slots
    // remain, runs with more lanes per slot, and sizes the grid by the fullest
    // partition's live count instead of its capacity.  Results never depend on the layout.
    uint64_t live_hint = n;
    uint32_t live_part_max = P.part_cap;
    std::vector<uint64_t> launch_live;   // the live hint each step launch was sized with
    size_t step_idx = 0;
    for (; it < cap_iters && !done; ++it) {
        const int cur = (int)(it & 1), nxt = cur ^ 1;
        uint32_t* live = nullptr;
        if (fused) {
            const int ci = (int)(it % 3), co = (int)((it + 1) % 3), cz = (int)((it + 2) % 3);
            live = counts_at(co);
            launch_live.push_back(live_hint);
            if (merged) {
                const uint32_t spw = step_merged_spw(P, live_hint);
                S.layout_launches[spw == 64 ? 0 : spw == 32 ? 1 : spw == 16 ? 2 : spw == 8 ? 3 : 4]++;
            }
            // speculative starts in the group layouts (4 lanes per slot; 16 in the tail; 8 when forced)
            const uint32_t spw_now = merged ? step_merged_spw(P, live_hint) : 0;
            const bool spec_now = spec && P.camlist && (spw_now == 16 || spw_now == 8 || (XRT_SPEC_TAIL && spw_now == 4)) &&
                                  step_merged_group(P, spw_now) * spw_now == 64;
            if (spec_now) S.spec_launches++;
            if (spec_now && camlist_pending) HIPCHK(c, build_camlist());
            hipError_t e = launch(XRT_K_STEP, [&] {
                if (spec_now)
                    return launch_step_spec(P, dP, lists[cur], counts_at(ci), lists[nxt], counts_at(co), counts_at(cz),
                                            spec_visits, live_part_max, spw_now, c->stream);
                if (merged)
                    return launch_step_merged(P, dP, c->step_objs, lists[cur], counts_at(ci), lists[nxt],
                                              counts_at(co), counts_at(cz), req_counts + (epoch & 1) * kMaxParts,
                                              step_visits, live_hint, live_part_max, c->stream);
                return launch_step(P, dP, lists[cur], counts_at(ci), lists[nxt], counts_at(co), counts_at(cz),
                                   req_counts + (epoch & 1) * kMaxParts, step_visits, blocks, live_hint, c->stream);
            });
            if (e != hipSuccess) return hip_err(c, e, "k_step");
            // both step kernels refill their slots' rings themselves (wave_refill)
        } else {
            live = counts_at(nxt);
            hipError_t e = launch(XRT_K_SHADE, [&] {
                return launch_shade(P, lists[cur], counts_at(cur), lists[nxt], counts_at(nxt),
                                    req_counts + (epoch & 1) * kMaxParts, blocks, c->stream);
            });
            if (e != hipSuccess) return hip_err(c, e, "k_shade");
            e = launch(XRT_K_TRACE, [&] {
                return launch_trace(P, lists[nxt], counts_at(nxt), counts_at(cur), blocks, c->stream, false);
            });
            if (e != hipSuccess) return hip_err(c, e, "k_trace");
            if (P.two_level && P.bvh_node && P.scene_kind == SCN_TRI) {
                e = launch(XRT_K_DEEP, [&] { return launch_trace_deep(P, c->stream); });
                if (e != hipSuccess) return hip_err(c, e, "k_trace_deep4");
            }
            // no k_refill: k_shade twists its slots' rings itself (wave_refill)
        }
        if (it % poll_every == poll_every - 1) {
            const int ps = poll_slot++ % 8;
            HIPCHK(c, hipMemcpyAsync(c->h_poll + ps * kMaxParts, live, P.n_part * 4, hipMemcpyDeviceToHost,
                                     c->stream));
            HIPCHK(c, hipEventRecord(poll_ev[ps], c->stream));
            polls.push_back({it, poll_ev[ps], ps});
        }
        // retire polls: non-blocking when possible, blocking when too far ahead
        while (!polls.empty()) {
            Poll& q = polls.front();
            const bool must_wait = it - q.it >= ahead;
            if (!must_wait && hipEventQuery(q.ev) != hipSuccess) break;
            HIPCHK(c, hipEventSynchronize(q.ev));
            uint64_t alive = 0;
            uint32_t pmax = 0;
            for (uint32_t k = 0; k < P.n_part; ++k)
                alive += c->h_poll[q.slot * kMaxParts + k], pmax = std::max(pmax, c->h_poll[q.slot * kMaxParts + k]);
            if (alive == 0) done = true;
            if (alive < live_hint) {
                live_hint = alive;
                if (merged && !P.spw_req) live_part_max = std::max(1u, pmax);
            }
            polls.erase(polls.begin());
            if (done) break;
        }
    }
    S.iterations = it;
    HIPCHK(c, launch(XRT_K_FINISH, [&] { return launch_finish(P, c->stream); }));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!done) {
        // the iteration cap was reached without observing an empty list: verify
        uint32_t left[kMaxParts] = {0};
        HIPCHK(c, hipMemcpy(left, counts_at(fused ? it % 3 : it & 1), P.n_part * 4, hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < P.n_part; ++k)
            if (left[k] != 0) return set_err(c, XRT_ERR_HIP, "iteration cap reached with live paths");
    }
    unsigned long long hs[48] = {0};
    HIPCHK(c, hipMemcpy(hs, P.stats, 48 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (XRT_PHASE_CLOCK)   // experiment builds: k_step_spec's visit phases (shader-clock cycles summed over waves)
        std::fprintf(stderr, "[xrt] spec phase cycles head %llu trace %llu candidates %llu end-test %llu shading %llu"
                     " moves %llu cursor+reload %llu launch %llu\n", hs[40], hs[41], hs[42], hs[43], hs[44], hs[45],
                     hs[46], hs[47]);
    if (hs[38])   // experiment builds (-DXRT_EXPERIMENTS): BVH walk counters
        std::fprintf(stderr, "[xrt] deep rays %llu node steps %llu wave iterations %llu max wave iterations %llu"
                     " in-wave walks %llu\n", hs[38], hs[39], hs[37], hs[36], hs[35]);
    S.segments = hs[0], S.shadow_rays = hs[1], S.draws = hs[2], S.rejected = hs[3], S.stalled = hs[4];
    S.rng_twists = hs[7];
    S.pix_windows = hs[kStatsPix], S.pix_stride4 = hs[kStatsPix + 1], S.pix_frustum = hs[kStatsPix + 2];
    S.pix_frustum_overflow = hs[kStatsPix + 3], S.pix_shadow_list = hs[kStatsPix + 4];
    S.pix_shadow_overflow = hs[kStatsPix + 5], S.pix_flushes = hs[kStatsPix + 6];
    S.schedule = pixel   ? XRT_SCHED_PIXEL
                 : !fused ? XRT_SCHED_WAVEFRONT
                 : bvh    ? XRT_SCHED_STEP_BVH
                 : merged ? XRT_SCHED_STEP_MERGED
                 : use_step_tri(P) ? XRT_SCHED_STEP_TRI : XRT_SCHED_STEP;
    S.partitions = P.n_part;
    if (fused && !pixel) S.visits_per_launch = step_visits;
    if (merged && !pixel) {
        S.slots_per_wave = step_merged_spw(P, n);   // the layout of the first launch (every launch's: layout_launches)
        S.group_lanes = step_merged_group(P, S.slots_per_wave);
    }
    if (timing) {
        const bool trace = exp_env("XRT_TRACE_LAUNCHES") != nullptr;   // experiments: per-launch times
        for (size_t q = 0; q < ev_use.size(); ++q) {
            const auto& u = ev_use[q];
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, c->events[u.second], c->events[u.second + 1]) == hipSuccess)
                S.kernel_ms[u.first] += ms;
            if (trace) {
                float gap = 0.0f;
                if (q) (void)hipEventElapsedTime(&gap, c->events[ev_use[q - 1].second + 1], c->events[u.second]);
                std::fprintf(stderr, "[xrt] launch %zu kernel %d %.3f ms (gap %.3f)%s", q, u.first, ms, gap,
                             u.first == XRT_K_STEP && q < launch_live.size() + 2 ? "" : "\n");
                if (u.first == XRT_K_STEP) {
                    const size_t si = step_idx++;
                    std::fprintf(stderr, " live %llu\n",
                                 si < launch_live.size() ? (unsigned long long)launch_live[si] : 0ull);
                }
            }
        }
    }
    if (h_out) HIPCHK(c, hipMemcpy(h_out, fb, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
    S.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (st) *st = S;
    return XRT_OK;
}

// ------------------------------------------------------------ multi-GPU context ----
// ParallelRenderer::render fans the pixel loop out over the whole machine
// (Src/renderer.cpp:83-99); here the machine is the listed GPUs.  Pixels are independent
// (per-pixel seed and accumulation, Src/renderer.cpp:35-36,75), so device i renders the
// interleaved rows y % (n * shard_count) == shard_index + shard_count * i — one host thread
// and one HIP stream per device, all devices at once — and the frame is assembled in the
// first device's framebuffer by one strided 2-D copy per other device (its own rows only,
// over xGMI peer access): the same frame a zero-padded sum-reduce would produce, with 1/n
// of the bytes and no arithmetic.  Bit-identical to the one-device render.
int xrt_create_multi(const int* devices, int n_devices, xrt_ctx** out) {
    if (!out) return XRT_ERR_INVALID;
    *out = nullptr;
    if (!devices || n_devices < 1 || n_devices > 64) return XRT_ERR_INVALID;
    xrt_ctx* m = new xrt_ctx();
    m->device = devices[0];
    for (int i = 0; i < n_devices; ++i) {
        xrt_ctx* s = nullptr;
        const int rc = xrt_create(devices[i], &s);
        if (rc != XRT_OK) {
            xrt_destroy(m);
            return rc;
        }
        m->subs.push_back(s);
    }
    // peer access from the first device to every other one (for the row gather); devices
    // that cannot map each other fall back to the runtime's staged peer copy
    (void)hipSetDevice(devices[0]);
    for (int i = 1; i < n_devices; ++i) {
        int can = 0;
        if (devices[i] != devices[0] && hipDeviceCanAccessPeer(&can, devices[0], devices[i]) == hipSuccess && can) {
            const hipError_t e = hipDeviceEnablePeerAccess(devices[i], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        }
    }
    *out = m;
    return XRT_OK;
}

int xrt_device_count(const xrt_ctx* c) { return !c ? 0 : c->subs.empty() ? 1 : (int)c->subs.size(); }

static int multi_fail(xrt_ctx* m, xrt_ctx* s, int rc, const char* what) {
    return set_err(m, rc, std::string(what) + " on device " + std::to_string(s->device) + ": " + s->err);
}

int xrt_upload_scene(xrt_ctx* c, const xrt_scene_desc* s) {
    if (!c || c->subs.empty()) return upload_scene_one(c, s);
    for (xrt_ctx* d : c->subs) {
        const int rc = upload_scene_one(d, s);
        if (rc) return multi_fail(c, d, rc, "xrt_upload_scene");
    }
    return XRT_OK;
}

int xrt_set_camera(xrt_ctx* c, const float c2w[16], float scale, float aspect) {
    if (!c || c->subs.empty()) return set_camera_one(c, c2w, scale, aspect);
    for (xrt_ctx* d : c->subs) {
        const int rc = set_camera_one(d, c2w, scale, aspect);
        if (rc) return multi_fail(c, d, rc, "xrt_set_camera");
    }
    return XRT_OK;
}

int xrt_set_medium(xrt_ctx* c, const xrt_medium_desc* md) {
    if (!c || c->subs.empty()) return set_medium_one(c, md);
    for (xrt_ctx* d : c->subs) {
        const int rc = set_medium_one(d, md);
        if (rc) return multi_fail(c, d, rc, "xrt_set_medium");
    }
    return XRT_OK;
}

// d_out: the caller's device image on subs[0]'s GPU (or null: host image h_io).
static int render_multi(xrt_ctx* m, const xrt_render_params* p, float* d_out, float* h_io, xrt_stats* st, int wait,
                        hipStream_t wait_stream) {
    const auto t_start = std::chrono::steady_clock::now();
    if (!p) return set_err(m, XRT_ERR_INVALID, "null params");
    if (p->width == 0 || p->height == 0 || p->shard_count == 0 || p->shard_index >= p->shard_count)
        return set_err(m, XRT_ERR_INVALID, "bad image size or shard");
    const uint32_t n = (uint32_t)m->subs.size();
    const size_t npix = (size_t)p->width * p->height, bytes = npix * 3 * sizeof(float);
    const bool acc = (p->flags & XRT_FLAG_ACCUMULATE) != 0;
    xrt_ctx* s0 = m->subs[0];
    HIPCHK(m, hipSetDevice(s0->device));
    if (wait == 1) {
        HIPCHK(m, hipDeviceSynchronize());
    } else if (wait == 2) {
        HIPCHK(m, hipEventRecord(s0->wait_ev, wait_stream));
        HIPCHK(m, hipEventSynchronize(s0->wait_ev));
    }
    // every device renders into its own framebuffer; device 0 directly into the output
    std::vector<float*> fbs(n, nullptr);
    for (uint32_t i = 0; i < n; ++i) {
        xrt_ctx* s = m->subs[i];
        HIPCHK(m, hipSetDevice(s->device));
        if (i == 0 && d_out) {
            fbs[0] = d_out;
        } else {
            int rc = ensure(s, s->fb, bytes);
            if (rc) return multi_fail(m, s, rc, "framebuffer");
            fbs[i] = as<float>(s->fb);
        }
        if (acc) {   // each device starts its rows from the caller's image
            if (d_out && i > 0)
                HIPCHK(m, hipMemcpy(fbs[i], d_out, bytes, hipMemcpyDefault));
            else if (!d_out)
                HIPCHK(m, hipMemcpy(fbs[i], h_io, bytes, hipMemcpyHostToDevice));
        }
    }
    std::vector<xrt_stats> S(n);
    std::vector<int> rcs(n, XRT_OK);
    std::vector<std::thread> th;
    for (uint32_t i = 0; i < n; ++i) {
        th.emplace_back([&, i] {
            xrt_render_params q = *p;
            q.shard_count = p->shard_count * n;
            q.shard_index = p->shard_index + p->shard_count * i;
            rcs[i] = render_impl(m->subs[i], &q, fbs[i], nullptr, &S[i]);
        });
    }
    for (std::thread& t : th) t.join();
    for (uint32_t i = 0; i < n; ++i)
        if (rcs[i] != XRT_OK) return multi_fail(m, m->subs[i], rcs[i], "render");
    // gather: device i's rows are y = shard_index + shard_count * (i + n * r)
    HIPCHK(m, hipSetDevice(s0->device));
    const size_t row = (size_t)p->width * 3 * sizeof(float), pitch = row * p->shard_count * n;
    for (uint32_t i = 1; i < n; ++i) {
        const uint32_t y0 = p->shard_index + p->shard_count * i;
        if (y0 >= p->height) continue;
        const uint32_t rows = (p->height - y0 + p->shard_count * n - 1) / (p->shard_count * n);
        const size_t off = (size_t)y0 * row;
        HIPCHK(m, hipMemcpy2DAsync(reinterpret_cast<char*>(fbs[0]) + off, pitch, reinterpret_cast<char*>(fbs[i]) + off,
                                   pitch, row, rows, hipMemcpyDefault, s0->stream));
    }
    HIPCHK(m, hipStreamSynchronize(s0->stream));
    if (h_io) HIPCHK(m, hipMemcpy(h_io, fbs[0], bytes, hipMemcpyDeviceToHost));
    if (st) {
        xrt_stats T = S[0];
        for (uint32_t i = 1; i < n; ++i) {
            for (int k = 0; k < XRT_K_COUNT; ++k) T.kernel_ms[k] += S[i].kernel_ms[k], T.launches[k] += S[i].launches[k];
            T.samples += S[i].samples, T.segments += S[i].segments, T.shadow_rays += S[i].shadow_rays;
            T.draws += S[i].draws, T.rejected += S[i].rejected, T.stalled += S[i].stalled;
            T.rng_twists += S[i].rng_twists;
            T.pix_windows += S[i].pix_windows, T.pix_stride4 += S[i].pix_stride4, T.pix_frustum += S[i].pix_frustum;
            T.pix_frustum_overflow += S[i].pix_frustum_overflow, T.pix_shadow_list += S[i].pix_shadow_list;
            T.pix_shadow_overflow += S[i].pix_shadow_overflow, T.pix_flushes += S[i].pix_flushes;
            T.spec_launches += S[i].spec_launches;
            for (int k = 0; k < 5; ++k) T.layout_launches[k] += S[i].layout_launches[k];
            T.path_slots += S[i].path_slots;
            T.iterations = std::max(T.iterations, S[i].iterations);
        }
        T.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        *st = T;
    }
    return XRT_OK;
}

// Scene::intersect / Scene::occluded (Src/scene.cpp:190-211) for caller rays, on the GPU
int xrt_query(xrt_ctx* c, uint32_t n, const float* rays, const float* tmax, int32_t mode, xrt_hit* out) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || (n && (!rays || !out))) return XRT_ERR_INVALID;
    if (mode != XRT_QUERY_INTERSECT && mode != XRT_QUERY_OCCLUDED) return set_err(c, XRT_ERR_INVALID, "bad query mode");
    if (!c->has_scene) return set_err(c, XRT_ERR_STATE, "upload a scene first");
    if (n == 0) return XRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c, c->ray_o, n * 16)) || (rc = ensure(c, c->ray_d, n * 16)) || (rc = ensure(c, c->hit, n * 16)) ||
        (rc = ensure(c, c->hit2, n * 16)) || (rc = ensure(c, c->hit3, n * 16)) || (rc = ensure(c, c->sh_o, n * 16)) ||
        (rc = ensure(c, c->sh_d, n * 16)) || (rc = ensure(c, c->state, n * 4)) || (rc = ensure(c, c->occ, n * 4)) ||
        (rc = ensure(c, c->lists, (n + 64) * 4)) || (rc = ensure(c, c->counts, 5 * kMaxParts * 4)) ||
        (rc = ensure(c, c->q_rays, (size_t)n * 24)) || (rc = ensure(c, c->q_tmax, (size_t)n * 4)) ||
        (rc = ensure(c, c->q_out, (size_t)n * sizeof(xrt_hit))))
        return rc;
    // (buffers only ever grow, so the render's cap_slots invariant still holds)
    KParams P = c->base;
    P.n_slots = n, P.n_part = 1, P.part_cap = n;
    P.ray_o = as<f4>(c->ray_o), P.ray_d = as<f4>(c->ray_d), P.hit = as<f4>(c->hit), P.hit2 = as<f4>(c->hit2);
    P.hit3 = as<f4>(c->hit3), P.sh_o = as<f4>(c->sh_o), P.sh_d = as<f4>(c->sh_d);
    P.state = as<uint32_t>(c->state), P.occ = as<uint32_t>(c->occ);
    if ((rc = setup_deep(c, P))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->q_rays.p, rays, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
    if (tmax) HIPCHK(c, hipMemcpyAsync(c->q_tmax.p, tmax, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    uint32_t* cnt = as<uint32_t>(c->counts);
    HIPCHK(c, launch_query(P, as<float>(c->q_rays), tmax ? as<float>(c->q_tmax) : nullptr, mode, as<uint32_t>(c->lists),
                           cnt, cnt + kMaxParts, as<xrt_hit>(c->q_out), c->stream));
    HIPCHK(c, hipMemcpyAsync(out, c->q_out.p, (size_t)n * sizeof(xrt_hit), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < n; ++i) {   // the triangle within its object's mesh
        xrt_hit& q = out[i];
        if (q.primitive >= 0 && q.object >= 0 && (size_t)q.object < c->obj_tri_first.size() &&
            c->obj_tri_first[q.object] >= 0)
            q.primitive -= c->obj_tri_first[q.object];
    }
    return XRT_OK;
}

int xrt_render(xrt_ctx* c, const xrt_render_params* p, float* rgb_out, xrt_stats* st) {
    if (!rgb_out) return set_err(c, XRT_ERR_INVALID, "null output");
    if (c && !c->subs.empty()) return render_multi(c, p, nullptr, rgb_out, st, 0, nullptr);
    return render_impl(c, p, nullptr, rgb_out, st);
}

int xrt_render_device(xrt_ctx* c, const xrt_render_params* p, float* d_rgb_out, xrt_stats* st) {
    if (!d_rgb_out) return set_err(c, XRT_ERR_INVALID, "null output");
    if (c && !c->subs.empty()) return render_multi(c, p, d_rgb_out, nullptr, st, 1, nullptr);
    return render_impl(c, p, d_rgb_out, nullptr, st, 1);
}

int xrt_render_device_after(xrt_ctx* c, const xrt_render_params* p, float* d_rgb_out, void* hip_stream,
                            xrt_stats* st) {
    if (!d_rgb_out) return set_err(c, XRT_ERR_INVALID, "null output");
    if (c && !c->subs.empty()) return render_multi(c, p, d_rgb_out, nullptr, st, 2, (hipStream_t)hip_stream);
    return render_impl(c, p, d_rgb_out, nullptr, st, 2, (hipStream_t)hip_stream);
}

// ---------------------------------------------------------------- self-tests ----
int xrt_test_rng(xrt_ctx* c, const uint32_t* seeds, uint32_t n_seeds, uint32_t skip, uint32_t n, float* out) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !seeds || !out) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    DevBuf ds, dout, rings;
    int rc;
    if ((rc = ensure(c, ds, n_seeds * 4)) || (rc = ensure(c, dout, (size_t)n_seeds * n * 4)) ||
        (rc = ensure(c, rings, (size_t)n_seeds * kRing * 4)))
        return rc;
    hipError_t e = hipMemcpy(ds.p, seeds, n_seeds * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_test_rng(as<uint32_t>(ds), n_seeds, skip, n, as<float>(dout), as<uint32_t>(rings), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout.p, (size_t)n_seeds * n * 4, hipMemcpyDeviceToHost);
    free_buf(ds), free_buf(dout), free_buf(rings);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_test_rng");
}

int xrt_test_trig(xrt_ctx* c, const float* x, uint32_t n, float* out) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !x || !out) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    DevBuf dx, dout;
    int rc;
    if ((rc = ensure(c, dx, (size_t)n * 4 + 16)) || (rc = ensure(c, dout, (size_t)n * 8 + 16))) return rc;
    hipError_t e = hipMemcpy(dx.p, x, (size_t)n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_test_trig(as<float>(dx), n, as<float>(dout), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout.p, (size_t)n * 8, hipMemcpyDeviceToHost);
    free_buf(dx), free_buf(dout);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_test_trig");
}

int xrt_test_logexp(xrt_ctx* c, const float* x, uint32_t n, float* out) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !x || !out) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    DevBuf dx, dout;
    int rc;
    if ((rc = ensure(c, dx, (size_t)n * 4 + 16)) || (rc = ensure(c, dout, (size_t)n * 8 + 16))) return rc;
    hipError_t e = hipMemcpy(dx.p, x, (size_t)n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_test_logexp(as<float>(dx), n, as<float>(dout), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout.p, (size_t)n * 8, hipMemcpyDeviceToHost);
    free_buf(dx), free_buf(dout);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_test_logexp");
}

int xrt_test_powf(xrt_ctx* c, const float* x, uint32_t n, float y, float* out) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !x || !out) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    DevBuf dx, dout;
    int rc;
    if ((rc = ensure(c, dx, (size_t)n * 4 + 16)) || (rc = ensure(c, dout, (size_t)n * 4 + 16))) return rc;
    hipError_t e = hipMemcpy(dx.p, x, (size_t)n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_test_powf(as<float>(dx), n, y, as<float>(dout), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout.p, (size_t)n * 4, hipMemcpyDeviceToHost);
    free_buf(dx), free_buf(dout);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_test_powf");
}

int xrt_tonemap(xrt_ctx* c, const float* d_rgb, uint32_t n_pixels, float gamma, uint8_t* rgb8_out) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !rgb8_out) return XRT_ERR_INVALID;
    const float* src = d_rgb ? d_rgb : as<float>(c->fb);
    if (!src || (!d_rgb && (size_t)n_pixels * 3 * sizeof(float) > c->fb.bytes))
        return set_err(c, XRT_ERR_STATE, "xrt_tonemap: no framebuffer of that size (render first)");
    HIPCHK(c, hipSetDevice(c->device));
    DevBuf out;
    int rc;
    const size_t n = (size_t)n_pixels * 3;
    if ((rc = ensure(c, out, n + 16))) return rc;
    hipError_t e = launch_tonemap(src, (uint32_t)n, 1.0f / gamma, as<uint8_t>(out), c->stream);   // Src/image.h:85
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(rgb8_out, out.p, n, hipMemcpyDeviceToHost);
    free_buf(out);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_tonemap");
}

int xrt_test_trig_draw_domain(xrt_ctx* c, uint32_t first, uint32_t count, float* out_sin, float* out_cos, float* out_r) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !out_sin || !out_cos || !out_r) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    DevBuf ds, dc, dr;
    int rc;
    const size_t b = (size_t)count * 4 + 16;
    if ((rc = ensure(c, ds, b)) || (rc = ensure(c, dc, b)) || (rc = ensure(c, dr, b))) return rc;
    hipError_t e = launch_test_trig_domain(first, count, as<float>(ds), as<float>(dc), as<float>(dr), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out_sin, ds.p, (size_t)count * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_cos, dc.p, (size_t)count * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_r, dr.p, (size_t)count * 4, hipMemcpyDeviceToHost);
    free_buf(ds), free_buf(dc), free_buf(dr);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_test_trig_draw_domain");
}

}  // extern "C"

// every 32-bit input: mode 0 rcp_rn vs 1/b, mode 1 div_const(x, c, rc) vs x / c (device_math.h)
int xrt_test_fastdiv(xrt_ctx* c, uint32_t mode, float cst, float rc, uint64_t* n_bad, uint32_t* first_bad16) {
    if (c && !c->subs.empty()) c = c->subs[0];   // multi-GPU context: its first device
    if (!c || !n_bad || !first_bad16) return XRT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    unsigned long long* d_n = nullptr;
    uint32_t* d_bad = nullptr;
    HIPCHK(c, hipMalloc(&d_n, 8));
    HIPCHK(c, hipMalloc(&d_bad, 64));
    hipError_t e = hipMemsetAsync(d_n, 0, 8, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0xff, 64, c->stream);
    const uint32_t chunk = 1u << 30;
    for (uint64_t f = 0; f < (1ull << 32) && e == hipSuccess; f += chunk)
        e = launch_test_fastdiv(mode, cst, rc, (uint32_t)f, chunk, d_n, d_bad, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(n_bad, d_n, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(first_bad16, d_bad, 64, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_n);
    (void)hipFree(d_bad);
    return e == hipSuccess ? XRT_OK : hip_err(c, e, "xrt_test_fastdiv");
}
