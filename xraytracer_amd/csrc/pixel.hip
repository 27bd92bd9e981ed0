// pixel.hip — pixel-parallel sample chains for the one-trace integrators
// (DirectIntegrator, Src/integrator.h:82-119; NormalIntegrator, :22-74).
//
// NormalRenderer::doRender (Src/renderer.cpp:29-81) runs a pixel's samples in order on one
// mt19937 stream, so every other schedule gives a pixel one lane and runs its samples one
// after the other: a frame is as long as its slowest pixel's chain of traces, and a row
// shard of an 8-GPU frame leaves most of the chip idle.  For these two integrators a
// sample's draw count depends only on its camera ray:
//   Direct : 2 jitter words, then 2 words per area light iff the camera ray hits a surface
//            that is not an area light (every light's sample() draws exactly 2, whether or
//            not it returns pdf 0: Src/light.cpp:21-68, light.h:157-197)
//   Normal : 2 jitter words, nothing else
// so the stream offset of sample k+1 is f(o_k) = o_k + 2 + 2·NL·hit(o_k), and hit(o) is a
// function of the two words at o alone.  One wave takes one pixel and evaluates a window of
// 64 candidate offsets o, o+2, ..., o+126 at once — every lane traces the camera ray its
// candidate's jitter words give — then walks the chain o -> f(o) through the window with
// scalar bit operations on the ballot of surface hits.  The candidates on the chain are the
// pixel's next samples, in order: they shade (light samples from the words after their
// jitter, shadow rays), pass the reference's NaN / Inf / negative check, and are added to the
// pixel's running sum one after the other in sample order by three lanes (one per channel),
// exactly Image::addPixel's sequence.  The candidates off the chain (offsets inside another
// sample's light words) are discarded.  Every sample therefore draws the same words, traces
// the same rays and adds the same floats as the reference: the image, the counters and the
// final stream cursor are bit-identical (tests/test_gpu_pixel.py).
//
// The 64 camera rays of a window leave one pixel through nearly the same point, so the
// wave's traversals are coherent (the per-slot k_step walks 64 unrelated pixels, and a
// visit lasts as long as its slowest lane's walk), and the frame has one work item per
// pixel instead of one serial chain per pixel: a row shard of 1/8 of the pixels still
// fills the chip.  Cost: the off-chain candidates' camera traces (a fraction h/(1+h) of
// the candidates for a surface-hit rate h and one light).
//
// The stream lives in LDS: each wave keeps its pixel's last 624 words in a circular buffer
// (x[i] at st[i % 624]; the state k_seed wrote is x[0..623]) and generates 128 words at a
// time before a window needs them — x[i] = x[i-227] ^ mix(x[i-624], x[i-623]) for the
// 128 words i in [g, g+128), whose inputs are all generated and none of which are
// overwritten before they are read (i - 227 >= g - 227 lies outside the chunk's slots).
// Persistent waves take pixels from an atomic counter until none are left.
#include <hip/hip_runtime.h>

#include "lscene.h"
#include "path_common.h"

namespace xrt {

constexpr bool kPixStride4 = XRT_PIX_STRIDE4;   // stride-4 candidate windows after all-hit windows
constexpr int kPixBlock = XRT_PIX_BLOCK;           // threads per block: 8 waves share one LDS scene copy
constexpr uint32_t kPixSumStride = 68;             // ordered-sum buffer row (floats): 64 + 4, rows on other banks
constexpr uint32_t kPixList = 64;                   // camera-frustum sphere list entries per wave (16-bit)
constexpr uint32_t kPixWaveLds = (kMT + 3 * kPixSumStride) * 4 + kPixList * 2;   // stream + sum buffer + list
constexpr uint32_t kPixFrustumMax = XRT_PIX_FRUSTUM_MAX;   // sphere scenes up to this size build the lists

constexpr bool kPixPacket = XRT_PIX_PACKET != 0;   // wave-uniform scene walks (lscene.h closest_w)
constexpr bool kPixShadowList = XRT_PIX_SHADOW_LIST != 0;   // per-pixel shadow-ray occluder lists

// the words generated per chunk: one pair per lane
constexpr uint32_t kPixChunk = 128;

// LDS-fed UniformSampler of one lane: x[c], x[c+1], ... from the wave's circular buffer.  The
// window logic guarantees every word it is asked for has been generated and not overwritten.
struct LdsRng {
    const uint32_t* st;
    uint32_t i;   // c % kMT
    __device__ __forceinline__ float next() {
        const uint32_t y = st[i];
        i = (i + 1 == kMT) ? 0u : i + 1;
        return canonical(mt_temper(y));
    }
};

// x[g .. g+127] into the circular buffer (x[g-624 .. g-1] in it): lane l makes x[g+2l] and
// x[g+2l+1] (libstdc++ _M_gen_rand's recurrence, one word at a time).  Every operand is read
// before any lane writes: lane l's second word needs x[g+2l+2-624], which lane l+1 replaces.
__device__ __forceinline__ void pix_gen(uint32_t* st, uint32_t g, int lane) {
    uint32_t i0 = g % kMT + 2u * (uint32_t)lane;
    if (i0 >= kMT) i0 -= kMT;
    const uint32_t i1 = i0 + 1u;   // g and kMT are even: a pair never wraps
    uint32_t i2 = i1 + 1u;
    if (i2 >= kMT) i2 -= kMT;
    uint32_t j0 = i0 + (kMT - 227u);   // x[i - 227] sits at (i + 397) % 624 (odd: j0 + 1 may wrap)
    if (j0 >= kMT) j0 -= kMT;
    uint32_t j1 = j0 + 1u;
    if (j1 >= kMT) j1 -= kMT;
    const uint32_t a0 = st[i0], a1 = st[i1], a2 = st[i2], b0 = st[j0], b1 = st[j1];
    wave_sync();
    st[i0] = b0 ^ mt_mix(a0, a1);
    st[i1] = b1 ^ mt_mix(a1, a2);
    wave_sync();
}

// The spheres a camera ray of pixel (col, row) can hit, for sphere-BVH scenes (C3): every
// camera ray of a pixel leaves the camera origin o through its jitter square, so it lies in
// the pyramid spanned by the square's corner directions — widened here by 0.01 pixel on every
// side, far beyond the float error of div_w / div_h / camera_ray's direction (~1e-7 relative
// against 1e-5 of the pixel's angle).  A ray that Sphere::intersect reports hitting passes
// within float error of the sphere, i.e. through the ball of radius |r| + sph_pad around it
// (sph_pad, the BVH's own box margin, is orders of magnitude above that error), and a ball
// that meets the pyramid is on the inner side of (or crosses) all four side planes.  So the
// list holds every sphere any of the pixel's camera rays can hit (and a few more), and its
// windows test only those, in any order: the closest hit is the (t, index) minimum either way.
// Each lane tests 1/64 of the spheres; returns the list length, or -1 when it overflows
// kPixList (the pixel's camera rays then walk the BVH).  Every lane must call it.
template <int SCN>
__device__ int pix_frustum(const KParams& P, const LScene& L, uint32_t col, uint32_t row, uint16_t* list, int lane) {
    const float m = 0.01f;
    const float u0 = ((float)col - m) / P.fw, u1 = ((float)col + (1.0f + m)) / P.fw;
    const float v0 = ((float)row - m) / P.fh, v1 = ((float)row + (1.0f + m)) / P.fh;
    const float* x = P.c2w;
    auto world = [&](float u, float v) {
        const v3 dir = mk((2.0f * u - 1.0f) * P.scale, (1.0f - 2.0f * v) * P.scale / P.aspect, -1.0f);
        return mk(dir.x * x[0] + dir.y * x[4] + dir.z * x[8], dir.x * x[1] + dir.y * x[5] + dir.z * x[9],
                  dir.x * x[2] + dir.y * x[6] + dir.z * x[10]);
    };
    const v3 D0 = world(u0, v0), D1 = world(u1, v0), D2 = world(u1, v1), D3 = world(u0, v1);
    const v3 Dc = (D0 + D1) + (D2 + D3);
    v3 n[4] = {cross(D0, D1), cross(D1, D2), cross(D2, D3), cross(D3, D0)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float s = dot(n[k], Dc) < 0.0f ? -1.0f : 1.0f;
        n[k] = n[k] * (s / length(n[k]));   // unit normal pointing into the pyramid
    }
    const v3 o = mk(x[12], x[13], x[14]);
    auto meets = [&](v3 c, float rr) {
        return dot(n[0], c) >= rr && dot(n[1], c) >= rr && dot(n[2], c) >= rr && dot(n[3], c) >= rr;
    };
    uint32_t cnt = 0;
    // blocks of 64 spheres (KParams::sblk) whose ball meets the pyramid, then their members
    const int nblk = (P.n_sph + 63) >> 6;
    for (int b0 = 0; b0 < nblk; b0 += 64) {
        bool bin = false;
        if (b0 + lane < nblk) {
            const f4 B = P.sblk[b0 + lane];
            const v3 c = xyz(B) - o;
            bin = !XRT_PIX_BLOCKS || meets(c, -(B.w + 1e-5f * length(c)));   // + the float slack of the block's dot products
        }
        for (uint64_t bm = __ballot(bin); bm; bm &= bm - 1ull) {
            const int j = ((b0 + __builtin_ctzll(bm)) << 6) + lane;
            bool in = false;
            if (j < P.n_sph) {
                const f4 S = L.ssph[j];
                in = meets(xyz(S) - o, -(__builtin_fabsf(S.w) + P.sph_pad));
            }
            const uint64_t mk_ = __ballot(in);
            const uint32_t at = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk_ >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk_, 0u));
            if (in && at < kPixList) list[at] = (uint16_t)j;
            cnt += (uint32_t)__builtin_popcountll(mk_);
        }
    }
    wave_sync();
    return cnt <= kPixList ? (int)cnt : -1;
}

// Scene::intersect over a pixel's frustum list (pix_frustum): the (t, index) minimum over the
// listed spheres, as sphere_bvh's.  Lane e holds list entry e's sphere (lsph: center, radius;
// lk: original index), broadcast to the wave one entry at a time (readlane: no memory latency
// inside the loop).
__device__ __forceinline__ void closest_list(f4 lsph, int lk, int nlist, v3 o, v3 d, HitRec& h, bool active) {
    h.t = kINF, h.u = h.v = 0.0f, h.code = -1, h.surf = -1, h.dp = -1, h.t1 = kINF;
    h.st = h.su = h.sv = h.du = h.dv = 0.0f;
    float bt = kINF;
    int bk = -1;
    for (int e = 0; e < nlist; ++e) {
        const v3 c = mk(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.x), e)),
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.y), e)),
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.z), e)));
        const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.w), e));
        const int k = __builtin_amdgcn_readlane(lk, e);
        float t = 0.0f;
        const bool hit = active && sphere_hit(o, d, c, r, t);
        const bool upd = hit && (t < bt || (t == bt && k < bk));
        bt = upd ? t : bt;
        bk = upd ? k : bk;
    }
    if (bk >= 0) h.t = bt, h.code = (1 << 28) | bk;
}

// Shadow-ray occluder lists (Direct on sphere-BVH scenes with one area light).  A shadow ray
// of the pixel starts at S.pos + 0.01 ng, S.pos within float error of a sphere s its camera
// rays can hit (a frustum-list sphere), and runs tmax - 0.01 along wi towards a light sample
// point p (within float error of the light), ending within 0.02 of p: so the whole segment
// lies in the convex hull of the ball around s (radius |r_s| + 0.01 + margin) and the light's
// bounding ball (+ 0.02 + margin).  A sphere whose occlusion test reports a hit has the hit
// point on that segment within float error of its surface, so its ball (|r| + sph_pad) meets
// that hull.  The hull of two balls is {x : min_s |x - a - s u| - ra - s (rb - ra) <= 0}
// (a convex function of s); ball_meets_hull lower-bounds the minimum by the tangent at the
// closed-form minimiser (convexity), so the test never drops a sphere that meets the hull.
__device__ __forceinline__ bool ball_meets_hull(v3 c, float rho, v3 a, float ra, v3 b, float rb) {
    const v3 u = b - a, w = c - a;
    const float L2 = dot(u, u), L = __builtin_sqrtf(L2), D = rb - ra;
    if (!(L > __builtin_fabsf(D)) || !(L2 > 0.0f)) return true;   // one ball inside the other: keep
    const float t0 = dot(w, u) / L2;
    const float h = length(w - u * t0);
    float s = t0 + D * h / (L * __builtin_sqrtf(L2 - D * D));
    s = s < 0.0f ? 0.0f : (s > 1.0f ? 1.0f : s);
    const v3 q = w - u * s;
    const float dq = length(q);
    if (!(dq > 1e-6f * (L + length(w)))) return true;   // at the axis: the tangent is undefined, keep
    const float f = dq - (ra + s * D);
    const float fp = -dot(u, q) / dq - D;   // f'(s)
    const float lb = f - __builtin_fabsf(fp) * (s > 0.5f ? s : 1.0f - s);
    return lb <= rho + 1e-4f * (L + length(w)) + 1e-4f;   // + the float slack of the evaluation
}

// Every occluder sphere that meets the hull of one of the pixel's camera-list spheres and the
// light's bounding ball, into `list` (each lane tests 1/64 of the spheres); returns the count,
// or -1 when it overflows kPixList (the pixel's shadow rays then walk the BVH).  lsph: lane e
// holds camera-list sphere e (nlist of them).  Every lane must call it.
__device__ int pix_shadow_list(const KParams& P, const LScene& L, f4 lsph, int nlist, uint16_t* list, int lane) {
    const DLight& lt = L.light[0];
    v3 lc;
    float lr;
    if (lt.kind == XRT_LIGHT_SPHERE || lt.kind == XRT_LIGHT_SPHERE_AREA) {   // either sampling: a point on the sphere
        lc = ld3(lt.center), lr = __builtin_fabsf(lt.radius);
    } else {   // quad / triangle: the centroid of its corners and the farthest corner
        const v3 v0 = ld3(lt.v0), e1 = ld3(lt.e1), e2 = ld3(lt.e2);
        const v3 cs[4] = {v0, v0 + e1, v0 + e2, v0 + e1 + e2};
        const int nc = lt.kind == XRT_LIGHT_QUAD ? 4 : 3;
        lc = mk(0, 0, 0);
        for (int q = 0; q < nc; ++q) lc = lc + cs[q];
        lc = lc / (float)nc;
        lr = 0.0f;
        for (int q = 0; q < nc; ++q) lr = smax(lr, length(cs[q] - lc));
        lr = lr * 1.001f;
    }
    const float pad = P.sph_pad;
    lr = lr + 0.02f + pad;
    // does the ball (p, rho) meet the hull of camera-list sphere e's ball and the light's?
    auto meets = [&](v3 p, float rho) {
        bool in = false;
        for (int e = 0; e < nlist && !in; ++e) {
            const v3 c = mk(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.x), e)),
                            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.y), e)),
                            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.z), e)));
            const float r = __builtin_fabsf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lsph.w), e))) +
                            0.01f + pad;
            // the hull's bounding box (grown by rho) first: most spheres are far from it
            const v3 lo = mk(smin(c.x - r, lc.x - lr), smin(c.y - r, lc.y - lr), smin(c.z - r, lc.z - lr));
            const v3 hi = mk(smax(c.x + r, lc.x + lr), smax(c.y + r, lc.y + lr), smax(c.z + r, lc.z + lr));
            const bool near = p.x >= lo.x - rho && p.x <= hi.x + rho && p.y >= lo.y - rho && p.y <= hi.y + rho &&
                              p.z >= lo.z - rho && p.z <= hi.z + rho;
            in = near && ball_meets_hull(p, rho, c, r, lc, lr);
        }
        return in;
    };
    uint32_t cnt = 0;
    // blocks of 64 spheres (KParams::sblk; each member's ball lies in the block's) whose ball
    // meets a hull, then their occluders
    const int nblk = (P.n_sph + 63) >> 6;
    for (int b0 = 0; b0 < nblk; b0 += 64) {
        bool bin = false;
        if (b0 + lane < nblk) {
            const f4 B = P.sblk[b0 + lane];
            bin = !XRT_PIX_BLOCKS || meets(xyz(B), B.w);
        }
        for (uint64_t bm = __ballot(bin); bm; bm &= bm - 1ull) {
            const int j = ((b0 + __builtin_ctzll(bm)) << 6) + lane;
            bool in = false;
            if (j < P.n_sph && (L.sbk[j] & (1 << 30))) {   // occluders only (Scene::occluded skips lights)
                const f4 S = L.ssph[j];
                in = meets(xyz(S), __builtin_fabsf(S.w) + pad);
            }
            const uint64_t mk_ = __ballot(in);
            const uint32_t at = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk_ >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk_, 0u));
            if (in && at < kPixList) list[at] = (uint16_t)j;
            cnt += (uint32_t)__builtin_popcountll(mk_);
        }
    }
    wave_sync();
    return cnt <= kPixList ? (int)cnt : -1;
}

// Scene::occluded over a pixel's shadow list: lane e holds occluder e (center, radius)
__device__ __forceinline__ bool occluded_list(f4 ssph, int nsl, v3 o, v3 d, float tmax, bool active) {
    bool occ = false;
    for (int e = 0; e < nsl; ++e) {
        const v3 c = mk(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(ssph.x), e)),
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ssph.y), e)),
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ssph.z), e)));
        const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ssph.w), e));
        float t = 0.0f;
        occ = occ || (active && sphere_hit(o, d, c, r, t) && t < tmax);
    }
    return occ;
}

// Deferred shading (Direct on sphere-BVH scenes): a window's samples that hit a surface are
// ~1/4 of its lanes, so shading them in the window (light samples, the shadow rays' wave walk)
// would run the wave at a quarter of its width.  Instead they join a queue of up to 64 shading
// items (the candidate's stream position and hit record), and every sample of the window
// leaves a one-byte code in a pending list: 0 = the miss radiance 0.18, 1 + l = light l's Le
// (an area light seen from its front), 255 = zero (seen from the back), 128 + i = queue item
// i.  Every third window (or when the queue might overflow, or the pixel is done) the queue is
// shaded by the whole wave at once and the pending codes are added to the running sum in
// sample order.  An item's words are still in the 624-word stream window then: three windows
// span at most 3 * (128 + 2 NL) words and generation runs at most 255 + 2 NL past the current
// window's start, within 624 for NL <= 18.  Same draws, same rays, same float sums.
constexpr bool pix_defer(int scn, int integ) {
    return XRT_PIX_DEFER && scn == SCN_SPHERE && integ == XRT_INTEGRATOR_DIRECT;
}
constexpr uint32_t kPixPend = 192;   // pending samples of three windows (codes)
// the 624-word stream buffer holds three windows' items and the generation lookahead only for
// NL <= 18 (above), and the plain window's own words bound NL further; xrt_api.cpp refuses
// scenes with more than kMaxLights lights
static_assert(kMaxLights <= 18, "k_pixel's stream window assumes at most 18 area lights");
constexpr uint32_t kPixWaveDeferLds = kPixWaveLds + 3 * kPixSumStride * 4 + 3 * 64 * 4 + kPixPend;
constexpr int pix_block(int scn, int integ) { return pix_defer(scn, integ) ? XRT_PIX_DEFER_BLOCK : kPixBlock; }
__host__ __device__ inline bool pix_defer_rt(const KParams& P) {
    return XRT_PIX_DEFER && P.scene_kind == SCN_SPHERE && P.integrator == XRT_INTEGRATOR_DIRECT;
}

// LDS bytes of the pixel schedule: the scene carve, then one slice per wave
// (with XRT_PIX_GLOBAL_BVH the sphere BVH — the carve's last three regions — stays in global
// memory: the lists hold a pixel's spheres in registers, so the BVH is read only by the list
// scans (from L1 / L2) and by overflow pixels, and the block skips copying ~36 KB into LDS)
__host__ __device__ inline uint32_t pix_wave_off(const KParams& P) {
    const StepLayout Lo = step_layout(P);
    return ((XRT_PIX_GLOBAL_BVH && P.n_snode > 0 ? Lo.snode : Lo.total) + 15u) & ~15u;
}

template <int SCN, int INTEG, int BS>
__global__ __launch_bounds__(BS, XRT_PIX_WAVES) void k_pixel(KParams P, uint32_t* __restrict__ work) {
    constexpr bool DEFER = pix_defer(SCN, INTEG);
    constexpr uint32_t kWave = DEFER ? kPixWaveDeferLds : kPixWaveLds;
    extern __shared__ __attribute__((aligned(16))) f4 lds_pix[];
    char* lb = reinterpret_cast<char*>(lds_pix);
    const int tid = threadIdx.x, lane = tid & 63;
    const LScene L = load_lscene(P, lb, tid, BS, !XRT_PIX_GLOBAL_BVH);
    uint32_t* st = reinterpret_cast<uint32_t*>(lb + pix_wave_off(P) + (tid >> 6) * kWave);
    float* sum = reinterpret_cast<float*>(st + kMT);
    uint16_t* list = reinterpret_cast<uint16_t*>(sum + 3 * kPixSumStride);
    float* ires = reinterpret_cast<float*>(list + kPixList);        // DEFER: shaded items' radiance
    uint32_t* it_i = reinterpret_cast<uint32_t*>(ires + 3 * kPixSumStride);   // item: jitter word's slot
    float* it_t = reinterpret_cast<float*>(it_i + 64);                        // item: hit t
    int* it_c = reinterpret_cast<int*>(it_t + 64);                            // item: hit code
    uint8_t* codes = reinterpret_cast<uint8_t*>(it_c + 64);                   // pending samples
    __syncthreads();
    const bool frustum = SCN == SCN_SPHERE && L.n_snode > 0 && P.n_sph <= (int)kPixFrustumMax;
    // words a surface hit draws beyond its jitter, in pairs: one pair per area light (Direct)
    const uint32_t NLD = INTEG == XRT_INTEGRATOR_DIRECT ? (uint32_t)P.n_lights : 0u;
    const uint32_t per_window = (64u + NLD) / (1u + NLD);   // most surface hits one window's chain holds
    // which paths ran (xrt_stats pix_*), per wave, added to KParams::stats when the wave retires:
    // windows, stride-4 windows, frustum lists, their overflows, shadow lists, their overflows, flushes
    uint32_t cnt_win = 0, cnt_s4 = 0, cnt_fr = 0, cnt_fro = 0, cnt_sl = 0, cnt_slo = 0, cnt_fl = 0;
    for (;;) {
        uint32_t s = 0;
        if (lane == 0) s = atomicAdd(work, 1u);
        s = (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
        if (s >= P.n_slots) break;   // every wave reaches this: the grid drains
        const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
        // the seeded state x[0..623] (k_seed) -> the circular buffer, 16 B per lane and load
        {
            const u32x4* src = reinterpret_cast<const u32x4*>(P.ring + (size_t)s * kRing);
            u32x4 v[3];
#pragma unroll
            for (int k = 0; k < 3; ++k)
                v[k] = __builtin_nontemporal_load(src + min((uint32_t)lane + 64u * k, kMT / 4 - 1u));
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if ((uint32_t)lane + 64u * k < kMT / 4) reinterpret_cast<u32x4*>(st)[lane + 64 * k] = v[k];
            wave_sync();
        }
        const int nlist = frustum ? pix_frustum<SCN>(P, L, col, row, list, lane) : -1;
        cnt_fr += nlist >= 0 ? 1u : 0u;
        cnt_fro += frustum && nlist < 0 ? 1u : 0u;
        f4 lsph = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // lane e: list entry e's sphere and index
        int lk = 0;
        if (lane < nlist) {
            const int j = list[lane];
            lsph = L.ssph[j];
            lk = L.sbk[j] & 0x3fffffff;
        }
        // DEFER with one light: the pixel's shadow-ray occluders (the LDS list is free again)
        int nsl = -1;
        f4 ssph = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (DEFER && kPixShadowList && P.n_lights == 1 && nlist >= 1 && nlist <= 4) {
            wave_sync();   // every lane has read its camera-list entry
            nsl = pix_shadow_list(P, L, lsph, nlist, list, lane);
            if (lane < nsl) ssph = L.ssph[list[lane]];
            cnt_sl += nsl >= 0 ? 1u : 0u;
            cnt_slo += nsl < 0 ? 1u : 0u;
        }
        float* px = P.fb + 3 * ((size_t)col + (size_t)P.width * row);
        float acc = lane < 3 ? px[lane] : 0.0f;   // lane c < 3: channel c of the running sum
        uint32_t o = kMT, g = kMT, k = 0;        // next draw x[o]; x[0 .. g) generated
        uint32_t nsh = 0, nrej = 0;
        uint32_t qn = 0, pn = 0, pw = 0;         // DEFER: queued items, pending samples, windows since a flush
        bool s4next = false;                     // the next window is a stride-4 window

        // Image::addPixel in sample order for the lanes of vm (lane order), each with value r:
        // ranked into the sum buffer, then added one after the other by lanes 0..2 (a channel each)
        auto add_in_order = [&](uint64_t vm, v3 r) {
            if ((vm >> lane) & 1ull) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(vm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)vm, 0u));
                sum[rank] = r.x, sum[kPixSumStride + rank] = r.y, sum[2 * kPixSumStride + rank] = r.z;
            }
            wave_sync();
            if (lane < 3) {
                const float* q = sum + kPixSumStride * lane;
                const f4* q4 = reinterpret_cast<const f4*>(q);
                const uint32_t nv = (uint32_t)__builtin_popcountll(vm);
                uint32_t j = 0;
                for (; j + 8 <= nv; j += 8) {
                    const f4 a = q4[j / 4], b = q4[j / 4 + 1];
                    acc = acc + a.x, acc = acc + a.y, acc = acc + a.z, acc = acc + a.w;
                    acc = acc + b.x, acc = acc + b.y, acc = acc + b.z, acc = acc + b.w;
                }
                for (; j < nv; ++j) acc = acc + q[j];
            }
            wave_sync();   // the buffer is rewritten next time
        };
        // integrate(...) / pdf (pinhole pdf 1) and the invalid-radiance check (Src/renderer.cpp:53-73)
        auto invalid = [](v3 r) {
            return __builtin_isnan(r.x) || __builtin_isnan(r.y) || __builtin_isnan(r.z) || __builtin_isinf(r.x) ||
                   __builtin_isinf(r.y) || __builtin_isinf(r.z) || r.x < 0.0f || r.y < 0.0f || r.z < 0.0f;
        };
        // DirectIntegrator's light loop for a sample at surface S (Src/integrator.h:94-110), every
        // lane (the shadow rays are a wave walk); `shade`: this lane's sample hit a surface
        auto direct_light = [&](bool shade, const Surf& S, int obj, LdsRng& rng, v3& rad) {
            for (int l = 0; l < P.n_lights; ++l) {
                v3 wi = mk(0, 0, 0), Lv = mk(0, 0, 0);
                float tmax = 0.0f, pdf = 0.0f;
                if (shade) Lv = light_sample(L.light[l], S.pos, wi, pdf, tmax, rng);
                const bool ray = shade && pdf != 0.0f;
                const float bias = 0.01f;
                nsh += ray ? 1u : 0u;
                bool vis = true;
                if (nsl >= 0) vis = !occluded_list(ssph, nsl, S.pos + S.ng * bias, wi, tmax - bias, ray);
                else if (kPixPacket) vis = !occluded_w<SCN>(P, L, S.pos + S.ng * bias, wi, tmax - bias, ray);
                else if (ray) vis = !occluded_l<SCN>(P, L, S.pos + S.ng * bias, wi, tmax - bias);
                if (ray) {
                    const float cosv = smax(0.0f, dot(S.ng, wi));
                    const v3 fr = eval_bxdf(L.obj[obj]);
                    rad = rad + div3s(((fr * (float)vis) * Lv) * cosv, pdf);
                }
            }
        };
        // DEFER: shade the queue (lane i: item i), then add the pending samples in order
        auto flush = [&]() {
            const bool act = (uint32_t)lane < qn;
            v3 rad = mk(0, 0, 0);
            Surf S;
            int obj = -1;
            LdsRng rng{st, act ? it_i[lane] : 0u};
            if (act) {
                // the item's camera ray again (its jitter words), and its hit record
                const float u = div_w(P, (float)(int)col + rng.next());
                const float v = div_h(P, (float)(int)row + rng.next());
                v3 ro, rd;
                camera_ray(P, u, v, ro, rd);
                HitRec h;
                h.t = it_t[lane], h.u = h.v = 0.0f, h.code = it_c[lane], h.surf = -1, h.dp = -1, h.t1 = kINF;
                h.st = h.su = h.sv = h.du = h.dv = 0.0f;
                obj = surface_l<SCN>(L, ro, rd, h, S);
            }
            direct_light(act, S, obj, rng, rad);
            const v3 r = rad / 1.0f;
            const uint64_t badm = __ballot(act && invalid(r));
            if (act) ires[lane] = r.x, ires[kPixSumStride + lane] = r.y, ires[2 * kPixSumStride + lane] = r.z;
            wave_sync();
            for (uint32_t base = 0; base < pn; base += 64) {
                const uint32_t m = base + (uint32_t)lane;
                const bool in = m < pn;
                const uint32_t code = in ? codes[m] : 0u;
                v3 val = mk((float)0.18, (float)0.18, (float)0.18);   // miss: Vec3f(0.18) / 1
                bool ok = true;
                if (code == 255u) {
                    val = mk(0, 0, 0) / 1.0f;
                } else if (code >= 128u) {
                    const uint32_t i = code - 128u;
                    val = mk(ires[i], ires[kPixSumStride + i], ires[2 * kPixSumStride + i]);
                    ok = !((badm >> i) & 1ull);
                } else if (code > 0u) {
                    val = ld3(L.light[code - 1u].Le) / 1.0f;
                    ok = !invalid(val);
                }
                const uint64_t vm = __ballot(in && ok);
                nrej += (uint32_t)(__builtin_popcountll(__ballot(in)) - __builtin_popcountll(vm));
                add_in_order(vm, val);
            }
            qn = 0, pn = 0, pw = 0;
            ++cnt_fl;
        };

        while (k < P.spp) {
            const uint32_t rem = P.spp - k;
            // candidates that can lie on the chain: rem samples advance at most 1 + NLD each
            // stride-4 windows (DEFER, one light): after a window whose samples all hit a
            // surface, the candidates sit 4 words apart — the offsets of a run of hits — and
            // the window ends at the first candidate that is not a hit (its successor lies
            // between two candidates).  Queued items are flushed before and after it, so its
            // 258 words and its items' stay within the 624-word buffer.
            const bool s4 = DEFER && NLD == 1 && kPixStride4 && s4next && rem >= 64u;
            if (s4 && qn) flush();
            const uint32_t stride = s4 ? 4u : 2u;
            ++cnt_win;
            cnt_s4 += s4 ? 1u : 0u;
            const uint32_t span = rem >= 64u ? 64u : min(64u, rem * (1u + NLD));
            const uint32_t need = o + stride * span + 2u * NLD;   // words this window may read
            while (g < need) {
                pix_gen(st, g, lane);
                g += kPixChunk;
            }
            // the candidate sample at offset o + 2·lane: jitter, camera ray, Scene::intersect
            // (Src/renderer.cpp:44-53)
            const bool cand = (uint32_t)lane < span;
            uint32_t ci = (o % kMT) + stride * (uint32_t)lane;
            if (ci >= kMT) ci -= kMT;
            LdsRng rng{st, ci};
            v3 ro = mk(0, 0, 0), rd = mk(0, 0, 0);
            Surf S;
            HitRec h;
            int obj = -1, kind = 0;   // 0 miss, 1 area light, 2 surface
            if (cand) {
                const float u = div_w(P, (float)(int)col + rng.next());
                const float v = div_h(P, (float)(int)row + rng.next());
                camera_ray(P, u, v, ro, rd);
            }
            if (nlist >= 0) closest_list(lsph, lk, nlist, ro, rd, h, cand);
            else if (kPixPacket) closest_w<SCN>(P, L, ro, rd, h, cand);
            else if (cand) closest_l<SCN>(P, L, ro, rd, h);
            if (cand) {
                obj = surface_l<SCN>(L, ro, rd, h, S);
                kind = obj < 0 ? 0 : (L.obj[obj].light >= 0 ? 1 : 2);
            }
            // the chain through the window (scalar): from candidate 0 (the next sample), a
            // sample at candidate q moves to q + 1, or to q + 1 + NLD after a surface hit
            const uint64_t smask = NLD ? (uint64_t)__ballot(kind == 2) : 0ull;
            uint64_t M = 0;
            uint32_t cnt = 0, pos = 0;   // pos: words consumed / 2
            if (s4) {
                const uint64_t nh = ~smask;   // span == 64
                const uint32_t last = nh ? (uint32_t)__builtin_ctzll(nh) : 63u;
                M = last == 63u ? ~0ull : ((1ull << (last + 1u)) - 1ull);
                cnt = last + 1u;
                pos = 2u * last + (((smask >> last) & 1ull) ? 2u : 1u);
                s4next = nh == 0ull;
            } else if (NLD == 1 && rem >= 64u) {
                // one light, a full window (bit-parallel): a surface-hit sample skips the next
                // candidate, so within a run of surface hits that starts on the chain every
                // other candidate is a sample.  kill = the surface hits on the chain: a run's
                // even offsets from its start (the carry of s + start clears exactly the runs
                // that start at even positions), M = every candidate not right after a kill.
                constexpr uint64_t kEven = 0x5555555555555555ull;
                const uint64_t start = smask & ~(smask << 1);
                const uint64_t even_runs = smask & ~(smask + (start & kEven));
                const uint64_t kill = (even_runs & kEven) | (smask & ~even_runs & ~kEven);
                M = ~(kill << 1);
                cnt = (uint32_t)__builtin_popcountll(M);
                const uint32_t last = 63u - (uint32_t)__builtin_clzll(M);
                pos = last + 1u + (uint32_t)((kill >> last) & 1ull);
            } else {
                while (pos < 64u && cnt < rem) {
                    const uint64_t ahead = smask >> pos;
                    const uint32_t q = ahead ? pos + (uint32_t)__builtin_ctzll(ahead) : 64u;
                    uint32_t run = q - pos;   // samples without a surface hit, then the one at q
                    if (run > rem - cnt) run = rem - cnt;
                    M |= (run == 64u ? ~0ull : ((1ull << run) - 1ull)) << pos;
                    cnt += run;
                    pos += run;
                    if (cnt == rem || q == 64u) break;   // sample budget reached, or the window ends
                    M |= 1ull << q;   // pos == q here
                    ++cnt;
                    pos = q + 1u + NLD;
                }
            }
            if (!s4) s4next = kPixStride4 && DEFER && NLD == 1 && cnt >= 32u && (M & ~smask) == 0ull;
            const bool member = (M >> lane) & 1ull;
            if constexpr (DEFER) {
                // the window's samples as pending codes, its surface hits as queue items
                const bool shade = member && kind == 2;
                const uint64_t im = __ballot(shade);
                if (member) {
                    uint32_t code = 0u;
                    if (kind == 1) code = dot(rd, S.ns) < 0.0f ? 1u + (uint32_t)L.obj[obj].light : 255u;   // light_Le
                    if (shade) code = 128u + qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0u));
                    codes[pn + __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u))] = (uint8_t)code;
                }
                if (shade) {
                    const uint32_t at = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0u));
                    it_i[at] = ci, it_t[at] = h.t, it_c[at] = h.code;
                }
                qn += (uint32_t)__builtin_popcountll(im);
                pn += cnt, ++pw;
                k += cnt;
                o += 2u * pos;
                wave_sync();
                // a stride-4 window spans 258 words: its items are shaded before the next window
                if (s4 || pw == 3u || qn + (s4next ? 64u : per_window) > 64u || k >= P.spp) flush();
            } else {
                v3 rad = mk(0, 0, 0);
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    // DirectIntegrator::integrate (Src/integrator.h:82-119)
                    if (member && kind == 0) rad = mk((float)0.18, (float)0.18, (float)0.18);
                    if (member && kind == 1) rad = light_Le(L.light[L.obj[obj].light], S.ns, rd);
                    direct_light(member && kind == 2, S, obj, rng, rad);
                } else if (member && obj >= 0) {
                    rad = normal_color(S.ns);   // NormalIntegrator::integrate (Src/integrator.h:28-37)
                }
                const v3 r = rad / 1.0f;
                const uint64_t vm = __ballot(member && !invalid(r));
                nrej += (uint32_t)(__builtin_popcountll(M) - __builtin_popcountll(vm));
                add_in_order(vm, r);
                k += cnt;
                o += 2u * pos;
            }
        }
        if (lane < 3) px[lane] = acc;
        // the pixel's counters, as the per-slot schedules leave them for k_finish: one
        // Scene::intersect per sample, its shadow rays and rejects, the stream cursor, and the
        // twists a std::mt19937 makes to produce x[624 .. o)
        for (int off = 32; off > 0; off >>= 1) nsh += __shfl_down(nsh, off);
        if (lane == 0) {
            P.c_seg[s] = P.spp;
            P.c_shadow[s] = nsh;
            P.c_rej[s] = nrej;
            P.c_stall[s] = 0;
            P.rng_c[s] = o;
            P.rng_g[s] = kMT + kMT * ((o - kMT + kMT - 1u) / kMT);
            P.sample_k[s] = P.spp;
            P.state[s] = ST_DONE;
        }
    }
    if (lane == 0) {   // wave-uniform counts: one add per counter and wave
        const uint32_t c[7] = {cnt_win, cnt_s4, cnt_fr, cnt_fro, cnt_sl, cnt_slo, cnt_fl};
#pragma unroll
        for (int q = 0; q < 7; ++q)
            if (c[q]) atomicAdd(P.stats + kStatsPix + q, (unsigned long long)c[q]);
    }
}

}  // namespace xrt

#include "launch.h"

namespace xrt {

bool use_pixel(const KParams& P) {
    // within the design budget and what this device gives a workgroup (an oversize k_pixel
    // launch would fail; the per-slot schedule serves the scene instead)
    return one_hit(P.integrator) && step_lds_bytes(P) != 0 && pix_lds_bytes(P) <= kPixLds &&
           pix_lds_bytes(P) <= P.lds_max;
}

size_t pix_lds_bytes(const KParams& P) {
    const bool defer = pix_defer_rt(P);
    const uint32_t bs = defer ? (uint32_t)XRT_PIX_DEFER_BLOCK : (uint32_t)kPixBlock;
    return pix_wave_off(P) + (size_t)(bs / 64) * (defer ? kPixWaveDeferLds : kPixWaveLds);
}

template <int SCN, int INTEG>
static hipError_t pixel_i(const KParams& P, uint32_t* work, hipStream_t st) {
    constexpr int BS = pix_block(SCN, INTEG);
    const size_t lds = pix_lds_bytes(P);
    auto kern = k_pixel<SCN, INTEG, BS>;
    // persistent grid: as many blocks as fit on the device at once (LDS and VGPR bound), at
    // most one wave per pixel
    int dev = 0, ncu = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BS, lds);
    if (e != hipSuccess) return e;
    const uint64_t want = ((uint64_t)P.n_slots + BS / 64 - 1) / (BS / 64);
    const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, per_cu) * ncu, want));
    hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(BS), lds, st, P, work);
    return hipGetLastError();
}

template <int SCN>
static hipError_t pixel_s(const KParams& P, uint32_t* work, hipStream_t st) {
    if (P.integrator == XRT_INTEGRATOR_DIRECT) return pixel_i<SCN, XRT_INTEGRATOR_DIRECT>(P, work, st);
    return pixel_i<SCN, XRT_INTEGRATOR_NORMAL>(P, work, st);
}

hipError_t launch_pixel(const KParams& P, uint32_t* work, hipStream_t st) {
    if (!use_pixel(P)) return hipErrorInvalidValue;
    if (hipMemsetAsync(work, 0, sizeof(uint32_t), st) != hipSuccess) return hipErrorInvalidValue;
    switch (P.scene_kind) {
        case SCN_TRI: return pixel_s<SCN_TRI>(P, work, st);
        case SCN_SPHERE: return pixel_s<SCN_SPHERE>(P, work, st);
        default: return pixel_s<SCN_MIXED>(P, work, st);
    }
}

}  // namespace xrt
