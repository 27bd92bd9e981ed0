// spec.hip — speculative sample starts for the merged schedule's group layout (16 slots per
// wave, 4 lanes per slot: the layout of a multi-GPU row shard and of a frame's tail).
//
// NormalRenderer::doRender (Src/renderer.cpp:29-81) runs a pixel's samples in order on one
// mt19937 stream, so a slot's samples form a chain of dependent traces ("visits"): a
// GIIntegrator sample (Src/integrator.h:205-287) traces its camera ray, then up to maxDepth - 1
// bounces, and the next sample's camera ray can only be traced once the sample has ended —
// its jitter words follow the words the sample drew, and that count depends on what the
// sample's traces hit.  At a row shard of an 8-GPU frame that chain, not the GPU's throughput,
// sets the frame time.
//
// The chain is shortened exactly.  When a trace may end its sample, the words the sample will
// have drawn are one of three counts, each known before the trace: nothing more (the ray
// misses, or at depth 0 hits a light), one (the Russian-roulette word at depth > 0: it kills
// the path, or the path hits a light), or five (RR + the light sample + the BSDF sample of a
// surface hit at the last depth).  So with the trace of a sample's extension ray, the slot's
// other lanes trace the camera rays a successor starting at each of those offsets would trace
// (lanes 1, 2, 3: offsets 0, 1, 5), and in the same visit, once the trace tells which offset
// is the real one, that lane shades the successor's first hit while lane 0 shades the ending
// sample's last one — the same shading code on two lanes of one quad, so SIMT issues it once.
// A full-depth sample then costs one visit fewer: C2's longest chain 2,803 -> 1,780 visits
// (tools/sim/spec_sim.py).
//
// Lanes of a slot's quad and their registers:
//   lane 0  the sample in progress (A): path state, its pending NEE shadow ray, the pixel sum
//   lane 1  candidate offset 0; holds an ended sample whose last shadow ray is still in flight
//   lane 2  candidate offset 1; holds an ended sample waiting for lane 1's to be added first
//   lane 3  candidate offset 5
// Each lane draws from its own window of the stream (6 words at cursor + its offset), so the
// successor's lane finds its light and BSDF words right after its jitter words.  The trace of
// a visit takes lane 0's extension ray and shadow ray and lane 1's shadow ray (group trace:
// every lane of the quad tests a quarter of the candidate triangles); a candidate's camera ray
// is tested by its own lane against the pixel's camera list (k_camlist).  Every draw, ray,
// hit and float operation is the reference's, and samples are added to the pixel sum in
// sample order: bit-identical to the other schedules (tests/test_gpu_spec.py).
#include "launch.h"
#include "merged.h"
#include "path_common.h"

namespace xrt {

// quad broadcasts (DPP quad_perm [l, l, l, l]); every lane of the quad must be active
template <int L>
__device__ __forceinline__ uint32_t qb(uint32_t x) {
    return dpp32<L | (L << 2) | (L << 4) | (L << 6)>(x);
}
template <int L>
__device__ __forceinline__ float qbf(float x) {
    return __uint_as_float(qb<L>(__float_as_uint(x)));
}
template <int L>
__device__ __forceinline__ v3 qb3(v3 v) {
    return mk(qbf<L>(v.x), qbf<L>(v.y), qbf<L>(v.z));
}
// from lane `src` of the quad (quad-uniform, dynamic): ds_bpermute
__device__ __forceinline__ uint32_t qsel(uint32_t x, int src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)x);
}
__device__ __forceinline__ float qself(float x, int src_lane) { return __uint_as_float(qsel(__float_as_uint(x), src_lane)); }
__device__ __forceinline__ v3 qsel3(v3 v, int src_lane) {
    return mk(qself(v.x, src_lane), qself(v.y, src_lane), qself(v.z, src_lane));
}

// ------------------------------------------------------------------ camera lists ----
// The triangles a camera ray of pixel (col, row) can hit, for scenes of at most 64 triangles
// (KParams::camlist[slot] = {mask bits 0-31, mask bits 32-63, covering triangle or -1, 0}).
// Every camera ray of a pixel leaves o through the pixel's jitter square, so it lies in the
// cone over the square's corner directions D0..D3 (widened by 0.01 pixel, as pix_frustum).
// A triangle is left out when the cone and the triangle's cone from o are separated by one of
// the cone's four side planes or one of the triangle's three edge planes through o (for two
// convex cones with a common apex that is an exact test), each with a margin of 1e-4 of the
// vectors' scale — far above the float error of these tests and of Moller-Trumbore's
// acceptance at an edge.  A triangle that every corner ray hits with barycentric margin 1e-3
// (so every ray of the cone does: u and v are ratios of linear functions of the direction)
// hides every triangle that lies wholly beyond its plane by a margin: such a triangle's t is
// larger on every ray of the cone, so it is never the (t, index) minimum.  When one triangle
// is left and it covers the cone, every camera ray of the pixel hits it: `covering` is then
// its index and the candidate rays need no test (the shading recomputes t, u, v anyway).
__global__ __launch_bounds__(kBlock) void k_camlist(KParams P) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= P.n_slots) return;
    const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
    const float m = 0.01f;
    const float u0 = ((float)col - m) / P.fw, u1 = ((float)col + (1.0f + m)) / P.fw;
    const float v0 = ((float)row - m) / P.fh, v1 = ((float)row + (1.0f + m)) / P.fh;
    const float* x = P.c2w;
    auto world = [&](float u, float v) {
        const v3 dir = mk((2.0f * u - 1.0f) * P.scale, (1.0f - 2.0f * v) * P.scale / P.aspect, -1.0f);
        return mk(dir.x * x[0] + dir.y * x[4] + dir.z * x[8], dir.x * x[1] + dir.y * x[5] + dir.z * x[9],
                  dir.x * x[2] + dir.y * x[6] + dir.z * x[10]);
    };
    v3 D[4] = {world(u0, v0), world(u1, v0), world(u1, v1), world(u0, v1)};
    const v3 Dc = (D[0] + D[1]) + (D[2] + D[3]);
    v3 n[4];
    float Dl[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        n[k] = cross(D[k], D[(k + 1) & 3]);
        const float sg = dot(n[k], Dc) < 0.0f ? -1.0f : 1.0f;
        n[k] = n[k] * (sg / length(n[k]));   // unit, pointing into the cone
        Dl[k] = length(D[k]);
    }
    const v3 o = mk(x[12], x[13], x[14]);
    const float tol = 1e-4f;
    uint64_t mask = 0, cover = 0;
    for (int t = 0; t < P.n_tris && t < 64; ++t) {
        const v3 p0 = xyz(P.tri[3 * t]), e1 = xyz(P.tri[3 * t + 1]), e2 = xyz(P.tri[3 * t + 2]);
        const v3 a[3] = {p0 - o, (p0 + e1) - o, (p0 + e2) - o};
        const float al[3] = {length(a[0]), length(a[1]), length(a[2])};
        bool out = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // the cone's side planes
            bool all = true;
#pragma unroll
            for (int q = 0; q < 3; ++q) all = all && dot(n[k], a[q]) < -tol * (al[q] + 1.0f);
            out = out || all;
        }
#pragma unroll
        for (int e = 0; e < 3; ++e) {   // the triangle's edge planes through o
            const v3 pa = a[e], pb = a[(e + 1) % 3], pc = a[(e + 2) % 3];
            v3 pn = cross(pa, pb);
            const float sc = al[e] * al[(e + 1) % 3];
            const float side = dot(pn, pc);
            if (!(__builtin_fabsf(side) > tol * sc * al[(e + 2) % 3])) continue;   // o near the triangle's plane
            if (side < 0.0f) pn = pn * -1.0f;
            bool all = true;
#pragma unroll
            for (int k = 0; k < 4; ++k) all = all && dot(pn, D[k]) < -tol * sc * Dl[k];
            out = out || all;
        }
        if (out) continue;
        mask |= 1ull << t;
        // does every corner ray hit it well inside (Moller-Trumbore, barycentric margin 1e-3)?
        bool cov = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const v3 pvec = cross(D[k], e2);
            const float det = dot(e1, pvec);
            const v3 tvec = o - p0;
            const float uu = dot(tvec, pvec) / det;
            const v3 qvec = cross(tvec, e1);
            const float vv = dot(D[k], qvec) / det, tt = dot(e2, qvec) / det;
            cov = cov && __builtin_fabsf(det) > 1e-6f * length(e1) * length(e2) * Dl[k] && uu >= 1e-3f &&
                  vv >= 1e-3f && uu + vv <= 1.0f - 1e-3f && tt > 0.0f;
        }
        if (cov) cover |= 1ull << t;
    }
    // a covering triangle hides the triangles wholly beyond its plane (as seen from o)
    uint64_t keep = mask;
    for (uint64_t cb = cover; cb; cb &= cb - 1ull) {
        const int t = __builtin_ctzll(cb);
        const v3 p0 = xyz(P.tri[3 * t]);
        const v3 nt = cross(xyz(P.tri[3 * t + 1]), xyz(P.tri[3 * t + 2]));
        const float ntl = length(nt);
        const float so = dot(nt, o - p0);
        const float sg = so < 0.0f ? -1.0f : 1.0f;
        const float ol = length(o - p0);
        for (uint64_t b = mask & ~(1ull << t); b; b &= b - 1ull) {
            const int t2 = __builtin_ctzll(b);
            const v3 q0 = xyz(P.tri[3 * t2]);
            const v3 qs[3] = {q0, q0 + xyz(P.tri[3 * t2 + 1]), q0 + xyz(P.tri[3 * t2 + 2])};
            bool beyond = so != 0.0f;
#pragma unroll
            for (int q = 0; q < 3; ++q)
                beyond = beyond && sg * dot(nt, qs[q] - p0) < -tol * ntl * (length(qs[q] - p0) + ol);
            if (beyond) keep &= ~(1ull << t2);
        }
    }
    const int covering = (__builtin_popcountll(keep) == 1 && (keep & cover)) ? __builtin_ctzll(keep) : -1;
    P.camlist[s] = make_uint4((uint32_t)keep, (uint32_t)(keep >> 32), (uint32_t)covering, 0u);
}

// ---------------------------------------------------------------- the step kernel ----
template <int SPW, int G>
__global__ __launch_bounds__(kBlock, XRT_STEP_WAVES) void k_step_spec(
    const KParams* __restrict__ Pp, const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
    uint32_t* __restrict__ out, uint32_t* out_count, uint32_t* zero_count, uint32_t visits) {
    // G lanes per slot: the slot's quad (roles below) and, for G = 8 or 16, replicas of it that
    // run the same code on the same state and only widen the slot's group trace
    static_assert((G == 4 || G == 8 || G == 16) && SPW * G == 64, "a slot per group of 4, 8 or 16 lanes");
    constexpr int NL = 1;            // one area light (use_step_spec)
    constexpr int NW = 6;            // stream words per lane window
    constexpr uint32_t kSpan = kSpecDraws;   // the quad's windows reach cursor + 10
    const KParams& P = *Pp;
    extern __shared__ __attribute__((aligned(16))) f4 lds_s[];
    char* lb = reinterpret_cast<char*>(lds_s);
    const int tid = threadIdx.x, lane = tid & 63;
    LScene L;
    const StepLayout Lo = step_layout(P);
    L.tri = reinterpret_cast<const f4*>(lb + Lo.tri);
    L.tng = reinterpret_cast<const f4*>(lb + Lo.tng);
    L.nrm = reinterpret_cast<const f4*>(lb + Lo.nrm);
    L.box = reinterpret_cast<const DObjBox*>(lb + Lo.box);
    L.obj = reinterpret_cast<const DObj*>(lb + Lo.obj);
    L.light = reinterpret_cast<const DLight*>(lb + Lo.light);
    const DObjPlane* lplane = reinterpret_cast<const DObjPlane*>(lb + merged_plane_off(Lo));
    uint32_t* scratch = reinterpret_cast<uint32_t*>(lb + merged_wave_off(P, Lo) + (tid >> 6) * sizeof(MergedWave<NL>));
    static_assert(sizeof(MergedWave<NL>) >= kMT * 4, "the wave's scratch doubles as the refill buffer");
    lds_copy(const_cast<f4*>(L.tri), P.tri, 3 * P.n_tris, tid);
    lds_copy(const_cast<f4*>(L.tng), P.tri_ng, P.n_tris, tid);
    lds_copy(const_cast<f4*>(L.nrm), P.tri_nrm, 3 * P.n_tris, tid);
    lds_copy(const_cast<DObj*>(L.obj), P.objs, P.n_objs, tid);
    lds_copy(const_cast<DLight*>(L.light), P.lights, P.n_lights, tid);
    lds_copy(const_cast<DObjBox*>(L.box), P.obj_box, P.n_objs, tid);
    lds_copy(const_cast<DObjPlane*>(lplane), P.obj_plane, P.n_objs, tid);
    __syncthreads();
    zero_parts(P, zero_count);
    // experiment builds (XRT_PHASE_CLOCK, tools/phase.sh): shader-clock cycles per phase of a
    // visit, per wave: loop head, trace, candidates, end test, shading, moves, cursor + reload,
    // launch prologue / epilogue
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t_ph = XRT_PHASE_CLOCK ? clock64() : 0ull;
    auto tick = [&](int q) {
        if constexpr (XRT_PHASE_CLOCK) {
            const unsigned long long t = clock64();
            ph[q] += t - t_ph;
            t_ph = t;
        }
    };
    const int u = lane & 3;                                   // the lane's role in its quad
    const int qbase = lane & ~3;
    const uint32_t off = u == 2 ? 1u : (u == 3 ? 5u : 0u);    // its window / candidate offset
    const PartIter it = part_iter(P, count, (kBlock / 64) * SPW);
    const uint32_t spp = P.spp, max_depth = P.max_depth, width = P.width;
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + (uint32_t)(tid >> 6) * SPW + (uint32_t)lane / G;
        const bool own = lane / G < SPW && i < it.n;
        const bool lead = own && (lane & (G - 1)) == 0;   // writes the slot back
        const uint32_t s = own ? list[it.p * P.part_cap + i] : 0;
        uint32_t st = own ? glb<gu32>(P.state)[s] : ST_DONE;
        st &= ~ST_RNGREQ;
        const bool live = !(st & ST_DONE);
        uint32_t g = 0, cc = 0, k = 0, kst = 0;
        // the lane's context (role above): path state, one pending NEE shadow ray (GI with one
        // light: folded as in k_step_merged, c1 = thr * (0 + (0 + c1)), c0z its +-0 / NaN codes)
        v3 thr = mk(1, 1, 1), rad = mk(0, 0, 0), o = mk(0, 0, 0), d = mk(0, 0, 0);
        uint32_t depth = 0, shm = 0, c0z = 0;
        v3 so = mk(0, 0, 0), sd = mk(0, 0, 0), c1 = mk(0, 0, 0);
        float stm = 0.0f;
        bool has = false;   // lane 0: a sample in progress, its extension ray (o, d) pending
        bool fin = false;   // lane 1: an ended sample waiting for its shadow ray; lane 2: one waiting its turn
        v3 acc = mk(0, 0, 0);
        RngRegs<NW> rng;
        rng.c = 0;
        const uint32_t* ring = P.ring + (size_t)s * kRing;
        const uint32_t col = s % width, row = P.shard_index + P.shard_count * (s / width);
        float* px = P.fb + 3 * ((size_t)col + (size_t)width * row);
        uint64_t cm = 0;    // the pixel's camera list
        int cov = -1;
        if (live) {
            g = glb<gu32>(P.rng_g)[s];
            cc = glb<gu32>(P.rng_c)[s];
            depth = glb<gu32>(P.depth)[s];
            k = glb<gu32>(P.sample_k)[s];
            kst = k;
            if (!(st & ST_REGEN)) {
                thr = ld3g(P.thr, s), rad = ld3g(P.rad, s);
                o = ld3g(P.ray_o, s), d = ld3g(P.ray_d, s);
                has = true;
                kst = k + 1;
            }
            gf32* pxg = glb<gf32>(px);
            acc = mk(pxg[0], pxg[1], pxg[2]);
            const uint4 cl = P.camlist[s];
            cm = (uint64_t)cl.x | ((uint64_t)cl.y << 32);
            cov = (int)cl.z;
            rng.c = cc + off;
            rng.load(ring);
        }
        st &= ~ST_REGEN;
        if (u != 0) has = false;
        uint32_t nseg = 0, nsh = 0, nrej = 0;
        // Image::addPixel of a finished sample (Src/renderer.cpp:57-75), lane 0
        auto finish = [&](v3 r0) {
            const v3 r = r0 / 1.0f;
            if (__builtin_isnan(r.x) || __builtin_isnan(r.y) || __builtin_isnan(r.z) || __builtin_isinf(r.x) ||
                __builtin_isinf(r.y) || __builtin_isinf(r.z) || r.x < 0.0f || r.y < 0.0f || r.z < 0.0f) {
                ++nrej;
            } else {
                acc = acc + r;
            }
            ++k;
        };
        // the quad's trace (every lane): lane 0's extension ray and shadow ray, lane 1's shadow
        // ray; then the shadow results and the finishes they complete, in sample order
        // (broadcast in place: lanes 1-3 hold no extension ray, and the shadow rays are dead once
        // traced — fewer registers live across the trace)
        auto trace_resolve = [&](bool ext_on, unsigned long long& best) {
            v3 so_t[3], sd_t[3];
            float stm_t[3];
            so_t[1] = qb3<1>(so), sd_t[1] = qb3<1>(sd), stm_t[1] = qbf<1>(stm);
            so_t[0] = so = qb3<0>(so), sd_t[0] = sd = qb3<0>(sd), stm_t[0] = stm = qbf<0>(stm);
            so_t[2] = sd_t[2] = mk(0, 0, 0), stm_t[2] = 0.0f;
            const uint32_t sh_t = (qb<0>(shm) & 1u) | ((qb<1>(shm) & 1u) << 1);
            o = qb3<0>(o), d = qb3<0>(d);
            uint32_t occ = 0;
            group_trace<2, G>(P.n_objs, L, lplane, lane, ext_on, o, d, sh_t, so_t, sd_t, stm_t, best, occ);
            // GIIntegrator: rad += thr * directL (folded into c1 / c0z when it was sampled)
            if (u <= 1 && shm) {
                rad = rad + (((occ >> u) & 1u) ? mk(zdecode(c0z & 3u), zdecode((c0z >> 2) & 3u), zdecode(c0z >> 4)) : c1);
                shm = 0;
            }
            const v3 r1 = qb3<1>(rad), r2 = qb3<2>(rad);
            const bool f1 = qb<1>(fin ? 1u : 0u) != 0u, f2 = qb<2>(fin ? 1u : 0u) != 0u;
            if (u == 0) {
                if (f1) finish(r1);
                if (f2) finish(r2);
            }
            if (u != 0) fin = false;
            k = qb<0>(k);
            if (k >= spp) st = ST_DONE;
        };
        __builtin_amdgcn_s_waitcnt(0);   // prologue loads done: the loop waits only on its own prefetches
        tick(7);
        for (uint32_t vis = 0; vis < visits; ++vis) {
            if (XRT_SPEC_TWIST) {
                // a slot whose windows would reach past its generated words twists its ring here,
                // the wave together as at the launch end (the block it overwrites is consumed:
                // fewer than kSpan words are left), so launches need not end for the RNG
                const bool need = live && !(st & ST_DONE) && g - cc < kSpan;   // group-uniform
                if (__ballot(need)) {
                    wave_refill(P, need && lead, s, g, lane, scratch);
                    // the new words are read back below by other lanes of this wave: stores
                    // done and this CU's L1 invalidated first
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
                    if (need) {
                        g += kMT;
                        rng.reload(ring);
                    }
                }
            }
            const bool act = live && !(st & ST_DONE) && g - cc >= kSpan;   // quad-uniform
            if (!__ballot(act || shm || fin)) break;
            tick(0);
            const bool has0 = qb<0>(has ? 1u : 0u) != 0u;
            const uint32_t depth0 = qb<0>(depth);
            unsigned long long best = ~0ull;
            trace_resolve(act && has0, best);
            tick(1);
            // ---- the candidates: the camera ray a successor starting at cursor + off traces
            // (Src/renderer.cpp:44-53), where a successor can start after this trace
            const bool more = kst < spp;
            const bool want_c = act && more && u >= 1 &&
                                (has0 ? (depth0 == 0 ? u == 1 : (u != 3 || depth0 + 1 >= max_depth)) : u == 1);
            // (lanes 1-3 hold no extension ray: the candidate takes their o, d and best registers)
            if (want_c) {
                const float jx = rng.next(), jy = rng.next();
                const float uu = div_w(P, (float)(int)col + jx);
                const float vv = div_h(P, (float)(int)row + jy);
                camera_ray(P, uu, vv, o, d);
                best = camlist_closest(L, make_uint4((uint32_t)cm, (uint32_t)(cm >> 32), (uint32_t)cov, 0u), o, d);
            }
            tick(2);
            // ---- does the sample in progress end with this trace, and after how many words? (lane 0)
            bool endA = false;
            uint32_t xoff = 0;
            if (u == 0 && act) {
                if (!has) {
                    endA = true;   // between samples: the next one starts at the cursor
                } else if (best == ~0ull) {
                    endA = true;   // miss
                } else {
                    const int ob = __float_as_int(L.tri[3 * (int)(uint32_t)best].w);
                    bool kill = false;
                    if (depth > 0) {
                        const float pr = smin(div_const(thr.x + thr.y + thr.z, 3.0f, kRcp3), 1.0f);
                        kill = canonical(mt_temper(rng.b[0])) >= pr;
                    }
                    const uint32_t rr = depth > 0 ? 1u : 0u;
                    if (kill || L.obj[ob].light >= 0) endA = true, xoff = rr;
                    else if (depth + 1 >= max_depth) endA = true, xoff = rr + 4u;
                }
            }
            endA = qb<0>(endA ? 1u : 0u) != 0u;
            xoff = qb<0>(xoff);
            const bool Bv = endA && more;   // a successor starts here
            const int bl = xoff == 0 ? 1 : (xoff == 1 ? 2 : 3);
            const bool isB = Bv && u == bl;
            const bool shadeA = u == 0 && act && has;
            tick(3);
            if (isB) {   // a fresh path from the candidate's camera ray (o, d) and closest hit (best)
                thr = mk(1, 1, 1), rad = mk(0, 0, 0), depth = 0;
                shm = 0;
            }
            // ---- shading: lane 0 the ending sample (A), lane bl the successor's first hit (B),
            // the same code (GIIntegrator::integrate's loop body, Src/integrator.h:214-284)
            bool ended = false;
            const uint32_t c_in = rng.c;
            if (shadeA || isB) {
                ++nseg;
                int hk = -1, obj = -1;
                float ht = kINF, hu = 0.0f, hv = 0.0f;
                if (best != ~0ull) {
                    hk = (int)(uint32_t)best;
                    const f4 ta = L.tri[3 * hk];
                    (void)ray_tri(o, d, xyz(ta), xyz(L.tri[3 * hk + 1]), xyz(L.tri[3 * hk + 2]), ht, hu, hv);
                    obj = __float_as_int(ta.w);
                }
                v3 pos = mk(0, 0, 0), ng = mk(0, 0, 0);
                if (hk >= 0) pos = ray_at(o, d, ht), ng = xyz(L.tng[hk]);
                bool alive = false;
                if (obj < 0) {
                    rad = rad + thr * mk(0.0f, 0.0f, 0.0f);
                    ended = true;
                } else {
                    alive = true;
                    if (depth > 0) {
                        const float pr = smin(div_const(thr.x + thr.y + thr.z, 3.0f, kRcp3), 1.0f);
                        if (rng.next() >= pr) alive = false, ended = true;
                        else thr = thr / mk(pr, pr, pr);
                    }
                    if (alive && L.obj[obj].light >= 0) {
                        if (depth == 0) rad = rad + thr * light_Le(L.light[L.obj[obj].light], tri_ns_l(L, hk, hu, hv), d);
                        alive = false, ended = true;
                    }
                }
                if (alive) {
                    const DObj& ob = L.obj[obj];
                    const v3 fr = ob.material == 1 ? mk(ob.fr[0], ob.fr[1], ob.fr[2]) : mk(0, 0, 0);
                    v3 wi = mk(0, 0, 0);
                    float tmax = 0.0f, pdf = 0.0f;
                    const v3 Lv = light_sample(L.light[0], pos, wi, pdf, tmax, rng);
                    if (pdf != 0.0f) {
                        ++nsh;
                        shm = 1;
                        const float bias = 0.01f;
                        so = pos + ng * bias, sd = wi, stm = tmax - bias;
                        const float cosv = smax(0.0f, dot(ng, wi));
                        const v3 cv1 = ((fr * Lv) * cosv) / pdf;
                        const v3 z = ((fr * 0.0f) * Lv) * cosv;
                        const v3 cv0 = pdf == pdf ? z : mk(pdf, pdf, pdf);
                        const v3 zero = mk(0, 0, 0);
                        c1 = thr * (zero + (zero + cv1));
                        const v3 w = thr * (zero + (zero + cv0));
                        c0z = zcode(w.x) | (zcode(w.y) << 2) | (zcode(w.z) << 4);
                    } else {
                        rad = rad + thr * mk(0.0f, 0.0f, 0.0f);   // no shadow ray: directL = 0
                    }
                    v3 nd = mk(0, 0, 0);
                    const bool lamb = ob.material == 1;
                    if (lamb) {
                        v3 dpdu, dpdv;
                        onb(tri_ns_l(L, hk, hu, hv), dpdu, dpdv);
                        nd = lambert_sample_f(ng, dpdu, dpdv, rng);
                    }
                    const float cosv = smax(0.0f, dot(nd, ng));
                    const v3 fc = fr * cosv;
                    thr = thr * (lamb ? mk(div_const(fc.x, kLambertPdf, kLambertPdfRcp),
                                           div_const(fc.y, kLambertPdf, kLambertPdfRcp),
                                           div_const(fc.z, kLambertPdf, kLambertPdfRcp))
                                      : fc / 1.0f);
                    o = pos + ng * 0.01f;
                    d = nd;
                    ++depth;
                    if (depth >= max_depth) ended = true;
                }
            }
            tick(4);
            // ---- the quad's new state
            const uint32_t usedA = qb<0>(rng.c - c_in);          // words lane 0 drew in the shading
            const uint32_t usedB = qsel(rng.c - cc - off, qbase + bl);   // lane bl: jitter + its shading
            const bool pendA = qb<0>((endA && shm) ? 1u : 0u) != 0u;   // A ended with its shadow ray in flight
            // A ended: its radiance is added now, or (shadow ray pending) its context moves to lane 1
            // (one register at a time: few extra registers live)
            if (endA && qb<0>(has ? 1u : 0u)) {
                const bool mv = u == 1 && pendA;
                auto to1 = [&](float& x) { const float y = qbf<0>(x); x = mv ? y : x; };
                to1(rad.x), to1(rad.y), to1(rad.z);
                if (u == 0 && !pendA) finish(rad);
                to1(so.x), to1(so.y), to1(so.z), to1(sd.x), to1(sd.y), to1(sd.z);
                to1(c1.x), to1(c1.y), to1(c1.z), to1(stm);
                const uint32_t c0za = qb<0>(c0z);
                if (mv) c0z = c0za, shm = 1, fin = true;
                if (u == 0) has = false, shm = 0;
            }
            // B: the successor's state moves from lane bl to lane 0 (or, ended at its camera ray,
            // it is added after A — by lane 2 next visit when A's shadow ray is still in flight)
            if (Bv) {
                const int src = qbase + bl;
                const bool bend = qsel(ended ? 1u : 0u, src) != 0u;
                const bool take = u == 0 && !bend;
                auto from = [&](float& x) { const float y = qself(x, src); x = take ? y : x; };
                auto fromu = [&](uint32_t& x) { const uint32_t y = qsel(x, src); x = take ? y : x; };
                {   // the radiance: taken by lane 0, or the finished successor's by lane 0 / lane 2
                    const v3 brad = qsel3(rad, src);
                    if (take) rad = brad;
                    if (u == 0 && bend && !pendA) finish(brad);
                    if (u == 2 && bend && pendA) rad = brad, fin = true;
                }
                from(o.x), from(o.y), from(o.z), from(d.x), from(d.y), from(d.z);
                from(thr.x), from(thr.y), from(thr.z);
                from(so.x), from(so.y), from(so.z), from(sd.x), from(sd.y), from(sd.z);
                from(c1.x), from(c1.y), from(c1.z), from(stm);
                fromu(depth), fromu(c0z), fromu(shm);
                if (take) has = true;
                if (u == 3 || u == 2 || (u == 1 && !pendA)) shm = 0;
                ++kst;
            }
            tick(5);
            // the quad's cursor and the next windows
            if (act) cc = endA ? (Bv ? cc + xoff + usedB : cc + xoff) : cc + usedA;
            k = qb<0>(k);   // every finished sample is counted (pending ones are not yet)
            if (k >= spp) st = ST_DONE;
            rng.c = cc + off;
            rng.reload(ring);   // first read after the next visit's trace
            tick(6);
        }
        // drain: the shadow rays still in flight and the samples waiting behind them, so no NEE
        // state crosses launches
        if (__ballot(shm || fin)) {
            unsigned long long best = ~0ull;
            trace_resolve(false, best);
        }
        // counters of the quad's lanes
        nseg += dpp32<0xB1>(nseg), nseg += dpp32<0x4E>(nseg);
        nsh += dpp32<0xB1>(nsh), nsh += dpp32<0x4E>(nsh);
        bool want_req = false;
        if (live && lead) {
            px[0] = acc.x, px[1] = acc.y, px[2] = acc.z;
            want_req = !(st & ST_DONE) && g - cc < P.rng_keep;
            const uint32_t st_out = (st & ST_DONE) ? ST_DONE : (has ? 0u : ST_REGEN);
            P.state[s] = st_out;
            if (!st_out) {
                P.depth[s] = depth;
                P.thr[s] = pk(thr);
                P.rad[s] = pk(rad);
                P.ray_o[s] = pk(o);
                P.ray_d[s] = pk(d);
            }
            P.sample_k[s] = k;
            P.rng_c[s] = cc;
            if (nseg) P.c_seg[s] += nseg;
            if (nsh) P.c_shadow[s] += nsh;
            if (nrej) P.c_rej[s] += nrej;
        }
        wave_append(live && lead && !(st & ST_DONE), s, out + it.p * P.part_cap, out_count + it.p, lane);
        wave_refill(P, want_req, s, g, lane, scratch);
        tick(7);
    }
    if constexpr (XRT_PHASE_CLOCK) {
        if (lane == 0)
            for (int q = 0; q < 8; ++q) atomicAdd(P.stats + kStatsPhase + q, ph[q]);
    }
}

// ------------------------------------------------------------------- host side ----
// GIIntegrator with one area light and maxDepth >= 2 over a merged-schedule triangle scene of
// at most 64 triangles (the camera lists' masks; the group traces' masks need the same)
bool use_step_spec(const KParams& P) {
    return P.scene_kind == SCN_TRI && P.integrator == XRT_INTEGRATOR_GI && P.n_lights == 1 && P.max_depth >= 2 &&
           P.n_tris <= 64 && !(P.rflags & XRT_FLAG_NO_GROUP) && use_step_merged(P);
}

hipError_t launch_camlist(const KParams& P, hipStream_t st) {
    hipLaunchKernelGGL(k_camlist, dim3((P.n_slots + kBlock - 1) / kBlock), dim3(kBlock), 0, st, P);
    return hipGetLastError();
}

hipError_t launch_step_spec(const KParams& P, const KParams* dP, const uint32_t* list, const uint32_t* count,
                            uint32_t* out, uint32_t* out_count, uint32_t* zero, uint32_t visits, uint32_t part_live,
                            uint32_t spw, hipStream_t st) {
    const uint32_t per_block = (kBlock / 64) * spw;
    const uint32_t blocks = P.n_part * ((std::min(part_live, P.part_cap) + per_block - 1) / per_block);
    const size_t lds = step_merged_lds_bytes(P);
    if (spw == 16)
        hipLaunchKernelGGL((k_step_spec<16, 4>), dim3(blocks), dim3(kBlock), lds, st, dP, list, count, out, out_count,
                           zero, visits);
    else if (spw == 8)
        hipLaunchKernelGGL((k_step_spec<8, 8>), dim3(blocks), dim3(kBlock), lds, st, dP, list, count, out, out_count,
                           zero, visits);
    else if (spw == 4)
        hipLaunchKernelGGL((k_step_spec<4, 16>), dim3(blocks), dim3(kBlock), lds, st, dP, list, count, out, out_count,
                           zero, visits);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace xrt
