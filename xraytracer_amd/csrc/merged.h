// merged.h — helpers shared by the merged-trace kernels (step_tri.hip: k_step_merged,
// k_trace_2a_coop; spec.hip: k_step_spec): global-address-space loads, the exact plane cull,
// the branch-free Moller-Trumbore test and the group trace (G lanes per slot split a slot's
// candidate triangles).  Device code only.
#pragma once
#include "path_common.h"

namespace xrt {

using gu32 = __attribute__((address_space(1))) const uint32_t;
using gf32 = __attribute__((address_space(1))) const float;
// one float4 by a global (not flat) load
__device__ __forceinline__ f4 ldg4(const f4* p, size_t i) {
    typedef float fv4 __attribute__((ext_vector_type(4)));
    using gv4 = __attribute__((address_space(1))) const fv4;
    const fv4 v = ((gv4*)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
// global-address-space view of a generic pointer to device memory: global_load instead of
// flat_load (a flat load also counts in lgkmcnt, so every LDS wait would wait for it too)
template <class G, class T>
__device__ __forceinline__ G* glb(T* p) {
    return (G*)(p);
}
__device__ __forceinline__ v3 ld3g(const f4* p, size_t i) {
    gf32* q = glb<gf32>(p) + 4 * i;
    return mk(q[0], q[1], q[2]);
}

constexpr float kRcp3 = 1.0f / 3.0f;                         // RN(1/3) for div_const
constexpr float kLambertPdf = 1.0f / (2.0f * kPI);            // Lambert sampleBxDF pdf
constexpr float kLambertPdfRcp = 1.0f / kLambertPdf;          // RN(1/pdf)

// Stream words of one slot held in registers: b[0] is the next draw.  A segment draws at
// most NW words (checked before it starts), so there is no fallback load.
// The words of the next segment are prefetched into pf[] at the end of a segment and moved
// into b[] only after the next trace (take), so the loads' latency hides behind the trace:
// the move is the loads' first use, and nothing else in the loop reads pf[].
template <int NW>
struct RngRegs {
    uint32_t b[NW];
    uint32_t pf[NW];
    uint32_t c;
    __device__ __forceinline__ void load(const uint32_t* ring) {
        gu32* r = glb<gu32>(ring);
        uint32_t i = c % kRing;
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            b[j] = r[i];
            i = (i + 1 == kRing) ? 0u : i + 1;
        }
    }
    // NW consecutive words in ceil(NW / 4) vector loads (dword-aligned dwordx4 / dwordx2:
    // a quarter of the address work of NW dword loads); a lane whose window wraps past the
    // ring's end takes dword loads
    __device__ __forceinline__ void prefetch(const uint32_t* ring) {
        typedef uint32_t u4u __attribute__((ext_vector_type(4), aligned(4)));
        typedef uint32_t u2u __attribute__((ext_vector_type(2), aligned(4)));
        using gu4 = __attribute__((address_space(1))) const u4u;
        using gu2 = __attribute__((address_space(1))) const u2u;
        static_assert(NW % 2 == 0, "even window");
        const uint32_t i = c % kRing;
        if (i <= kRing - NW) {
#pragma unroll
            for (int j = 0; j + 4 <= NW; j += 4) {
                const u4u v = *(gu4*)(ring + i + j);
                pf[j] = v.x, pf[j + 1] = v.y, pf[j + 2] = v.z, pf[j + 3] = v.w;
            }
            if constexpr (NW % 4 == 2) {
                const u2u v = *(gu2*)(ring + i + NW - 2);
                pf[NW - 2] = v.x, pf[NW - 1] = v.y;
            }
        } else {
            gu32* r = glb<gu32>(ring);
            uint32_t k = i;
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                pf[j] = r[k];
                k = (k + 1 == kRing) ? 0u : k + 1;
            }
        }
    }
    // the same loads straight into b[] (for a kernel that reads no word between the end of one
    // visit and the trace of the next: the loads still land behind that trace)
    __device__ __forceinline__ void reload(const uint32_t* ring) {
        prefetch(ring);
        take();
    }
    __device__ __forceinline__ void take() {
#pragma unroll
        for (int j = 0; j < NW; ++j) b[j] = pf[j];
    }
    __device__ __forceinline__ float next() {
        const uint32_t y = b[0];
#pragma unroll
        for (int j = 0; j + 1 < NW; ++j) b[j] = b[j + 1];
        ++c;
        return canonical(mt_temper(y));
    }
};

// A float that is +0, -0 or NaN as a 2-bit code (0, 1, 2) and back (NaN: the canonical
// quiet NaN — a NaN contribution makes its sample's radiance NaN, which Image::addPixel's
// reject drops, so the payload never reaches the image)
__device__ __forceinline__ uint32_t zcode(float x) { return x != x ? 2u : (__float_as_uint(x) >> 31); }
__device__ __forceinline__ float zdecode(uint32_t c) {
    return __uint_as_float(c == 2u ? 0x7fc00000u : (c << 31));
}

__device__ __forceinline__ uint32_t lanemask_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Conservative overlap of the ray segment [0, tlim] with the object's culling box.  oi = o *
// inv, once per ray: each slab distance is one fma, b * inv - oi, whose error (~2^-24 |o|
// along the axis, whatever inv) is far inside the box margin.  inv is rcp3c(d): clamped to
// +-1e30, so no inf enters (an fma of two infinities would be a NaN, and fminf / fmaxf
// would then keep the wrong slab end); an axis-parallel ray then gets slab distances of
// magnitude >= 1e30 * |b - o|, beyond any ray length, or the right sign within 2^-24 |o|
// of a slab plane — a margin away from the geometry.
__device__ __forceinline__ bool obj_overlap(v3 oi, v3 inv, const StepObj& B, float tlim) {
    const float tx0 = __builtin_fmaf(B.bmin[0], inv.x, -oi.x), tx1 = __builtin_fmaf(B.bmax[0], inv.x, -oi.x);
    const float ty0 = __builtin_fmaf(B.bmin[1], inv.y, -oi.y), ty1 = __builtin_fmaf(B.bmax[1], inv.y, -oi.y);
    const float tz0 = __builtin_fmaf(B.bmin[2], inv.z, -oi.z), tz1 = __builtin_fmaf(B.bmax[2], inv.z, -oi.z);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
    return !(tn > tf);
}
__device__ __forceinline__ bool box_overlap_f(v3 oi, v3 inv, const DObjBox& B, float tlim) {
    const float tx0 = __builtin_fmaf(B.bmin[0], inv.x, -oi.x), tx1 = __builtin_fmaf(B.bmax[0], inv.x, -oi.x);
    const float ty0 = __builtin_fmaf(B.bmin[1], inv.y, -oi.y), ty1 = __builtin_fmaf(B.bmax[1], inv.y, -oi.y);
    const float tz0 = __builtin_fmaf(B.bmin[2], inv.z, -oi.z), tz1 = __builtin_fmaf(B.bmax[2], inv.z, -oi.z);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
    return !(tn > tf);
}

// Exact plane cull.  Every vertex of the object has coordinate c on axis a (DObjPlane), so
// e1_a = e2_a = 0 exactly and, in Mesh::rayTriangleIntersect's float evaluation, every term
// of det = e1 . (d x e2) and of t's numerator e2 . ((o - v0) x e1) that involves e1_a or e2_a
// is an exact +-0: det is d_a (A - B) and the numerator -(o_a - c) (A - B), up to roundings
// that cannot flip the sign of A - B (plane_tri_ok, host).  So whenever (o_a - c) * d_a >= 0
// the test rejects every triangle of the object: t = num / det <= 0, or d_a = 0 gives
// |det| < eps, or o_a = c gives t = +-0.  (Where |d_a| < 1e-20 or |o_a - c| < 1e-25 a
// product may leave the normal range, but then |det| < eps resp. |t| < eps for the edge
// lengths plane_tri_ok admits, so the test rejects anyway.)  NaNs are not culled.
__device__ __forceinline__ bool plane_away(v3 o, v3 d, int axis, float c) {
    const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
    const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
    return axis >= 0 && (oa - c) * da >= 0.0f;
}

// Mesh::rayTriangleIntersect (Src/primitive.cpp:140-168) without branches: the same float
// operations, and the same accept/reject decisions (NaN comparisons included).  invDet is
// the Newton reciprocal without the IEEE fallback: only scenes with det_bounded (xrt_api.cpp:
// |det| < 2^120) reach this test, where a finite det is either < kEPSILON — rejected, so
// invDet does not matter — or inside rcp_newton's exhaustively checked exact range, and a
// NaN det gives NaN both ways.
__device__ __forceinline__ bool ray_tri_nb(v3 o, v3 d, v3 v0, v3 e1, v3 e2, float& t) {
    const v3 pvec = cross(d, e2);
    const float det = dot(e1, pvec);
    const float invDet = rcp_newton(det);   // == 1.0f / det wherever it matters
    const v3 tvec = o - v0;
    const float u = dot(tvec, pvec) * invDet;
    const v3 qvec = cross(tvec, e1);
    const float v = dot(d, qvec) * invDet;
    t = dot(e2, qvec) * invDet;
    const bool rej = (__builtin_fabsf(det) < kEPSILON) | (u < 0.0f) | (u > 1.0f) | (v < 0.0f) | (u + v > 1.0f);
    return !rej & (t > kEPSILON);
}

// Group trace (G = 2, 4 or 16 lanes per slot, scenes of <= 64 triangles): the G lanes of a
// slot hold identical path state (every shading instruction runs on all of them) and split
// its traces among themselves, with no LDS traffic but the triangle fetches: lane u culls
// objects u, u+G, ... into 64-bit triangle masks (one per ray), the masks are OR-ed across
// the group by DPP, lane u tests the candidate triangles k = u (mod G) in increasing k, and
// the group reduces by DPP: min of (t bits << 32 | k) for the extension ray — smallest t,
// then lowest index, the reference's in-order `t < best` scan — and OR of occlusion bits.
// LAZY: form each ray's o * inv per object test instead of keeping it (fewer live registers)
template <int NL, int G, bool LAZY = false>
__device__ __forceinline__ void group_trace(int n_objs, const LScene& L, const DObjPlane* pl, int lane, bool ext, v3 o, v3 d,
                                            uint32_t shm, const v3 (&so)[NL + 1], const v3 (&sd)[NL + 1],
                                            const float (&stm)[NL + 1], unsigned long long& best, uint32_t& occ) {
    constexpr int R = 1 + NL;
    const int u = lane & (G - 1);
    uint64_t tm[R];
    v3 inv[R], oi[R];
#pragma unroll
    for (int q = 0; q < R; ++q) tm[q] = 0ull;
    inv[0] = rcp3c(d);
    if (!LAZY) oi[0] = o * inv[0];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        inv[1 + l] = rcp3c(sd[l]);
        if (!LAZY) oi[1 + l] = so[l] * inv[1 + l];
    }
    for (int ob0 = 0; ob0 < n_objs; ob0 += G) {
        const int ob = ob0 + u;
        if (ob < n_objs) {
            const DObjBox B = L.box[ob];
            const DObjPlane pb = pl[ob];
            const uint32_t cnt = (uint32_t)(B.count_occ & 0x7fffffff);
            const uint64_t bits = (cnt >= 64u ? ~0ull : ((1ull << cnt) - 1ull)) << B.first;
            if (ext && !plane_away(o, d, pb.axis, pb.c) && box_overlap_f(LAZY ? o * inv[0] : oi[0], inv[0], B, kINF))
                tm[0] |= bits;
#pragma unroll
            for (int l = 0; l < NL; ++l)
                if (B.count_occ < 0 && ((shm >> l) & 1u) && !plane_away(so[l], sd[l], pb.axis, pb.c) &&
                    box_overlap_f(LAZY ? so[l] * inv[1 + l] : oi[1 + l], inv[1 + l], B, stm[l]))
                    tm[1 + l] |= bits;
        }
    }
    const uint64_t pat = (G == 16  ? 0x0001000100010001ull
                          : G == 8 ? 0x0101010101010101ull
                          : G == 4 ? 0x1111111111111111ull
                          : G == 2 ? 0x5555555555555555ull
                                   : ~0ull)
                         << u;
    // Candidates two at a time: both triangles' LDS loads are issued before either test, so
    // a lane pays one LDS latency per pair of candidates (with few waves per SIMD — the tail of
    // a shard — the loop is bound by that latency, not by issue).  An odd last candidate is
    // tested twice (same key: harmless for the min and the or).
    unsigned long long bk = ~0ull;
    for (uint64_t bits = group_or64<G>(tm[0]) & pat; bits;) {
        const uint32_t k0 = (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1ull;
        const uint32_t k1 = bits ? (uint32_t)__builtin_ctzll(bits) : k0;
        bits &= bits - 1ull;
        const f4 a0 = L.tri[3 * k0], b0 = L.tri[3 * k0 + 1], c0 = L.tri[3 * k0 + 2];
        const f4 a1 = L.tri[3 * k1], b1 = L.tri[3 * k1 + 1], c1 = L.tri[3 * k1 + 2];
        float t0, t1;
        const bool h0 = ray_tri_nb(o, d, xyz(a0), xyz(b0), xyz(c0), t0);
        const bool h1 = ray_tri_nb(o, d, xyz(a1), xyz(b1), xyz(c1), t1);
        const unsigned long long key0 = h0 ? ((unsigned long long)__float_as_uint(t0) << 32) | k0 : ~0ull;
        const unsigned long long key1 = h1 ? ((unsigned long long)__float_as_uint(t1) << 32) | k1 : ~0ull;
        const unsigned long long key = key0 < key1 ? key0 : key1;
        bk = key < bk ? key : bk;
    }
    uint32_t oc = 0;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        for (uint64_t bits = group_or64<G>(tm[1 + l]) & pat; bits;) {
            const uint32_t k0 = (uint32_t)__builtin_ctzll(bits);
            bits &= bits - 1ull;
            const uint32_t k1 = bits ? (uint32_t)__builtin_ctzll(bits) : k0;
            bits &= bits - 1ull;
            const f4 a0 = L.tri[3 * k0], b0 = L.tri[3 * k0 + 1], c0 = L.tri[3 * k0 + 2];
            const f4 a1 = L.tri[3 * k1], b1 = L.tri[3 * k1 + 1], c1 = L.tri[3 * k1 + 2];
            float t0, t1;
            const bool h0 = ray_tri_nb(so[l], sd[l], xyz(a0), xyz(b0), xyz(c0), t0) && t0 < stm[l];
            const bool h1 = ray_tri_nb(so[l], sd[l], xyz(a1), xyz(b1), xyz(c1), t1) && t1 < stm[l];
            if (h0 || h1) {
                oc |= 1u << l;
                bits = 0ull;   // occluded: the rest need no test
            }
        }
    }
    best = group_min64<G>(bk);
    occ = group_or32<G>(oc);
}

// Scene::intersect for a camera ray of the pixel whose camera list (k_camlist, spec.hip) is
// cl = {mask bits 0-31, 32-63, covering triangle or -1, 0}: the (t bits << 32 | triangle)
// minimum over the listed triangles — every triangle a camera ray of the pixel can hit, less
// those hidden behind a covering one — or, when one triangle covers the pixel alone, that
// triangle (every camera ray of the pixel hits it first; the caller recomputes t, u, v).
__device__ __forceinline__ unsigned long long camlist_closest(const LScene& L, uint4 cl, v3 o, v3 d) {
    if ((int)cl.z >= 0) return (unsigned long long)cl.z;
    unsigned long long best = ~0ull;
    for (uint64_t bits = (uint64_t)cl.x | ((uint64_t)cl.y << 32); bits; bits &= bits - 1ull) {
        const uint32_t k = (uint32_t)__builtin_ctzll(bits);
        float t;
        if (ray_tri_nb(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t)) {
            const unsigned long long key = ((unsigned long long)__float_as_uint(t) << 32) | k;
            best = key < best ? key : best;
        }
    }
    return best;
}

// LDS of k_step_merged: the scene (step_layout), the per-object planes (group traces), then
// one MergedWave of trace scratch per wave
__host__ __device__ inline uint32_t merged_plane_off(const StepLayout& Lo) { return (Lo.total + 15u) & ~15u; }
__host__ __device__ inline uint32_t merged_wave_off(const KParams& P, const StepLayout& Lo) {
    return merged_plane_off(Lo) + ((8u * (uint32_t)P.n_objs + 15u) & ~15u);
}

template <int NL>
struct MergedWave {
    static constexpr int R = 1 + NL;   // rays per lane: extension + one shadow ray per light
    f4 ro[R * 64];                     // the current object's rays, ranked: origin, w = tmax
    f4 rd[R * 64];                     // direction, w = ray id q * 64 + lane (bits)
    unsigned long long best[64];       // closest hit of the extension ray: (t bits << 32) | tri
    uint32_t occ[64];                  // bit l: shadow ray l is occluded
};

}  // namespace xrt
