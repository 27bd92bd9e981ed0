// path_common.h — device building blocks shared by the path-tracing kernels
// (wavefront.hip: wavefront + fused schedules; step_tri.hip: merged-trace triangle
// schedule): the mt19937 stream restatement, wave utilities, ray/primitive tests, light and
// BSDF sampling, the camera, and the LDS scene carve of the fused schedules.
#pragma once
#include <hip/hip_runtime.h>

#include "device_math.h"
#include "wavefront.h"
#include "xrt.h"

namespace xrt {

constexpr int kBlock = 256;
constexpr int kTriTile = 512;    // triangles per LDS tile (24 KiB)
constexpr int kSphTile = 1024;   // spheres per LDS tile (16 KiB + 4 KiB)

// ============================================================================ RNG ====
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
// generate_canonical<float,24>: (float)x / 2^32, nextafter(1,0) if it rounds to 1
__device__ __forceinline__ float canonical(uint32_t y) {
    const float f = (float)y * 0x1p-32f;
    return f >= 1.0f ? 0x1.fffffep-1f : f;
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// A slot's stream: ring words x[c], x[c+1], ...  prefetch() issues the loads of the next 8
// words at once (one memory latency for a whole shade pass instead of one per draw); a
// draw past them loads the next 8 again (long delta-tracking walks: one latency per 8
// draws, not per draw).  Words at or past the slot's generated end g may be loaded but are
// never drawn: every caller checks g - c before drawing, exactly as for single loads.
// Global (not flat) loads, so LDS waits do not also wait for them.
struct Rng {
    const uint32_t* ring;
    uint32_t c;
    uint32_t nb = 0;
    uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0, b4 = 0, b5 = 0, b6 = 0, b7 = 0;
    __device__ __forceinline__ void load8() {   // two dword-aligned dwordx4 unless the window wraps
        typedef uint32_t u4u __attribute__((ext_vector_type(4), aligned(4)));
        using g4 = __attribute__((address_space(1))) const u4u;
        using g32 = __attribute__((address_space(1))) const uint32_t;
        const uint32_t i = c % kRing;
        if (i <= kRing - 8) {
            const u4u lo = *(g4*)(ring + i), hi = *(g4*)(ring + i + 4);
            b0 = lo.x, b1 = lo.y, b2 = lo.z, b3 = lo.w, b4 = hi.x, b5 = hi.y, b6 = hi.z, b7 = hi.w;
        } else {
            g32* r = (g32*)ring;
            b0 = r[i], b1 = r[(i + 1) % kRing], b2 = r[(i + 2) % kRing], b3 = r[(i + 3) % kRing];
            b4 = r[(i + 4) % kRing], b5 = r[(i + 5) % kRing], b6 = r[(i + 6) % kRing], b7 = r[(i + 7) % kRing];
        }
    }
    __device__ __forceinline__ void prefetch(uint32_t avail) {
        nb = avail < 8u ? avail : 8u;
        load8();
    }
    __device__ __forceinline__ float next() {
        if (!nb) {
            load8();
            nb = 8;
        }
        const uint32_t y = b0;
        b0 = b1, b1 = b2, b2 = b3, b3 = b4, b4 = b5, b5 = b6, b6 = b7;
        --nb;
        ++c;
        return canonical(mt_temper(y));
    }
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One mt19937 twist of a slot's stream done by a whole wave: x[g+k] = x[g+k-227] ^
// mix(x[g+k-624], x[g+k-623]) for k = 0..623 (libstdc++ _M_gen_rand).  Split into the
// chunks k = m, 227 + m, 454 + m (m = lane + 64 j), the word each chunk needs from the
// previous one, x[g+k-227], is the same lane's register — no LDS, no barrier.  The new
// block lands in ring half g % 1248, over the oldest (fully consumed) block.  Must be
// called by every lane of the wave.
__device__ inline void wave_twist(uint32_t* ring, uint32_t g, int lane) {
    const uint32_t h = g % kRing;
    const uint32_t* old = ring + (kMT - h);
    uint32_t* nw = ring + h;
    uint32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t m = lane + 64 * j;
        if (m < 227) a[j] = old[m + 397] ^ mt_mix(old[m], old[m + 1]);
    }
    const uint32_t n0 = __shfl(a[0], 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t m = lane + 64 * j;
        if (m < 227) b[j] = a[j] ^ mt_mix(old[227 + m], old[228 + m]);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint32_t m = lane + 64 * j;
        if (m < 170) nw[454 + m] = b[j] ^ mt_mix(old[454 + m], m + 455 < kMT ? old[455 + m] : n0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t m = lane + 64 * j;
        if (m < 227) nw[m] = a[j], nw[227 + m] = b[j];
    }
}

// In-line refill from global memory (no LDS buffer): every lane with `need` gets its slot's
// next block, twisted by the whole wave (wave_twist).  Used by the RNG self-test and by
// k_step on sphere-BVH scenes (XRT_KSTEP_LDS_REFILL = 2, whose LDS holds the BVH).
// Invariants: a slot asks only when fewer than rng_keep <= kMT words are left, so the new
// block x[g, g + 624) overwrites only words the slot has drawn (the other ring half), and
// reads only the old half, which no lane writes; the workgroup fence orders the stores before
// the launch ends, and the next reader of the ring is a later kernel launch.
// Must be called by every lane of the wave (wave-uniform control flow).
__device__ inline void wave_refill(bool need, uint32_t slot, uint32_t& g, uint32_t* rings, int lane) {
    uint64_t m = __ballot(need);
    if (m == 0) return;
    while (m) {
        const int L = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint32_t sl = __shfl(slot, L);
        const uint32_t gl = __shfl(g, L);
        wave_twist(rings + (size_t)sl * kRing, gl, lane);
    }
    if (need) g += kMT;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// One twist of a slot's ring by a whole wave, staged through LDS: the old block (624 words,
// 16-byte aligned because kRing*4 and kMT*4 are multiples of 16) comes in as 156 dwordx4
// loads (3 instructions per wave) and every recurrence operand is then an LDS read, instead
// of 26 overlapping global_load_dword per lane whose 64-lane requests re-fetch each cache
// line ~2.6 times through the TA.  The new words go out as 11 coalesced dword stores.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct Staged { u32x4 v[3]; };

__device__ __forceinline__ Staged load_block(const uint32_t* ring, uint32_t g, int lane) {
    const u32x4* old = reinterpret_cast<const u32x4*>(ring + (kMT - g % kRing));
    Staged r;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        r.v[k] = __builtin_nontemporal_load(old + min((uint32_t)lane + 64u * k, (uint32_t)(kMT / 4 - 1)));
    return r;
}

__device__ __forceinline__ void store_block(const Staged& r, int lane, uint32_t* lds) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t q = (uint32_t)lane + 64u * k;
        if (q < kMT / 4) reinterpret_cast<u32x4*>(lds)[q] = r.v[k];
    }
    wave_sync();
}

// The new block goes back out through the same LDS buffer (its old words are all in
// registers by then) as 156 dwordx4 stores: whole 64-byte runs instead of 11 dword stores
// per lane that start at arbitrary offsets within a cache line.
__device__ __forceinline__ void twist_block(uint32_t* ring, uint32_t g, int lane, uint32_t* buf) {
    const uint32_t* old = buf;
    uint32_t x0[4], x1[4], x397[4], y0[4], y1[4], z0[3], z1[3];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t m = min((uint32_t)lane + 64u * j, 226u);
        x0[j] = old[m], x1[j] = old[m + 1], x397[j] = old[m + 397];
        y0[j] = old[227 + m], y1[j] = old[228 + m];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint32_t m = min((uint32_t)lane + 64u * j, 169u);
        z0[j] = old[454 + m], z1[j] = old[min(455 + m, kMT - 1)];
    }
    uint32_t a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = x397[j] ^ mt_mix(x0[j], x1[j]);
    const uint32_t n0 = __builtin_amdgcn_readfirstlane(a[0]);   // x[g]: the new block's first word
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = a[j] ^ mt_mix(y0[j], y1[j]);
    wave_sync();   // every old word is in registers before the buffer is overwritten
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint32_t m = (uint32_t)lane + 64u * j;
        if (m < 170u) buf[454 + m] = b[j] ^ mt_mix(z0[j], m + 455 < kMT ? z1[j] : n0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t m = (uint32_t)lane + 64u * j;
        if (m < 227u) buf[m] = a[j], buf[227 + m] = b[j];
    }
    wave_sync();
    u32x4* nw = reinterpret_cast<u32x4*>(ring + g % kRing);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t q = (uint32_t)lane + 64u * k;
        if (q < kMT / 4) nw[q] = reinterpret_cast<const u32x4*>(buf)[q];
    }
}

// Inline refill (the merged schedule): at the end of a step launch each wave twists the
// rings of its own slots that are running low, one slot at a time through `buf` (the
// wave's trace scratch, idle by then), the next slot's old block loading into registers
// while the current one twists — instead of queueing them for a separate k_refill_merged
// launch after every step launch (6 ms of an 80 ms C2 frame, serialised).  Safe for the
// unconsumed words: a slot asks when fewer than rng_keep (<= 624) words are left, so the
// new block x[g, g + 624) overwrites only words the slot has already drawn.
__device__ __forceinline__ void wave_refill(const KParams& P, bool want, uint32_t s, uint32_t g, int lane,
                                            uint32_t* buf) {
    uint64_t rq = __ballot(want);
    if (!rq) return;
    int l = __builtin_ctzll(rq);
    rq &= rq - 1ull;
    uint32_t sc = (uint32_t)__builtin_amdgcn_readlane((int)s, l), gc = (uint32_t)__builtin_amdgcn_readlane((int)g, l);
    Staged blk = load_block(P.ring + (size_t)sc * kRing, gc, lane);
    for (;;) {
        store_block(blk, lane, buf);
        const bool more = rq != 0ull;
        uint32_t sn = sc, gn = gc;
        if (more) {
            l = __builtin_ctzll(rq);
            rq &= rq - 1ull;
            sn = (uint32_t)__builtin_amdgcn_readlane((int)s, l), gn = (uint32_t)__builtin_amdgcn_readlane((int)g, l);
            blk = load_block(P.ring + (size_t)sn * kRing, gn, lane);
        }
        twist_block(P.ring + (size_t)sc * kRing, gc, lane, buf);
        if (lane == 0) P.rng_g[sc] = gc + kMT;
        if (!more) break;
        wave_sync();
        sc = sn, gc = gn;
    }
}

// Cross-lane reductions within groups of G = 2, 4, 8 or 16 adjacent lanes by DPP (no LDS):
// quad_perm swaps for 2 and 4, row_half_mirror / row_mirror for 8 and 16.  Every lane of
// a group must be active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
template <int G>
__device__ __forceinline__ uint32_t group_or32(uint32_t x) {
    if (G >= 2) x |= dpp32<0xB1>(x);    // quad_perm(1, 0, 3, 2): partner lane ^ 1
    if (G >= 4) x |= dpp32<0x4E>(x);    // quad_perm(2, 3, 0, 1): partner lane ^ 2
    if (G >= 8) x |= dpp32<0x141>(x);   // row_half_mirror: lane 7 - i of its 8 (quads 0 and 1)
    if (G >= 16) x |= dpp32<0x140>(x);  // row_mirror: lane 15 - i of its 16 (halves 0 and 1)
    return x;
}
template <int G>
__device__ __forceinline__ uint64_t group_or64(uint64_t x) {
    return ((uint64_t)group_or32<G>((uint32_t)(x >> 32)) << 32) | group_or32<G>((uint32_t)x);
}
template <int CTRL>
__device__ __forceinline__ uint64_t min64_dpp(uint64_t x) {
    const uint64_t y = ((uint64_t)dpp32<CTRL>((uint32_t)(x >> 32)) << 32) | dpp32<CTRL>((uint32_t)x);
    return y < x ? y : x;
}
template <int G>
__device__ __forceinline__ uint32_t group_min32(uint32_t x) {
    if (G >= 2) x = min(x, dpp32<0xB1>(x));
    if (G >= 4) x = min(x, dpp32<0x4E>(x));
    if (G >= 8) x = min(x, dpp32<0x141>(x));
    if (G >= 16) x = min(x, dpp32<0x140>(x));
    return x;
}
template <int G>
__device__ __forceinline__ uint64_t group_min64(uint64_t x) {
    if (G >= 2) x = min64_dpp<0xB1>(x);
    if (G >= 4) x = min64_dpp<0x4E>(x);
    if (G >= 8) x = min64_dpp<0x141>(x);
    if (G >= 16) x = min64_dpp<0x140>(x);
    return x;
}

// Append v to list (count at cnt) for every lane with want set: one atomic per wave.
// Must be called by every lane of the wave (wave-uniform control flow).
__device__ __forceinline__ void wave_append(bool want, uint32_t v, uint32_t* list, uint32_t* cnt, int lane) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (want) list[base + __popcll(m & ((1ull << lane) - 1ull))] = v;
}

// Live and refill lists are partitioned: partition p owns the slots
// [p*part_cap, (p+1)*part_cap) and its entries list[p*part_cap + i], i < count[p]; block b
// serves partition b % n_part (grids are n_part * chunks blocks).  Appends then contend
// on n_part counters instead of one, and a partition's slots are always touched by the
// same XCD (blocks are dealt to the 8 XCDs round-robin and n_part is a multiple of 8).
struct PartIter {
    uint32_t p, first, stride, n;
};
__device__ __forceinline__ PartIter part_iter(const KParams& P, const uint32_t* count, uint32_t per_block) {
    PartIter it;
    it.p = blockIdx.x % P.n_part;
    const uint32_t chunk = blockIdx.x / P.n_part, nchunks = gridDim.x / P.n_part;
    it.first = chunk * per_block;
    it.stride = nchunks * per_block;
    it.n = count[it.p];
    return it;
}
__device__ __forceinline__ void zero_parts(const KParams& P, uint32_t* c) {
    if (blockIdx.x == 0)
        for (uint32_t i = threadIdx.x; i < P.n_part; i += kBlock) c[i] = 0;
}


// ====================================================================== geometry ====
// Mesh::rayTriangleIntersect, no CULLING (Src/primitive.cpp:140-168), with e1 = v1 - v0,
// e2 = v2 - v0 precomputed on the host by the same subtraction.
__device__ __forceinline__ bool ray_tri(v3 o, v3 d, v3 v0, v3 e1, v3 e2, float& t, float& u, float& v) {
    const v3 pvec = cross(d, e2);
    const float det = dot(e1, pvec);
    if (__builtin_fabsf(det) < kEPSILON) return false;
    const float invDet = rcp_rn(det);   // == 1.0f / det
    const v3 tvec = o - v0;
    u = dot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return false;
    const v3 qvec = cross(tvec, e1);
    v = dot(d, qvec) * invDet;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = dot(e2, qvec) * invDet;
    return t > kEPSILON;
}

// Sphere::doIntersect + solveQuadratic (Src/primitive.h:133-177): double -0.5*(b±sqrt).
// Past the discriminant test (a wave whose rays all miss skips the rest) the lanes compute
// the general root pair and select, so rays with different outcomes run one instruction
// stream (the branchy form spent about as many scalar exec-mask instructions as vector ones).
// Same values as the reference's branches:
//  * discr < 0: no hit (a NaN discriminant passes on, as in the reference, and yields NaN
//    roots, which every caller's `t < best` rejects);
//  * discr == 0: t0 = t1 = -0.5 * b / a in double — rare, so it keeps its own branch;
//  * q = -0.5 * (b ± sqrt): b - sq is b + (-sq) exactly;
//  * the swap and the t0 < 0 fallback as selects.
__device__ __forceinline__ bool sphere_hit(v3 o, v3 d, v3 c, float r, float& tnear) {
    const v3 L = o - c;
    const float a = dot(d, d);
    const float b = 2.0f * dot(d, L);
    const float cc = dot(L, L) - r * r;
    const float discr = b * b - 4.0f * a * cc;
    if (discr < 0.0f) return false;
    const double sq = __builtin_sqrt((double)discr);
    const float q = (float)(-0.5 * ((double)b + (b > 0.0f ? sq : -sq)));
    float t0 = q / a;
    float t1 = cc / q;
    if (discr == 0.0f) t0 = t1 = (float)(-0.5 * (double)b / (double)a);
    const bool sw = t0 > t1;
    const float lo = sw ? t1 : t0, hi = sw ? t0 : t1;
    tnear = lo < 0.0f ? hi : lo;
    return !(lo < 0.0f && hi < 0.0f);
}

// BoxMesh::intersect slab test (Src/primitive.h:243-264)
__device__ __forceinline__ bool box_hit(v3 o, v3 d, v3 pmin, v3 pmax, float& t0, float& t1) {
    const v3 di = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const v3 tt = di * (pmax - o), tb = di * (pmin - o);
    const v3 tmin = mk(smin(tt.x, tb.x), smin(tt.y, tb.y), smin(tt.z, tb.z));
    const v3 tmax = mk(smax(tt.x, tb.x), smax(tt.y, tb.y), smax(tt.z, tb.z));
    t0 = smax(smax(tmin.x, tmin.y), tmin.z);
    t1 = smin(smin(tmax.x, tmax.y), tmax.z);
    if (t0 > t1 || t1 <= 0.0f) return false;
    t0 = smax(t0, 0.0f);
    return true;
}


// Conservative ray/AABB overlap on [0, tlim] for culling (approximate reciprocal is fine:
// the boxes carry a margin; fminf/fmaxf drop the NaNs of 0*inf, which only widens the
// interval).
__device__ __forceinline__ bool box_overlap(v3 o, v3 inv, const DObjBox& B, float tlim) {
    const float tx0 = (B.bmin[0] - o.x) * inv.x, tx1 = (B.bmax[0] - o.x) * inv.x;
    const float ty0 = (B.bmin[1] - o.y) * inv.y, ty1 = (B.bmax[1] - o.y) * inv.y;
    const float tz0 = (B.bmin[2] - o.z) * inv.z, tz1 = (B.bmax[2] - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
    return !(tn > tf);
}
// entry distance of the ray segment [0, tlim] into a padded node box, +inf if it misses
__device__ __forceinline__ float bvh_enter(const f4& mn, const f4& mx, v3 o, v3 inv, float tlim) {
    const float tx0 = (mn.x - o.x) * inv.x, tx1 = (mx.x - o.x) * inv.x;
    const float ty0 = (mn.y - o.y) * inv.y, ty1 = (mx.y - o.y) * inv.y;
    const float tz0 = (mn.z - o.z) * inv.z, tz1 = (mx.z - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
    return tn > tf ? __builtin_inff() : tn;
}

// does the ray segment [0, tlim] overlap either child box of a BVH node (n0..n3, bvh.h)?
__device__ __forceinline__ bool root_overlap(const f4& n0, const f4& n1, const f4& n2, const f4& n3, v3 o, v3 inv,
                                             float tlim) {
    const bool l = __float_as_int(n1.w) >= 0 && bvh_enter(n0, n1, o, inv, tlim) != __builtin_inff();
    const bool r = __float_as_int(n3.w) >= 0 && bvh_enter(n2, n3, o, inv, tlim) != __builtin_inff();
    return l || r;
}

// rcp3 clamped to +-1e30 (the fma-form culling slabs, step_tri.hip obj_overlap)
__device__ __forceinline__ float rcpc(float x) {
    return __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(x), -1e30f, 1e30f);
}
__device__ __forceinline__ v3 rcp3c(v3 d) { return mk(rcpc(d.x), rcpc(d.y), rcpc(d.z)); }
__device__ __forceinline__ v3 rcp3(v3 d) {
    return mk(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
}


// =================================================================== shading ====
struct Surf {
    v3 pos, ng, ns, dpdu, dpdv;
    int obj;
};

__device__ __forceinline__ v3 tri_ns(const KParams& P, int i, float u, float v) {
    const float w = 1.0f - u - v;
    return xyz(P.tri_nrm[3 * i]) * w + xyz(P.tri_nrm[3 * i + 1]) * u + xyz(P.tri_nrm[3 * i + 2]) * v;
}

// Rebuild IntersectInfo::surfaceInfo as Scene::intersect leaves it (Src/primitive.cpp:
// 102-110, primitive.h:112-122).  Returns the hit object index (-1 = miss).
template <int SCN>
__device__ __forceinline__ int surface(const KParams& P, uint32_t s, v3 o, v3 d, f4 h, Surf& S, float& t1) {
    const int code = __float_as_int(h.w);
    S.pos = S.ng = S.ns = S.dpdu = S.dpdv = mk(0, 0, 0);
    t1 = kINF;
    if (code < 0) return -1;
    int surf = code, dp = (SCN == SCN_TRI) ? code : -1;
    float st = h.x, su = h.y, sv = h.z, du = h.y, dv = h.z;
    if (SCN == SCN_MIXED) {
        const f4 h2 = P.hit2[s], h3 = P.hit3[s];
        t1 = h2.x;
        surf = __float_as_int(h2.y), dp = __float_as_int(h2.z), st = h2.w;
        su = h3.x, sv = h3.y, du = h3.z, dv = h3.w;
    }
    if (surf >= 0) {
        const int kind = surf >> 28, idx = surf & 0x0fffffff;
        S.pos = ray_at(o, d, st);
        if (kind == SEG_TRI) {
            S.ng = xyz(P.tri_ng[idx]);
            S.ns = tri_ns(P, idx, su, sv);
        } else {
            S.ng = normalize(ray_at(o, d, st) - xyz(P.sph[idx]));
            S.ns = S.ng;
        }
    }
    if (dp >= 0) onb(tri_ns(P, dp & 0x0fffffff, du, dv), S.dpdu, S.dpdv);
    const int kind = code >> 28, idx = code & 0x0fffffff;
    if (kind == SEG_TRI) return __float_as_int(P.tri[3 * idx].w);
    if (kind == SEG_SPHERE) return P.sph_obj[idx] & 0x3fffffff;
    return __float_as_int(P.box[2 * idx].w);
}

// Component-wise quotients a / b and a / (b, b, b) with one division when the numerators (and
// denominators) are the same bits — achromatic media and throughputs (C5) — else three; the
// same IEEE quotients either way.  Bit equality, not ==: +0 and -0 differ in the quotient.
__device__ __forceinline__ bool same3(v3 a) {
    return __float_as_uint(a.x) == __float_as_uint(a.y) && __float_as_uint(a.y) == __float_as_uint(a.z);
}
__device__ __forceinline__ v3 div3s(v3 a, float b) {
    if (same3(a)) {
        const float q = a.x / b;
        return mk(q, q, q);
    }
    return a / b;
}
__device__ __forceinline__ v3 div3v(v3 a, v3 b) {
    if (same3(a) && same3(b)) {
        const float q = a.x / b.x;
        return mk(q, q, q);
    }
    return a / b;
}

// AreaLight::Le (Src/light.h:62-69)
__device__ __forceinline__ v3 light_Le(const DLight& L, v3 ns, v3 wi) {
    return dot(wi, ns) < 0.0f ? mk(L.Le[0], L.Le[1], L.Le[2]) : mk(0, 0, 0);
}

__device__ __forceinline__ v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

// QuadLight::sample (Src/light.cpp:59-68; first draw scales e2 under GCC),
// TriangleLight::sample (light.cpp:21-30,43-47; first draw is v),
// SphereLight::sample default branch (light.h:157-197) or, kind 3, its AREA_SAMPLING
// branch (light.h:131-135,185-191).  pdf is left untouched on the
// back-facing early return, as in the reference.
template <class RNG>
__device__ inline v3 light_sample(const DLight& L, v3 x, v3& wi, float& pdf, float& tmax, RNG& rng) {
    if (L.kind == 0) {
        const float ra = rng.next();
        const float rb = rng.next();
        const v3 dd = ((ld3(L.v0) + ld3(L.e1) * rb) + ld3(L.e2) * ra) - x;
        tmax = length(dd);
        const float dn = dot(dd, ld3(L.Ng));
        if (dn >= 0.0f) return mk(0, 0, 0);
        wi = dd / tmax;
        pdf = (tmax * tmax * tmax) / __builtin_fabsf(dn);
        return ld3(L.Le);
    } else if (L.kind == 1) {
        const float vv = rng.next();
        const float uu = rng.next();
        const float su = __builtin_sqrtf(uu);
        const v3 A = ld3(L.v0), B = ld3(L.v1), C = ld3(L.v2);
        const v3 p = (C + (A - C) * (1.0f - su)) + (B - C) * (vv * su);
        const v3 dd = p - x;
        tmax = length(dd);
        const float dn = dot(dd, ld3(L.Ng));
        if (dn >= 0.0f) return mk(0, 0, 0);
        wi = dd / tmax;
        pdf = (2.0f * tmax * tmax * tmax) / __builtin_fabsf(dn);
        return ld3(L.Le);
    } else if (L.kind == 3) {
        // SphereLight::sample built with AREA_SAMPLING (Src/light.h:131-135,185-191):
        // UniformSampleSphere(r1, r2) (Src/light.cpp:99-105) with GCC's right-to-left
        // operands — the first draw is r2 (phi), the second r1 (z)
        const float r2 = rng.next();
        const float r1 = rng.next();
        const float z = 1.f - 2.f * r1;
        const float sin_theta = __builtin_sqrtf(1.0f - z * z);
        float sphi, cphi;
        glibc_sincosf(kPI_MUL_2 * r2, sphi, cphi);
        const v3 nn = mk(cphi * sin_theta, sphi * sin_theta, z);
        const v3 dd = (ld3(L.center) + nn * L.radius) - x;
        tmax = length(dd);
        const float dn = dot(dd, nn);
        if (dn >= 0.0f) return mk(0, 0, 0);
        wi = dd / tmax;
        pdf = (2.0f * tmax * tmax * tmax) / __builtin_fabsf(dn);
        return ld3(L.Le);
    }
    const v3 center = ld3(L.center);
    const float radius = L.radius;
    v3 dz = center - x;
    const float dz_len_2 = dot(dz, dz);
    const float dz_len = __builtin_sqrtf(dz_len_2);
    dz = dz / mk(-dz_len, -dz_len, -dz_len);
    v3 dx, dy;
    onb(dz, dx, dy);
    const float sin_theta_max_2 = radius * radius / dz_len_2;
    const float sin_theta_max = __builtin_sqrtf(sin_theta_max_2);
    const float cos_theta_max = __builtin_sqrtf(smax(0.f, 1.f - sin_theta_max_2));
    const float cos_theta = 1.0f + (cos_theta_max - 1.0f) * rng.next();
    const float sin_theta_2 = 1.f - cos_theta * cos_theta;
    const float cos_alpha =
        sin_theta_2 / sin_theta_max + cos_theta * __builtin_sqrtf(smax(0.0f, 1.0f - sin_theta_2 / sin_theta_max_2));
    const float sin_alpha = __builtin_sqrtf(smax(0.0f, 1.0f - cos_alpha * cos_alpha));
    const float phi = kPI_MUL_2 * rng.next();
    float sphi, cphi;
    glibc_sincosf(phi, sphi, cphi);
    const v3 nn = (dx * (cphi * sin_alpha) + dy * (sphi * sin_alpha)) + dz * cos_alpha;
    const v3 p = center + nn * radius;
    const v3 dd = p - x;
    tmax = length(dd);
    if (dot(dd, nn) >= 0.0f) return mk(0, 0, 0);
    pdf = 1.f / (kPI_MUL_2 * (1.f - cos_theta_max));
    wi = dd / tmax;
    return ld3(L.Le);
}

// Lambert::sampleDir + uniformSampleHemisphere (Src/material.h:55-73)
template <class RNG>
__device__ __forceinline__ v3 lambert_sample_f(v3 ng, v3 dpdu, v3 dpdv, RNG& rng) {
    const float r1 = rng.next();
    const float r2 = rng.next();
    const float sinTheta = __builtin_sqrtf(1.0f - r1 * r1);
    const float phi = 2.0f * kPI * r2;
    float sphi, cphi;
    glibc_sincosf(phi, sphi, cphi);
    const float x = sinTheta * cphi;
    const float z = sinTheta * sphi;
    return local_to_world(mk(x, r1, z), dpdu, ng, dpdv);
}
__device__ __forceinline__ v3 lambert_sample(const Surf& S, Rng& rng) {
    const float r1 = rng.next();
    const float r2 = rng.next();
    const float sinTheta = __builtin_sqrtf(1.0f - r1 * r1);
    const float phi = 2.0f * kPI * r2;
    float sphi, cphi;
    glibc_sincosf(phi, sphi, cphi);
    const float x = sinTheta * cphi;
    const float z = sinTheta * sphi;
    return local_to_world(mk(x, r1, z), S.dpdu, S.ng, S.dpdv);
}

__device__ __forceinline__ v3 eval_bxdf(const DObj& ob) {   // Lambert::evaluateBxDF
    return ob.material == 1 ? ld3(ob.fr) : mk(0, 0, 0);   // albedo / PI, divided on the host
}

// x / (float)width, x / (float)height, x / aspect — the renderer's constant divisors.  Where
// the host proved Markstein's correction with its RN(1/c) equal to IEEE division for every
// mantissa of x (KParams::cdiv, xrt_api.cpp cdiv_exact), div_const's three operations
// replace the IEEE sequence; otherwise the IEEE division.  The flag is uniform: no
// divergence.
__device__ __forceinline__ float div_w(const KParams& P, float x) {
    return (P.cdiv & 1u) ? div_const(x, P.fw, P.rw) : x / (float)P.width;
}
__device__ __forceinline__ float div_h(const KParams& P, float x) {
    return (P.cdiv & 2u) ? div_const(x, P.fh, P.rh) : x / (float)P.height;
}
__device__ __forceinline__ float div_a(const KParams& P, float x) {
    return (P.cdiv & 4u) ? div_const(x, P.aspect, P.raspect) : x / P.aspect;
}

// PinholeCamera::sampleRay (Src/camera.h:49-60)
__device__ __forceinline__ void camera_ray(const KParams& P, float u, float v, v3& o, v3& d) {
    const v3 dir = mk((2.0f * u - 1.0f) * P.scale, div_a(P, (1.0f - 2.0f * v) * P.scale), -1.0f);
    const float* x = P.c2w;
    const v3 w = mk(dir.x * x[0] + dir.y * x[4] + dir.z * x[8], dir.x * x[1] + dir.y * x[5] + dir.z * x[9],
                    dir.x * x[2] + dir.y * x[6] + dir.z * x[10]);
    d = normalize(w);
    o = mk(x[12], x[13], x[14]);
}


// LDS carve of the fused schedule (bytes; every f4 region 16-aligned): triangles, their
// geometric and vertex normals, per-object culling boxes (triangle scenes), spheres,
// medium boxes, the object and light tables, sphere->object map.
struct StepLayout {
    uint32_t tri, tng, nrm, box, sph, bx, obj, light, sobj, snode, ssph, sbk, total;
};
// Sphere scenes with a skip-link BVH (P.n_snode > 0, C3) keep the BVH, the spheres in leaf
// order and their index/occluder words in LDS; the original-order sphere, sphere-object
// and object tables (read once per hit, at shading) stay in global memory.
__host__ __device__ inline StepLayout step_layout(const KParams& P) {
    const bool sb = P.n_snode > 0;
    StepLayout L;
    L.tri = 0;
    L.tng = L.tri + 48u * P.n_tris;
    L.nrm = L.tng + 16u * P.n_tris;
    L.box = L.nrm + 48u * P.n_tris;
    L.sph = L.box + (P.scene_kind == SCN_TRI ? 32u * P.n_objs : 0u);
    L.bx = L.sph + (sb ? 0u : 16u * P.n_sph);
    L.obj = L.bx + 32u * P.n_box;
    L.light = L.obj + (sb ? 0u : (uint32_t)sizeof(DObj) * P.n_objs);
    L.sobj = L.light + (uint32_t)sizeof(DLight) * P.n_lights;
    L.snode = L.sobj + (sb ? 0u : 4u * P.n_sph);
    L.ssph = L.snode + 32u * (uint32_t)P.n_snode;
    L.sbk = L.ssph + (sb ? 16u * P.n_sph : 0u);
    L.total = L.sbk + (sb ? 4u * P.n_sph : 0u);
    return L;
}

// NormalIntegrator's colour 0.5f * (ns + 1.0f) (Src/integrator.h:36): Vec3f + float, then
// float * Vec3f, component-wise
__device__ __forceinline__ v3 normal_color(v3 ns) {
    return mk(0.5f * (ns.x + 1.0f), 0.5f * (ns.y + 1.0f), 0.5f * (ns.z + 1.0f));
}

// ============================================================ fused schedule ====
// k_step: per live slot, up to `visits` path segments in one launch with the path state in
// registers: trace the pending ray, shade the hit (NEE shadow rays traced immediately, so
// no shadow state crosses a segment), finish/regenerate samples — the per-pixel sequence
// of NormalRenderer::doRender + integrate().  The scene and its tables live in LDS
// (step_layout), so this schedule serves scenes up to kStepLds bytes (C1, C2, C3, C5);
// larger scenes use the multi-pass wavefront (k_shade / k_trace with LDS tiles).  A slot
// stops early when its RNG ring runs low or it is done; at the end of the launch the slot
// is appended to the next round's live list and, when fewer than rng_keep words are left,
// its wave twists the slot's next block in-line (wave_refill) — only the seeding twist of
// every slot is a k_refill launch.
struct LScene {
    const f4* tri;      // 3 per triangle
    const f4* tng;      // geometric normal per triangle
    const f4* nrm;      // 3 vertex normals per triangle
    const DObjBox* box; // per object (SCN_TRI)
    const f4* sph;
    const int* sobj;
    const f4* bx;       // 2 per box
    const DObj* obj;
    const DLight* light;
    const f4* snode = nullptr;   // sphere BVH (SkipNode: {bmin, skip}, {bmax, leaf}); n_snode > 0
    const f4* ssph = nullptr;    // spheres in BVH leaf order
    const int* sbk = nullptr;    // original sphere index | (occluder << 30)
    int n_snode = 0;
};


__device__ __forceinline__ v3 tri_ns_l(const LScene& L, int i, float u, float v) {
    const float w = 1.0f - u - v;
    return xyz(L.nrm[3 * i]) * w + xyz(L.nrm[3 * i + 1]) * u + xyz(L.nrm[3 * i + 2]) * v;
}


template <typename T>
__device__ __forceinline__ void lds_copy(T* dst, const T* src, int n, int tid, int stride = kBlock) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    const int words = n * (int)(sizeof(T) / 4);
    for (int q = tid; q < words; q += stride) d[q] = s[q];
}


}  // namespace xrt
