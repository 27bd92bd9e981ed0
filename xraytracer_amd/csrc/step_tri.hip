// step_tri.hip — merged-trace fused schedule for small triangle scenes (C1, C2: the
// Cornell box), the latency-critical kernel of the renderer.
//
// Same per-pixel sequence as NormalRenderer::doRender + GIIntegrator / DirectIntegrator
// (Src/renderer.cpp:29-81, Src/integrator.h:82-119, 205-287), one path slot per pixel, path
// state in registers for `visits` segments per launch.  What differs from k_step_tri
// (wavefront.hip) is the schedule of the traces:
//
//  * One cooperative trace per segment.  The NEE shadow rays of segment i and the
//    extension ray of segment i+1 (or the next sample's camera ray) are traced together:
//    every RNG draw of segment i (RR, light samples, BSDF sample, the next sample's jitter)
//    happens in the reference's order before either ray is traced, and the occlusion
//    result only changes the radiance, never a draw.  The contribution is kept for both
//    outcomes (c1: visible, c0: occluded — the reference multiplies by vis first, so both
//    are computed with its operation order) and added after the trace, still before any
//    later radiance update of the same path, so every float sum happens in the
//    reference's order.  A sample that ends with shadow rays in flight is finished after
//    they resolve (rad_fin), while its successor's camera ray is traced.
//  * Object-major pair passes: for each object (kernel-argument record, scalar loads) the
//    wave ballots which of its rays (1 + NL per lane) overlap the object's culling box,
//    ranks those rays into LDS (mbcnt; origin + tmax, direction + ray id) and tests the
//    (ray, triangle) pairs 64 per pass,
//    pair j -> ray rank j / count (magic multiply), triangle first + j % count.  No prefix
//    scan, no per-lane expansion loop.  Closest hits merge with an LDS atomicMin of
//    (t bits << 32 | triangle): smallest t, ties to the lower triangle index — the
//    reference's in-order strict `t < best` scan; shadow rays set an occlusion bit.
//  * The RNG words a segment can use (6 + 2 NL at most) are prefetched into registers by
//    global (not flat) loads issued one segment ahead.
//
// GIIntegrator with maxDepth 0 and scenes with more than kMergedMaxObjs objects keep using
// k_step_tri.
#include "bvh.h"
#include "launch.h"
#include "merged.h"
#include "path_common.h"

namespace xrt {


// One cooperative trace of the wave: the extension ray (closest hit, if `ext`) and the
// pending shadow rays (any hit, bits of `shm`).  ORIG: the closest-hit key's low word is the
// triangle's original index (the w of its third float4, KParams::stri) instead of its LDS
// index — two-level scenes, whose BVH walk merges in the same (t, original index) order.
template <int NL, bool ORIG = false>
__device__ __forceinline__ void merged_trace(const StepObjs& SO, const LScene& L, MergedWave<NL>& W, int lane,
                                             bool ext, v3 o, v3 d, uint32_t shm, const v3 (&so)[NL + 1],
                                             const v3 (&sd)[NL + 1], const float (&stm)[NL + 1],
                                             unsigned long long& best, uint32_t& occ
) {
    constexpr int R = 1 + NL;
    W.best[lane] = ~0ull;
    W.occ[lane] = 0u;
    v3 inv[R], oi[R];
    inv[0] = rcp3c(d);
    oi[0] = o * inv[0];
#pragma unroll
    for (int l = 0; l < NL; ++l) inv[1 + l] = rcp3c(sd[l]), oi[1 + l] = so[l] * inv[1 + l];
    wave_sync();
    const int n = SO.n;
    for (int ob = 0; ob < n; ++ob) {
        const StepObj B = SO.o[ob];
        bool need[R];
#if XRT_TRACE_TLIM
        // the objects so far: an extension ray skips an object whose box it enters beyond its
        // closest hit (every triangle inside lies deeper than the box margin, far above the
        // float error of either t; ties are still tested), a shadow ray one it is occluded by
        const unsigned long long cur = W.best[lane];
        const float bt = cur == ~0ull ? kINF : __uint_as_float((uint32_t)(cur >> 32));
        const uint32_t done = W.occ[lane];
#else
        const float bt = kINF;
        const uint32_t done = 0u;
#endif
        need[0] = ext && !plane_away(o, d, B.axis, B.plane) && obj_overlap(oi[0], inv[0], B, bt);
#pragma unroll
        for (int l = 0; l < NL; ++l)
            need[1 + l] = B.occluder && ((shm & ~done) >> l & 1u) && !plane_away(so[l], sd[l], B.axis, B.plane) &&
                          obj_overlap(oi[1 + l], inv[1 + l], B, stm[l]);
        // the rays themselves are ranked into W (not their ids), so a pair reads its ray
        // with one LDS access instead of an id and then the ray
        uint32_t tot = 0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const uint64_t m = __ballot(need[q]);
            if (need[q]) {
                const uint32_t at = tot + lanemask_rank(m);
                const v3 ro = q == 0 ? o : so[q - 1], rd = q == 0 ? d : sd[q - 1];
                W.ro[at] = make_float4(ro.x, ro.y, ro.z, q == 0 ? kINF : stm[q - 1]);
                W.rd[at] = make_float4(rd.x, rd.y, rd.z, __uint_as_float((uint32_t)(q * 64 + lane)));
            }
            tot += (uint32_t)__popcll(m);
        }
        if (tot == 0) continue;
        wave_sync();
        const uint32_t c = B.count, first = (uint32_t)B.first;
        const uint32_t pairs = tot * c;
        const uint32_t magic = B.magic;
        // one (ray, triangle) pair per lane and step: an out-of-range lane of the last step
        // tests the last pair again with its result dropped (no divergent branch; two steps
        // per iteration with both tests before the merges measured 5% slower on C2)
        struct PairHit {
            bool hit;
            uint32_t e, idx;
            float t, tw;
        };
        auto test = [&](uint32_t j) {
            const bool valid = j < pairs;
            const uint32_t jj = valid ? j : pairs - 1u;
            const uint32_t r = (c == 1u) ? jj : __umulhi(jj, magic);
            const uint32_t k = first + (jj - r * c);
            const f4 A = W.ro[r];
            const f4 D = W.rd[r];
            const f4 C = L.tri[3 * k + 2];
            PairHit p;
            p.hit = ray_tri_nb(xyz(A), xyz(D), xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(C), p.t) && valid;
            p.e = __float_as_uint(D.w), p.tw = A.w, p.idx = ORIG ? __float_as_uint(C.w) : k;
            return p;
        };
        auto merge = [&](const PairHit& p) {
            if (p.hit) {
                if (p.e < 64u)
                    atomicMin(&W.best[p.e], ((unsigned long long)__float_as_uint(p.t) << 32) | p.idx);
                else if (p.t < p.tw)
                    atomicOr(&W.occ[p.e & 63u], 1u << ((p.e >> 6) - 1u));
            }
        };
        for (uint32_t j0 = 0; j0 < pairs; j0 += 64u) merge(test(j0 + (uint32_t)lane));
        wave_sync();
    }
    best = W.best[lane];
    occ = W.occ[lane];
}

// ------------------------------------------- two-level trace inside the wave ----
// The fused schedule for two-level scenes (C4: the Cornell box around a 51,200-triangle
// sphere mesh; k_step_merged<..., BVH = true>): after merged_trace has tested the small
// objects (LDS, pair passes, keys (t bits << 32 | original index)), the rays whose segment
// still reaches the BVH — extension rays over [0, best t], shadow rays over [0, tmax] if no
// small object occluded them — are ranked into the wave's scratch and walked by the wave's
// 16 quads, k_trace_deep4q's four-lanes-per-ray walk of the 4-wide BVH (lane c owns child
// c of the current node; the quad shares the pruning limit, occlusion and the next node by
// DPP), a quad taking the next ranked ray when its walk ends.  Results merge into the
// wave's records as merged_trace leaves them: the smallest (t, original index) key by the
// lane holding it, occlusion bits by an or.  Exact for the reasons k_trace_deep4q is (every
// triangle whose padded box overlaps [0, best t] is tested by some lane) — the same
// lexicographic minimum over every triangle the reference's linear scan tests
// (Src/scene.cpp:190-211, Src/primitive.cpp:83-168).
constexpr int kQs = 64;          // quad stack entries (circular; >= kBvh4Stack)
constexpr int kQsMask = kQs - 1;
static_assert(kQs >= kBvh4Stack, "quad stacks");

// The walk of n_deep ranked rays ray_o / ray_d (w: tmax resp. the ray id q * 64 + lane; q = 0:
// extension ray, closest hit from the key best[lane]; 1 + l: shadow ray l, occlusion bit l of
// occ[lane]).  top: the first ntop 4-wide nodes in LDS; stk: this wave's 16 quad stacks
// (stride 16).  Must be called by every lane of the wave.
template <typename SE>
__device__ __forceinline__ void wave_deep_walk(const KParams& P, const f4* top, int ntop, SE* stk, const f4* ray_o,
                                               const f4* ray_d, unsigned long long* best, uint32_t* occ, int lane,
                                               uint32_t n_deep) {
    constexpr uint64_t kLeads = 0x1111111111111111ull;   // lane 0 of every quad
    const int c = lane & 3;
    SE* qs = stk + (lane >> 2);
    uint32_t next = 0;   // wave-uniform: first ray not yet taken
    bool active = false, any = false;
    uint32_t id = 0;   // the ray's id
    int node = 0, sp = 0, base = 0, bk = -1;   // stack entries [base, sp), circular (kQs)
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0), inv = mk(0, 0, 0);
    float tmax = 0.0f, bt = kINF;
    while (true) {
        if (next < n_deep) {
            const uint64_t idle = __ballot(!active) & kLeads;
            if (idle) {
                const uint32_t idx = next + (uint32_t)__popcll(idle & ((1ull << (lane & ~3)) - 1ull));
                if (!active && idx < n_deep) {
                    const f4 A = ray_o[idx], D = ray_d[idx];
                    id = __float_as_uint(D.w);
                    any = id >= 64u;
                    o = xyz(A), d = xyz(D), tmax = A.w;
                    bt = kINF, bk = -1;
                    if (!any) {
                        const unsigned long long key = best[id];
                        if (key != ~0ull) bt = __uint_as_float((uint32_t)(key >> 32)), bk = (int)(uint32_t)key;
                    }
                    inv = rcp3(d);
                    node = 0, sp = 0, base = 0;
                    active = true;
                }
                next += (uint32_t)__popcll(idle);
            }
        }
        if (!__ballot(active)) break;
        if (!active) continue;
        // ---- one node, with as few divergent branches as the step allows (the loop's exec-mask
        // bookkeeping cost about as many scalar instructions as it had vector ones): the node
        // from LDS or global memory through one generic pointer, every leaf triangle's test and
        // both reductions computed for closest-hit and any-hit rays alike, the stack top read
        // every step.  (Measured and not kept, DESIGN.md §3: a branchy form, fetching the likely
        // next node before the leaf tests, work stealing between quads.)
        const f4* N = node < ntop ? top + 8 * node : P.bvh4 + 8 * (size_t)node;
        const f4 lo = N[c], hi = N[4 + c];
        const int cidx = __float_as_int(lo.w), ccnt = __float_as_int(hi.w);
        const float lim0 = any ? tmax : __uint_as_float(group_min32<4>(__float_as_uint(bt)));   // t >= 0: bits order
        const float e = ccnt >= 0 ? bvh_enter(lo, hi, o, inv, lim0) : __builtin_inff();
        bool oc = false;
        {
            // the overlapped leaf children's triangles, dealt round robin over the quad's lanes
            const uint32_t mine = (ccnt > 0 && e != __builtin_inff()) ? (uint32_t)ccnt : 0u;
            const uint32_t n0 = dpp32<0x00>(mine), n1 = dpp32<0x55>(mine), n2 = dpp32<0xAA>(mine), n3 = dpp32<0xFF>(mine);
            const uint32_t f0 = dpp32<0x00>((uint32_t)cidx), f1 = dpp32<0x55>((uint32_t)cidx);
            const uint32_t f2 = dpp32<0xAA>((uint32_t)cidx), f3 = dpp32<0xFF>((uint32_t)cidx);
            const uint32_t p1 = n0, p2 = n0 + n1, p3 = p2 + n2, tot = p3 + n3;
            constexpr int B = XRT_DEEP_LEAF_BATCH;
            for (uint32_t j0 = (uint32_t)c; j0 < tot; j0 += 4u * B) {
                f4 T[B][3];
                bool ok[B];
#pragma unroll
                for (int b = 0; b < B; ++b) {   // out-of-range slots load triangle 0, unused
                    const uint32_t j = j0 + 4u * (uint32_t)b;
                    ok[b] = j < tot;
                    const uint32_t t = !ok[b] ? 0u : j < p1 ? f0 + j : j < p2 ? f1 + (j - p1) : j < p3 ? f2 + (j - p2)
                                                                                                          : f3 + (j - p3);
                    const size_t i = 3 * (size_t)t;
                    T[b][0] = ldg4(P.bvh_tri, i), T[b][1] = ldg4(P.bvh_tri, i + 1), T[b][2] = ldg4(P.bvh_tri, i + 2);
                }
#pragma unroll
                for (int b = 0; b < B; ++b) {
                    float t;
                    const bool hit = ok[b] && ray_tri_nb(o, d, xyz(T[b][0]), xyz(T[b][1]), xyz(T[b][2]), t);
                    // any hit: area-light objects never occlude (e1.w = occluder flag)
                    oc |= hit && T[b][1].w != 0.0f && t < tmax;
                    const int k = __float_as_int(T[b][2].w);
                    const bool upd = !any && hit && (t < bt || (t == bt && k < bk));
                    bt = upd ? t : bt;
                    bk = upd ? k : bk;
                }
            }
        }
        bool done = any && group_or32<4>(oc ? 1u : 0u) != 0u;
        if (done && c == 0) atomicOr(&occ[id & 63u], 1u << ((id >> 6) - 1u));
        const float lim = any ? tmax : __uint_as_float(group_min32<4>(__float_as_uint(__builtin_fminf(lim0, bt))));
        {
            const bool inner = !done && ccnt == 0 && e <= lim;   // interior child still overlapping [0, lim]
            const uint32_t nkey = inner ? ((__float_as_uint(e) & ~3u) | (uint32_t)c) : ~0u;
            const uint32_t nmin = group_min32<4>(nkey);
            const bool has = nmin != ~0u;
            const bool nearest = inner && nkey == nmin;
            const uint32_t m4 = (uint32_t)(__ballot(inner && !nearest) >> (lane & ~3)) & 0xfu;
            if (inner && !nearest) qs[((sp + __popc(m4 & ((1u << c) - 1u))) & kQsMask) * 16] = (SE)cidx;
            sp += __popc(m4);
            const int child = (int)group_or32<4>(nearest ? (uint32_t)cidx : 0u);
            const bool pop = !done && !has && sp > base;
            const int top_entry = (int)qs[((sp - 1) & kQsMask) * 16];   // read every step; used on a pop
            sp -= pop ? 1 : 0;
            node = has ? child : top_entry;
            done = done || (!has && !pop);
        }
        if (done) {
            if (!any) {   // the quad's closest hit: the smallest (t bits, index) of the lanes
                const uint64_t key = bk >= 0 ? ((uint64_t)__float_as_uint(bt) << 32) | (uint32_t)bk : ~0ull;
                const uint64_t kmin = group_min64<4>(key);
                if (c == 0 && kmin != ~0ull) best[id] = kmin;
            }
            active = false;
        }
    }
}

// After merged_trace<NL, true> over the small objects: rank the rays whose segment still
// reaches the BVH root (the same root test as phase A's queueing, k_trace_2a_coop) into the
// wave's scratch, walk them, and return the merged records.  Must be called by every lane.
template <int NL, typename SE>
__device__ __forceinline__ void deep_pass(const KParams& P, const f4* top, int ntop, SE* stk, MergedWave<NL>& W,
                                          int lane, const f4 (&root)[4], bool ext, v3 o, v3 d, uint32_t shm,
                                          const v3 (&so)[NL + 1], const v3 (&sd)[NL + 1], const float (&stm)[NL + 1],
                                          unsigned long long& best, uint32_t& occ) {
    constexpr int R = 1 + NL;
    bool need[R];
    const float bt = best == ~0ull ? kINF : __uint_as_float((uint32_t)(best >> 32));
    need[0] = ext && root_overlap(root[0], root[1], root[2], root[3], o, rcp3(d), bt);
#pragma unroll
    for (int l = 0; l < NL; ++l)
        need[1 + l] = ((shm & ~occ) >> l & 1u) && root_overlap(root[0], root[1], root[2], root[3], so[l], rcp3(sd[l]), stm[l]);
    wave_sync();   // the last pair pass's reads of W.ro / W.rd are done
    uint32_t tot = 0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const uint64_t m = __ballot(need[q]);
        if (need[q]) {
            const uint32_t at = tot + lanemask_rank(m);
            const v3 ro = q == 0 ? o : so[q - 1], rd = q == 0 ? d : sd[q - 1];
            W.ro[at] = make_float4(ro.x, ro.y, ro.z, q == 0 ? kINF : stm[q - 1]);
            W.rd[at] = make_float4(rd.x, rd.y, rd.z, __uint_as_float((uint32_t)(q * 64 + lane)));
        }
        tot += (uint32_t)__popcll(m);
    }
    if (tot == 0) return;
    wave_sync();
    wave_deep_walk<SE>(P, top, ntop, stk, W.ro, W.rd, W.best, W.occ, lane, tot);
    wave_sync();
    best = W.best[lane];
    occ = W.occ[lane];
}

// LDS of k_step_merged<..., BVH = true> (bytes; the f4 regions 16-aligned): the small
// objects' triangles (KParams::stri), the object and light tables, the first ntop 4-wide
// BVH nodes, one MergedWave of trace scratch per wave, then 16 quad stacks of bvh4_stack 16-bit entries per wave
// (use_step_bvh: at most 65,536 nodes).
constexpr uint32_t kStackWave = 16u * kQs * 2u;   // a wave's 16 quad stacks (16-bit entries)
struct BvhStepLayout {
    uint32_t tri, obj, light, top, wave, stack, total;
    int ntop;
};
__host__ __device__ inline BvhStepLayout bvh_step_layout(const KParams& P, uint32_t wave_bytes) {
    BvhStepLayout B;
    B.tri = 0;
    B.obj = 48u * (uint32_t)P.n_stri;
    B.light = B.obj + (uint32_t)sizeof(DObj) * (uint32_t)P.n_objs;
    B.top = (B.light + (uint32_t)sizeof(DLight) * (uint32_t)P.n_lights + 15u) & ~15u;
    // as many of the top XRT_BVH_TOP nodes as the rest leaves room for within kStepLds
    const uint32_t rest = B.top + (kBlock / 64) * wave_bytes + (kBlock / 64) * kStackWave;
    const int fit = rest < kStepLds ? (int)((kStepLds - rest) / 128u) : 0;
    B.ntop = P.bvh4_nodes < XRT_BVH_TOP ? P.bvh4_nodes : XRT_BVH_TOP;
    B.ntop = B.ntop < fit ? B.ntop : fit;
    B.wave = B.top + 128u * (uint32_t)B.ntop;
    B.stack = B.wave + (kBlock / 64) * wave_bytes;
    B.total = B.stack + (kBlock / 64) * kStackWave;
    return B;
}

// ------------------------------------------------- two-level trace, phase A ----
// k_trace_2a (wavefront.hip) with the small objects traced by merged_trace's object-major
// pair passes instead of a per-lane object loop: one wave = 64 slots, their extension ray
// and shadow rays, the small objects' triangles in LDS (KParams::stri, iteration order, so
// the (t bits << 32 | local index) minimum is the (t, original index) minimum).  The winner's
// (t, u, v) are recomputed with Mesh::rayTriangleIntersect's ops as the merged kernel does;
// rays whose segment reaches the BVH root are queued for k_trace_deep.
template <int NL>
__global__ __launch_bounds__(kBlock, XRT_2A_WAVES) void k_trace_2a_coop(KParams P, const StepObjs SO, const uint32_t* __restrict__ list,
                                                          const uint32_t* __restrict__ count, uint32_t* zero_count) {
    extern __shared__ __attribute__((aligned(16))) f4 lds_2c[];
    LScene L;
    L.tri = lds_2c;
    MergedWave<NL>* Wv = reinterpret_cast<MergedWave<NL>*>(lds_2c + 3 * P.n_stri);
    const int tid = threadIdx.x, lane = tid & 63;
    MergedWave<NL>& W = Wv[tid >> 6];
    lds_copy(const_cast<f4*>(L.tri), P.stri, 3 * P.n_stri, tid);
    zero_parts(P, zero_count);
    __syncthreads();
    const f4 r0 = P.bvh_node[0], r1 = P.bvh_node[1], r2 = P.bvh_node[2], r3 = P.bvh_node[3];   // root
    const PartIter it = part_iter(P, count, kBlock);
    uint32_t* dq = P.deep + (size_t)it.p * P.deep_cap;
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        const bool valid = i < it.n;
        const uint32_t s = valid ? list[it.p * P.part_cap + i] : 0;
        const uint32_t st = valid ? P.state[s] : 0;
        const bool want = (st & ST_RAY) != 0;
        const uint32_t smask = (st >> ST_SHADOW_SHIFT) & ((1u << NL) - 1u);
        v3 o = mk(0, 0, 0), d = mk(0, 0, 0);
        if (want) o = xyz(P.ray_o[s]), d = xyz(P.ray_d[s]);
        v3 so[NL + 1], sd[NL + 1];
        float stm[NL + 1];
#pragma unroll
        for (int l = 0; l <= NL; ++l) so[l] = sd[l] = mk(0, 0, 0), stm[l] = 0.0f;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            if (smask & (1u << l)) {
                const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                so[l] = xyz(a), stm[l] = a.w;
                sd[l] = xyz(P.sh_d[(size_t)l * P.n_slots + s]);
            }
        }
        unsigned long long best;
        uint32_t occ;
        merged_trace<NL>(SO, L, W, lane, want, o, d, smask, so, sd, stm, best, occ);
        float bt = kINF, bu = 0.0f, bv = 0.0f;
        int bk = -1;
        if (want && best != ~0ull) {
            const int hk = (int)(uint32_t)best;
            (void)ray_tri(o, d, xyz(L.tri[3 * hk]), xyz(L.tri[3 * hk + 1]), xyz(L.tri[3 * hk + 2]), bt, bu, bv);
            bk = __float_as_int(L.tri[3 * hk + 2].w);
        }
        const v3 inv = rcp3(d);
        const bool dext = want && root_overlap(r0, r1, r2, r3, o, inv, bt);
        uint32_t dsh = 0;
#pragma unroll
        for (int l = 0; l < NL; ++l)
            if ((smask & ~occ & (1u << l)) && root_overlap(r0, r1, r2, r3, so[l], rcp3(sd[l]), stm[l])) dsh |= 1u << l;
        if (valid) {
            if (want) P.hit[s] = make_float4(bt, bu, bv, __int_as_float(bk));
            if (smask) P.occ[s] = occ & smask;
        }
        wave_append(valid && dext, s * 8u, dq, P.deep_count + it.p, lane);
#pragma unroll
        for (int l = 0; l < NL; ++l)
            wave_append(valid && ((dsh >> l) & 1u), s * 8u + 1u + (uint32_t)l, dq + P.part_cap,
                        P.deep_count + 2 * kMaxParts + it.p, lane);
        wave_sync();   // W is rewritten by the next round's rays
    }
}

hipError_t launch_trace_2a_coop(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* zero,
                                uint32_t blocks, hipStream_t st) {
    if (P.n_lights <= 1) {
        const size_t lds = (size_t)P.n_stri * 3 * sizeof(f4) + (kBlock / 64) * sizeof(MergedWave<1>);
        hipLaunchKernelGGL((k_trace_2a_coop<1>), dim3(blocks), dim3(kBlock), lds, st, P, *P.sstep, list, count, zero);
    } else {
        const size_t lds = (size_t)P.n_stri * 3 * sizeof(f4) + (kBlock / 64) * sizeof(MergedWave<kMaxLights>);
        hipLaunchKernelGGL((k_trace_2a_coop<kMaxLights>), dim3(blocks), dim3(kBlock), lds, st, P, *P.sstep, list, count,
                           zero);
    }
    return hipGetLastError();
}

// --------------------------------------------------------------- RNG refills ----
// k_refill_merged: every slot's first twist (the seeding refill after k_seed; later twists
// happen in-line at the end of the step launch a slot runs low in, wave_refill).  Same twist
// as wave_twist (libstdc++ _M_gen_rand: x[g+k] = x[g+k-227] ^ mix(x[g+k-624], x[g+k-623]),
// chunks k = m, 227+m, 454+m held in registers), arranged for bandwidth: the old block is
// staged through LDS (below), the next request's slot, stream position and old block are
// fetched while the current one twists, and the slot state is not touched — the merged
// kernel clears ST_RNGREQ when it first loads the slot, which is always after this kernel.


// SPW: path slots per wave (64, 32 or 16), G: lanes per slot (1, or 64 / SPW for the group
// trace).  With G = 1 and SPW < 64, lanes >= SPW own no slot but take part in every pair
// pass of the cooperative traces, so a half- or quarter-filled wave traces its rays in
// proportionally fewer passes; with G > 1 every lane of a slot's group runs its path
// (redundantly, results identical) and the group shares the traces (group_trace).  Either
// way, with few slots per GPU (a pixel shard of a multi-GPU frame) this puts more, shorter
// waves on every SIMD.
// BVH: two-level scenes (use_step_bvh: C4) — the small objects' triangles in LDS and traced
// by merged_trace with original-index keys, the rest by the wave's BVH walk (deep_pass);
// the hit triangle's shading data from global memory.  Same path
// code otherwise.

// WV (two-level scenes): a register budget for WV waves per SIMD instead of XRT_BVH_WAVES, for
// launches with too few live slots to fill more (fewer spills)
template <int INTEG, int NL, int SPW, int G, bool LANE, bool BVH, int WV = 0>
__global__ __launch_bounds__(kBlock, WV ? WV : (BVH ? XRT_BVH_WAVES : XRT_STEP_WAVES)) void k_step_merged(
    const KParams* __restrict__ Pp, const StepObjs SO, const uint32_t* __restrict__ list,
    const uint32_t* __restrict__ count, uint32_t* __restrict__ out, uint32_t* out_count, uint32_t* zero_count,
    uint32_t* req_count, uint32_t visits) {
    constexpr int NW = 6 + 2 * NL;   // most words one segment draws (see the header)
    static_assert(!BVH || (G == 1 && !LANE), "two-level scenes trace by pair passes");
    const KParams& P = *Pp;
    extern __shared__ __attribute__((aligned(16))) f4 lds_m[];
    char* lb = reinterpret_cast<char*>(lds_m);
    const int tid = threadIdx.x, lane = tid & 63;
    LScene L;
    const DObjPlane* lplane = nullptr;
    MergedWave<NL>* Wp;
    const f4* top = nullptr;   // BVH: the first ntop 4-wide nodes
    uint16_t* stk = nullptr;   // BVH: this wave's quad stacks
    int ntop = 0;
    f4 root[4];                // BVH: the binary root node (deep_pass's root test)
    if constexpr (BVH) {
        const BvhStepLayout Bl = bvh_step_layout(P, (uint32_t)sizeof(MergedWave<NL>));
        L.tri = reinterpret_cast<const f4*>(lb + Bl.tri);
        L.obj = reinterpret_cast<const DObj*>(lb + Bl.obj);
        L.light = reinterpret_cast<const DLight*>(lb + Bl.light);
        top = reinterpret_cast<const f4*>(lb + Bl.top);
        ntop = Bl.ntop;
        Wp = reinterpret_cast<MergedWave<NL>*>(lb + Bl.wave);
        stk = reinterpret_cast<uint16_t*>(lb + Bl.stack + (tid >> 6) * kStackWave);
        lds_copy(const_cast<f4*>(L.tri), P.stri, 3 * P.n_stri, tid);
        lds_copy(const_cast<DObj*>(L.obj), P.objs, P.n_objs, tid);
        lds_copy(const_cast<DLight*>(L.light), P.lights, P.n_lights, tid);
        lds_copy(const_cast<f4*>(top), P.bvh4, 8 * ntop, tid);
        root[0] = ldg4(P.bvh_node, 0), root[1] = ldg4(P.bvh_node, 1), root[2] = ldg4(P.bvh_node, 2);
        root[3] = ldg4(P.bvh_node, 3);
    } else {
        const StepLayout Lo = step_layout(P);
        L.tri = reinterpret_cast<const f4*>(lb + Lo.tri);
        L.tng = reinterpret_cast<const f4*>(lb + Lo.tng);
        L.nrm = reinterpret_cast<const f4*>(lb + Lo.nrm);
        L.box = reinterpret_cast<const DObjBox*>(lb + Lo.box);
        L.sph = reinterpret_cast<const f4*>(lb + Lo.sph);
        L.bx = reinterpret_cast<const f4*>(lb + Lo.bx);
        L.obj = reinterpret_cast<const DObj*>(lb + Lo.obj);
        L.light = reinterpret_cast<const DLight*>(lb + Lo.light);
        L.sobj = reinterpret_cast<const int*>(lb + Lo.sobj);
        lplane = reinterpret_cast<const DObjPlane*>(lb + merged_plane_off(Lo));
        Wp = reinterpret_cast<MergedWave<NL>*>(lb + merged_wave_off(P, Lo));
        lds_copy(const_cast<f4*>(L.tri), P.tri, 3 * P.n_tris, tid);
        lds_copy(const_cast<f4*>(L.tng), P.tri_ng, P.n_tris, tid);
        lds_copy(const_cast<f4*>(L.nrm), P.tri_nrm, 3 * P.n_tris, tid);
        lds_copy(const_cast<DObj*>(L.obj), P.objs, P.n_objs, tid);
        lds_copy(const_cast<DLight*>(L.light), P.lights, P.n_lights, tid);
        if (LANE) {
            lds_copy(const_cast<DObjBox*>(L.box), P.obj_box, P.n_objs, tid);
            lds_copy(const_cast<DObjPlane*>(lplane), P.obj_plane, P.n_objs, tid);
        }
    }
    MergedWave<NL>& W = Wp[tid >> 6];
    static_assert(sizeof(MergedWave<NL>) >= kMT * 4, "the wave's trace scratch doubles as the refill buffer");
    // the hit triangle's records: LDS (the whole scene is there) or, two-level, global memory
    // (hk is then the triangle's original index)
    auto tri_rec = [&](int i) -> f4 {
        if constexpr (BVH) return ldg4(P.tri, i);
        else return L.tri[i];
    };
    auto tri_ng_at = [&](int i) -> v3 {
        if constexpr (BVH) return xyz(ldg4(P.tri_ng, i));
        else return xyz(L.tng[i]);
    };
    auto tri_ns_at = [&](int i, float u, float v) -> v3 {
        if constexpr (BVH) {
            const float w = 1.0f - u - v;
            return xyz(ldg4(P.tri_nrm, 3 * (size_t)i)) * w + xyz(ldg4(P.tri_nrm, 3 * (size_t)i + 1)) * u +
                   xyz(ldg4(P.tri_nrm, 3 * (size_t)i + 2)) * v;
        } else {
            return tri_ns_l(L, i, u, v);
        }
    };
    __syncthreads();
    zero_parts(P, zero_count);
    const PartIter it = part_iter(P, count, (kBlock / 64) * SPW);
    const uint32_t spp = P.spp, max_depth = P.max_depth, width = P.width;
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + (uint32_t)(tid >> 6) * SPW + (uint32_t)lane / G;
        const bool own = lane / G < SPW && i < it.n;
        const bool lead = own && (lane % G) == 0;   // the lane of a group that writes back
        const uint32_t s = own ? list[it.p * P.part_cap + i] : 0;
        uint32_t st = own ? glb<gu32>(P.state)[s] : ST_DONE;
        st &= ~ST_RNGREQ;   // the refill this slot asked for ran after the previous launch
        const bool live = !(st & ST_DONE);
        uint32_t g = 0, depth = 0, k = 0, kst = 0;   // k: finished samples, kst: started samples
        RngRegs<NW> rng;
        rng.c = 0;
        const uint32_t* ring = P.ring + (size_t)s * kRing;
        v3 thr = mk(1, 1, 1), rad = mk(0, 0, 0), o = mk(0, 0, 0), d = mk(0, 0, 0), acc = mk(0, 0, 0);
        v3 rad_fin = mk(0, 0, 0), thr_nee = mk(0, 0, 0);
        v3 so[NL + 1], sd[NL + 1], c1[NL + 1], c0[NL + 1];
        // GI with one light: the NEE term is folded at sampling time — c1[0] holds
        // thr * (0 + (0 + c1)) and c0z the codes of thr * (0 + (0 + c0)) (each component +-0 or
        // NaN), the exact values resolve() would form from thr_nee and c0 / c1 — so neither
        // thr_nee nor c0 stays live across the trace
        constexpr bool kFold = INTEG == XRT_INTEGRATOR_GI && NL == 1;
        uint32_t c0z = 0;
        float stm[NL + 1];
#pragma unroll
        for (int l = 0; l <= NL; ++l) so[l] = sd[l] = c1[l] = c0[l] = mk(0, 0, 0), stm[l] = 0.0f;
        uint32_t shm = 0;          // shadow rays in flight (bit per light)
        bool ext = false, fin = false;
        const uint32_t col = s % width, row = P.shard_index + P.shard_count * (s / width);
        float* px = P.fb + 3 * ((size_t)col + (size_t)width * row);
        if (live) {
            g = glb<gu32>(P.rng_g)[s];
            rng.c = glb<gu32>(P.rng_c)[s];
            depth = glb<gu32>(P.depth)[s];
            k = glb<gu32>(P.sample_k)[s];
            kst = k;
            if (!(st & ST_REGEN)) {
                thr = ld3g(P.thr, s), rad = ld3g(P.rad, s);
                o = ld3g(P.ray_o, s), d = ld3g(P.ray_d, s);
                ext = true;
                kst = k + 1;
            }
            gf32* pxg = glb<gf32>(px);
            acc = mk(pxg[0], pxg[1], pxg[2]);
            rng.load(ring);
        }
        uint32_t nseg = 0, nsh = 0, nrej = 0;
        // Image::addPixel of a finished sample (Src/renderer.cpp:57-75)
        auto finish = [&](v3 r0) {
            const v3 r = r0 / 1.0f;
            if (__builtin_isnan(r.x) || __builtin_isnan(r.y) || __builtin_isnan(r.z) || __builtin_isinf(r.x) ||
                __builtin_isinf(r.y) || __builtin_isinf(r.z) || r.x < 0.0f || r.y < 0.0f || r.z < 0.0f) {
                ++nrej;
            } else {
                acc = acc + r;
            }
            ++k;
            if (k >= spp) st = ST_DONE;
        };
        // jitter draws + PinholeCamera::sampleRay for the next sample (Src/renderer.cpp:44-50)
        auto start_sample = [&]() {
            const float u = div_w(P, (float)(int)col + rng.next());
            const float v = div_h(P, (float)(int)row + rng.next());
            camera_ray(P, u, v, o, d);
            thr = mk(1, 1, 1), rad = mk(0, 0, 0);
            depth = 0;
            ext = true;
            ++kst;
        };
        // add the resolved NEE of the last shaded segment (GI: rad += thr * directL;
        // Direct: L += L_light per light) and finish its sample if it ended there
        auto resolve = [&](uint32_t occ) {
            if (!shm) return;
            v3& tgt = fin ? rad_fin : rad;
            if (INTEG == XRT_INTEGRATOR_DIRECT) {
#pragma unroll
                for (int l = 0; l < NL; ++l)
                    if ((shm >> l) & 1u) tgt = tgt + (((occ >> l) & 1u) ? c0[l] : c1[l]);
            } else if constexpr (kFold) {
                tgt = tgt + ((occ & 1u) ? mk(zdecode(c0z & 3u), zdecode((c0z >> 2) & 3u), zdecode(c0z >> 4)) : c1[0]);
            } else {
                v3 directL = mk(0, 0, 0);
#pragma unroll
                for (int l = 0; l < NL; ++l)
                    if ((shm >> l) & 1u) {
                        const v3 L_light = mk(0, 0, 0) + (((occ >> l) & 1u) ? c0[l] : c1[l]);
                        directL = directL + L_light;
                    }
                tgt = tgt + thr_nee * directL;
            }
            shm = 0;
            if (fin) {
                fin = false;
                finish(rad_fin);
            }
        };
        // a slot that starts a sample at the launch's first segment draws its jitter from
        // the words loaded above; later segments start samples at their end (start_sample
        // below), so no draw precedes the trace inside the loop
        if (live && !(st & ST_DONE) && g - rng.c >= (uint32_t)NW && (st & ST_REGEN)) {
            st &= ~ST_REGEN;
            start_sample();
        }
        __builtin_amdgcn_s_waitcnt(0);   // prologue loads done: the loop waits only on its own prefetches
        bool pf_pending = false;   // BVH: words in pf[]
        for (uint32_t vis = 0; vis < visits; ++vis) {
            const bool act = live && !(st & ST_DONE) && g - rng.c >= (uint32_t)NW;
            if (!__ballot(act || shm)) break;
            const bool ext_now = act && ext;
            // a sample's camera ray (depth 0) is tested against its pixel's camera list
            // (k_camlist, spec.hip: the triangles a camera ray of the pixel can hit, or the one
            // every such ray hits first) instead of taking part in the trace
            const bool cam = XRT_MERGED_CAMLIST && !BVH && P.camlist && ext_now && depth == 0;
            uint4 cl = make_uint4(0u, 0u, 0xffffffffu, 0u);
            if (cam) cl = P.camlist[s];   // used after the trace: its latency hides behind it
            unsigned long long best;
            uint32_t occ;
            if constexpr (BVH) {
                merged_trace<NL, true>(SO, L, W, lane, ext_now, o, d, shm, so, sd, stm, best, occ);
                deep_pass<NL, uint16_t>(P, top, ntop, stk, W, lane, root, ext_now, o, d, shm, so, sd, stm, best, occ);
            } else if constexpr (!LANE) {
                merged_trace<NL>(SO, L, W, lane, ext_now && !cam, o, d, shm, so, sd, stm, best, occ);
            } else {
                group_trace<NL, G>(P.n_objs, L, lplane, lane, ext_now && !cam, o, d, shm, so, sd, stm, best, occ);
            }
            if (cam) best = camlist_closest(L, cl, o, d);
            resolve(occ);
            if (BVH ? pf_pending : vis > 0) rng.take();   // the words prefetched at the end of the previous segment
            if (ext_now) {
                ++nseg;
                int hk = -1, obj = -1;
                float ht = kINF, hu = 0.0f, hv = 0.0f;
                if (best != ~0ull) {
                    hk = (int)(uint32_t)best;
                    const f4 ta = tri_rec(3 * hk);
                    (void)ray_tri(o, d, xyz(ta), xyz(tri_rec(3 * hk + 1)), xyz(tri_rec(3 * hk + 2)), ht, hu, hv);
                    obj = __float_as_int(ta.w);
                }
                v3 pos = mk(0, 0, 0), ng = mk(0, 0, 0);
                if (hk >= 0) pos = ray_at(o, d, ht), ng = tri_ng_at(hk);
                bool ended = false, alive = false;
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    // DirectIntegrator::integrate (Src/integrator.h:82-119)
                    if (obj < 0) {
                        rad = mk((float)0.18, (float)0.18, (float)0.18);
                        ended = true;
                    } else if (L.obj[obj].light >= 0) {
                        rad = light_Le(L.light[L.obj[obj].light], tri_ns_at(hk, hu, hv), d);
                        ended = true;
                    } else {
                        alive = true;
                    }
                } else {
                    // GIIntegrator::integrate loop body (Src/integrator.h:214-284)
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
                            if (depth == 0)
                                rad = rad + thr * light_Le(L.light[L.obj[obj].light], tri_ns_at(hk, hu, hv), d);
                            alive = false, ended = true;
                        }
                    }
                }
                if (alive) {
                    // next-event estimation: light samples now, shadow rays traced with the
                    // next trace of the wave
                    const DObj& ob = L.obj[obj];
                    const v3 fr = ob.material == 1 ? mk(ob.fr[0], ob.fr[1], ob.fr[2]) : mk(0, 0, 0);
#pragma unroll
                    for (int l = 0; l < NL; ++l) {
                        v3 wi = mk(0, 0, 0);
                        float tmax = 0.0f, pdf = 0.0f;
                        const v3 Lv = light_sample(L.light[l], pos, wi, pdf, tmax, rng);
                        if (pdf != 0.0f) {
                            ++nsh;
                            shm |= 1u << l;
                            const float bias = 0.01f;
                            so[l] = pos + ng * bias, sd[l] = wi, stm[l] = tmax - bias;
                            const float cosv = smax(0.0f, dot(ng, wi));
                            // vis * fr * L * cos / pdf (Src/integrator.h:250-262) for vis = 1, 0.
                            // fr * 1 == fr; for vis = 0 the product is +-0 or NaN and pdf is
                            // > 0 (or NaN), so the quotient is that product (NaN for a NaN pdf)
                            c1[l] = ((fr * Lv) * cosv) / pdf;
                            const v3 z = ((fr * 0.0f) * Lv) * cosv;
                            c0[l] = pdf == pdf ? z : mk(pdf, pdf, pdf);
                            if constexpr (kFold) {   // GIIntegrator: rad += thr * directL (resolve)
                                const v3 zero = mk(0, 0, 0);
                                c1[0] = thr * (zero + (zero + c1[0]));
                                const v3 w = thr * (zero + (zero + c0[0]));
                                c0z = zcode(w.x) | (zcode(w.y) << 2) | (zcode(w.z) << 4);
                            }
                        }
                    }
                    if (INTEG == XRT_INTEGRATOR_DIRECT) {
                        ended = true;
                    } else {
                        if (!kFold && shm) thr_nee = thr;
                        else rad = rad + thr * mk(0.0f, 0.0f, 0.0f);   // no shadow ray: directL = 0
                        v3 nd = mk(0, 0, 0);
                        const bool lamb = ob.material == 1;
                        if (lamb) {
                            v3 dpdu, dpdv;
                            onb(tri_ns_at(hk, hu, hv), dpdu, dpdv);
                            nd = lambert_sample_f(ng, dpdu, dpdv, rng);
                        }
                        const float cosv = smax(0.0f, dot(nd, ng));
                        // (fr * cos) / pdf, pdf = 1 / (2 PI) for Lambert (Src/material.h:60-73), else 1
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
                if (ended) {
                    ext = false;
                    if (shm) {
                        rad_fin = rad;
                        fin = true;
                    } else {
                        finish(rad);
                    }
                    if (kst < spp) start_sample();
                }
            }
            rng.prefetch(ring);   // unconditional; first read by take() after the next trace
            pf_pending = true;
        }
        // drain: trace the shadow rays still in flight, so no NEE state crosses launches
        if (__ballot(shm != 0)) {
            unsigned long long best;
            uint32_t occ;
            if constexpr (BVH) {
                merged_trace<NL, true>(SO, L, W, lane, false, o, d, shm, so, sd, stm, best, occ);
                deep_pass<NL, uint16_t>(P, top, ntop, stk, W, lane, root, false, o, d, shm, so, sd, stm, best, occ);
            } else if constexpr (!LANE) {
                merged_trace<NL>(SO, L, W, lane, false, o, d, shm, so, sd, stm, best, occ);
            } else {
                group_trace<NL, G>(P.n_objs, L, lplane, lane, false, o, d, shm, so, sd, stm, best, occ);
            }
            resolve(occ);
        }
        bool want_req = false;
        if (live && lead) {
            px[0] = acc.x, px[1] = acc.y, px[2] = acc.z;
            want_req = !(st & ST_DONE) && g - rng.c < P.rng_keep;
            P.state[s] = st;
            if (!(st & (ST_DONE | ST_REGEN))) {
                P.depth[s] = depth;
                P.thr[s] = pk(thr);
                P.rad[s] = pk(rad);
                P.ray_o[s] = pk(o);
                P.ray_d[s] = pk(d);
            }
            P.sample_k[s] = k;
            P.rng_c[s] = rng.c;
            if (nseg) P.c_seg[s] += nseg;
            if (nsh) P.c_shadow[s] += nsh;
            if (nrej) P.c_rej[s] += nrej;
        }
        wave_append(live && lead && !(st & ST_DONE), s, out + it.p * P.part_cap, out_count + it.p, lane);
        wave_refill(P, want_req, s, g, lane, reinterpret_cast<uint32_t*>(&W));
    }
}

// CLEAR: also clear the slot's ST_RNGREQ (the wavefront / k_step schedules, whose kernels
// test the flag; the merged kernel clears it itself when it next loads the slot).
template <bool CLEAR>
__global__ __launch_bounds__(kBlock) void k_refill_merged(KParams P, const uint32_t* __restrict__ req,
                                                          const uint32_t* __restrict__ count, uint32_t* zero_count) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kBlock / 64][2][kMT];
    zero_parts(P, zero_count);
    const PartIter it = part_iter(P, count, kBlock / 64);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t i = it.first + wv;
    if (i >= it.n) return;
    const uint32_t* rq = req + it.p * P.part_cap;
    uint32_t s = rq[i];
    uint32_t g = glb<gu32>(P.rng_g)[s];
    store_block(load_block(P.ring + (size_t)s * kRing, g, lane), lane, stage[wv][0]);
    for (int buf = 0;; buf ^= 1) {
        // Double-buffered: the next request's old block is in flight (in registers) while
        // this one twists out of LDS.
        const uint32_t in = i + it.stride;
        const bool more = in < it.n;
        uint32_t sn = s, gn = g;
        Staged nx;
        if (more) {
            sn = rq[in];
            gn = glb<gu32>(P.rng_g)[sn];
            nx = load_block(P.ring + (size_t)sn * kRing, gn, lane);
        }
        twist_block(P.ring + (size_t)s * kRing, g, lane, stage[wv][buf]);
        if (lane == 0) {
            P.rng_g[s] = g + kMT;
            if (CLEAR) P.state[s] &= ~ST_RNGREQ;
        }
        if (!more) break;
        store_block(nx, lane, stage[wv][buf ^ 1]);
        s = sn, g = gn, i = in;
    }
}

hipError_t launch_refill_merged(const KParams& P, const uint32_t* count, uint32_t* zero_count, hipStream_t st) {
    // 16384 blocks (64 Ki waves) measured best on C2: 2048 7.7 ms, 4096 6.9, 8192 6.6, 16384 6.5
    // per frame (tools/refill_sweep.sh).
    const uint32_t per = std::max<uint32_t>(1u, std::min<uint32_t>((P.part_cap + 3) / 4, 16384u / P.n_part));
    hipLaunchKernelGGL(k_refill_merged<false>, dim3(P.n_part * per), dim3(kBlock), 0, st, P, P.req, count,
                       zero_count);
    return hipGetLastError();
}

hipError_t launch_refill(const KParams& P, const uint32_t* count, uint32_t* zero_count, hipStream_t st) {
    const uint32_t per = std::max<uint32_t>(1u, std::min<uint32_t>((P.part_cap + 3) / 4, 16384u / P.n_part));
    hipLaunchKernelGGL(k_refill_merged<true>, dim3(P.n_part * per), dim3(kBlock), 0, st, P, P.req, count, zero_count);
    return hipGetLastError();
}

// ------------------------------------------------------------------- host side ----
bool use_step_merged(const KParams& P) {
    return P.scene_kind == SCN_TRI && P.small_tri && P.det_bounded && P.n_objs <= kMergedMaxObjs && P.n_lights <= kMaxLights &&
           (P.integrator == XRT_INTEGRATOR_DIRECT || (P.integrator == XRT_INTEGRATOR_GI && P.max_depth > 0)) &&
           !exp_env("XRT_NO_MERGED") && step_merged_lds_bytes(P) <= kStepLds;
}

// The merged schedule for two-level scenes (C4): k_step_merged<..., BVH = true>.  The small
// objects must be traceable by pair passes (KParams::sstep: at most kMergedMaxObjs objects,
// det_bounded), the 4-wide BVH's node indices fit the 16-bit quad stacks, one or two area
// lights (the kernel's two pair-pass scratch buffers per wave must fit kStepLds).
bool use_step_bvh(const KParams& P) {
    return P.scene_kind == SCN_TRI && P.two_level && P.sstep && P.det_bounded && P.bvh4 && P.bvh_node &&
           P.bvh4_nodes <= 0x10000 && P.bvh4_stack > 0 && P.bvh4_stack <= kBvh4Stack && P.n_lights >= 1 &&
           P.n_lights <= 2 &&
           (P.integrator == XRT_INTEGRATOR_DIRECT || (P.integrator == XRT_INTEGRATOR_GI && P.max_depth > 0)) &&
           !exp_env("XRT_NO_STEP_BVH") && step_merged_lds_bytes(P) <= kStepLds;
}

uint32_t step_merged_draws(const KParams& P) { return 6u + 2u * (uint32_t)P.n_lights; }

static size_t merged_wave_bytes(int n_lights) {
    switch (n_lights) {
        case 0: return sizeof(MergedWave<0>);
        case 1: return sizeof(MergedWave<1>);
        case 2: return sizeof(MergedWave<2>);
        case 3: return sizeof(MergedWave<3>);
        default: return sizeof(MergedWave<4>);
    }
}

size_t step_merged_lds_bytes(const KParams& P) {
    const size_t w = merged_wave_bytes(P.n_lights);
    if (P.two_level) return bvh_step_layout(P, (uint32_t)w).total;
    return merged_wave_off(P, step_layout(P)) + (kBlock / 64) * w;
}

void build_step_objs(const DObjBox* boxes, const DObjPlane* planes, int n, StepObjs& SO) {
    std::memset(&SO, 0, sizeof(SO));
    SO.n = n;
    for (int i = 0; i < n; ++i) {
        StepObj& o = SO.o[i];
        o.axis = planes[i].axis;
        o.plane = planes[i].c;
        for (int q = 0; q < 3; ++q) o.bmin[q] = boxes[i].bmin[q], o.bmax[q] = boxes[i].bmax[q];
        o.first = boxes[i].first;
        o.count = (uint32_t)(boxes[i].count_occ & 0x7fffffff);
        o.occluder = boxes[i].count_occ < 0 ? 1u : 0u;
        // ceil(2^32 / count): floor(j * magic / 2^32) = j / count for j * count < 2^32
        o.magic = o.count > 1 ? (uint32_t)(((1ull << 32) + o.count - 1) / o.count) : 0u;
    }
}

template <int INTEG, int SPW, int G, bool LANE, bool BVH = false, int WV = 0>
static void launch_merged_i(const KParams& P, const KParams* dP, const StepObjs& SO, const uint32_t* list,
                            const uint32_t* count, uint32_t* out, uint32_t* out_count, uint32_t* zero,
                            uint32_t* req_count, uint32_t visits, uint32_t part_live, size_t lds, hipStream_t st) {
    // one block per per_block live entries of the fullest partition (part_iter strides over
    // any remainder, so an upper bound on the live count is all the grid needs)
    const uint32_t per_block = (kBlock / 64) * SPW;
    const uint32_t blocks = P.n_part * ((std::min(part_live, P.part_cap) + per_block - 1) / per_block);
#define XRT_LAUNCH_MERGED(NLV)                                                                                       \
    hipLaunchKernelGGL((k_step_merged<INTEG, NLV, SPW, G, LANE, BVH, WV>), dim3(blocks), dim3(kBlock), lds, st, dP, SO, list, \
                       count, out, out_count, zero, req_count, visits)
    if constexpr (BVH) {   // use_step_bvh: 1 or 2 lights
        if (P.n_lights == 1) XRT_LAUNCH_MERGED(1);
        else XRT_LAUNCH_MERGED(2);
    } else {
        switch (P.n_lights) {
            case 0: XRT_LAUNCH_MERGED(0); break;
            case 1: XRT_LAUNCH_MERGED(1); break;
            case 2: XRT_LAUNCH_MERGED(2); break;
            case 3: XRT_LAUNCH_MERGED(3); break;
            default: XRT_LAUNCH_MERGED(4); break;
        }
    }
#undef XRT_LAUNCH_MERGED
}

// slots per wave for a shard of `live` slots
// (xrt_render_params.slots_per_wave overrides it; results do not depend on it)
uint32_t step_merged_spw(const KParams& P, uint64_t live) {
    const bool group = P.n_tris <= 64 && !(P.rflags & XRT_FLAG_NO_GROUP);   // 4 slots per wave: group traces only
    if (P.spw_req == 4) return group ? 4u : 16u;
    if (P.spw_req == 8) return group ? 8u : 16u;
    if (P.spw_req == 16 || P.spw_req == 32 || P.spw_req == 64) return P.spw_req;
    // two-level scenes (C4, tools/spw_sweep.sh): fewer slots per wave leave more
    // quads per deep ray and more lanes per pair pass, which pays once the GPU is not full:
    // full waves above kBvhLive64 live slots, 32 above kBvhLive32, then 16
    if (P.two_level) return live >= kBvhLive64 ? 64u : live >= kBvhLive32 ? 32u : 16u;
    // measured on C2 (tools/shard_sim.py): full waves down to ~160k live
    // slots, 32 slots per wave down to ~90k, 16 (4 lanes per slot) down to kMergedLive16,
    // then 4 (16 lanes per slot: the tail of a small shard, where a visit's latency, not
    // issue, sets the time)
    if (live >= kMergedLive64) return 64;
    if (live >= kMergedLive32) return 32;
    if (!group) return 16u;
    if (live < kMergedLive16) return 4u;
    return live < XRT_LIVE8 ? 8u : 16u;
}

// lanes that share one slot's traces at `spw` slots per wave (1 = pair passes over the wave)
uint32_t step_merged_group(const KParams& P, uint32_t spw) {
    const bool group = P.n_tris <= 64 && !(P.rflags & XRT_FLAG_NO_GROUP);   // group trace: 64-bit triangle masks
    return spw < 64 && group ? 64u / spw : 1u;
}

template <int INTEG>
static void launch_merged_spw(const KParams& P, const KParams* dP, const StepObjs& SO, const uint32_t* list,
                              const uint32_t* count, uint32_t* out, uint32_t* out_count, uint32_t* zero,
                              uint32_t* req_count, uint32_t visits, uint64_t live, uint32_t part_live, size_t lds,
                              hipStream_t st) {
    const bool group = P.n_tris <= 64 && !(P.rflags & XRT_FLAG_NO_GROUP);   // group trace: 64-bit triangle masks
    const bool lane64 = group && exp_env("XRT_LANE_TRACE");   // experiment: per-lane traces, full waves
    if (P.two_level) {   // use_step_bvh (never group traces: n_tris > 64)
#define XRT_BVH_CASE(SPWV) \
    launch_merged_i<INTEG, SPWV, 1, false, true>(P, dP, *P.sstep, list, count, out, out_count, zero, req_count, visits, \
                                                 part_live, lds, st)
        switch (step_merged_spw(P, live)) {
            case 64: XRT_BVH_CASE(64); break;
            case 32: XRT_BVH_CASE(32); break;
            default:
                // below XRT_BVH_LOW_LIVE live slots (a frame's or a row shard's tail) the
                // XRT_BVH_LOW_WAVES build: more registers per wave, fewer spills
                if (live < XRT_BVH_LOW_LIVE)
                    launch_merged_i<INTEG, 16, 1, false, true, XRT_BVH_LOW_WAVES>(
                        P, dP, *P.sstep, list, count, out, out_count, zero, req_count, visits, part_live, lds, st);
                else
                    XRT_BVH_CASE(16);
                break;
        }
#undef XRT_BVH_CASE
        return;
    }
#define XRT_MERGED_CASE(SPWV, GV, LV) \
    launch_merged_i<INTEG, SPWV, GV, LV>(P, dP, SO, list, count, out, out_count, zero, req_count, visits, part_live, lds, st)
    switch (step_merged_spw(P, live)) {
        case 64: if (lane64) XRT_MERGED_CASE(64, 1, true); else XRT_MERGED_CASE(64, 1, false); break;
        case 32: if (group) XRT_MERGED_CASE(32, 2, true); else XRT_MERGED_CASE(32, 1, false); break;
        case 4: XRT_MERGED_CASE(4, 16, true); break;   // only with group traces (step_merged_spw)
        case 8: XRT_MERGED_CASE(8, 8, true); break;    // only with group traces (step_merged_spw)
        default: if (group) XRT_MERGED_CASE(16, 4, true); else XRT_MERGED_CASE(16, 1, false); break;
    }
#undef XRT_MERGED_CASE
}

hipError_t launch_step_merged(const KParams& P, const KParams* dP, const StepObjs& SO, const uint32_t* list,
                              const uint32_t* count, uint32_t* out, uint32_t* out_count, uint32_t* zero,
                              uint32_t* req_count, uint32_t visits, uint64_t live, uint32_t live_part_max,
                              hipStream_t st) {
    const size_t lds = step_merged_lds_bytes(P);
    if (P.integrator == XRT_INTEGRATOR_DIRECT)
        launch_merged_spw<XRT_INTEGRATOR_DIRECT>(P, dP, SO, list, count, out, out_count, zero, req_count, visits,
                                                 live, live_part_max, lds, st);
    else
        launch_merged_spw<XRT_INTEGRATOR_GI>(P, dP, SO, list, count, out, out_count, zero, req_count, visits, live,
                                             live_part_max, lds, st);
    return hipGetLastError();
}

}  // namespace xrt
