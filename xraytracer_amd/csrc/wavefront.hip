// wavefront.hip — gfx950 kernels of the wavefront path tracer.
//
// One path slot per pixel of the shard.  Each iteration runs two passes over a compacted
// slot list:
//   k_shade : per slot — resolve last bounce's NEE (shadow results), shade the hit record
//             (RR, emitter, NEE light samples -> shadow rays, Lambert BSDF sample ->
//             extension ray), finalize a finished sample into the framebuffer and
//             regenerate the pixel's next camera ray; ballot/prefix-sum compaction of the
//             slots that still have rays to trace.
//   k_trace : closest-hit for extension rays and any-hit for shadow rays over the linear
//             primitive array, staged through LDS in tiles shared by the block's rays.
// Per-pixel RNG is an exact restatement of the reference's std::mt19937 stream; a pixel's
// samples run in order (sample k+1 starts in the same k_shade call that finalises k), so
// every pixel consumes its stream exactly as NormalRenderer::doRender does
// (Src/renderer.cpp:29-81).
#include <hip/hip_runtime.h>

#include "bvh.h"
#include "lscene.h"
#include "path_common.h"

// minimum waves per SIMD the wavefront kernels are compiled for (launch bounds; experiment
// builds override them)

namespace xrt {


// ==================================================================== k_seed ====
// mt19937::seed(j + width*i) for every slot (Src/renderer.cpp:35-36).  The recurrence is
// serial per pixel, so each lane runs one pixel's recurrence and the wave writes the words
// out through an LDS transpose (64 pixels x 64 words, padded row) as coalesced 256-B rows.
__global__ __launch_bounds__(kBlock) void k_seed(KParams P, uint32_t* list, uint32_t* count, uint32_t* count_other,
                                                  uint32_t* req_count) {
    __shared__ uint32_t lds[4][64][65];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t base = (blockIdx.x * kBlock) + wv * 64;
    const uint32_t s = base + lane;
    const bool valid = s < P.n_slots;
    uint32_t row = 0, col = 0;
    if (valid) {
        col = s % P.width;
        row = P.shard_index + P.shard_count * (s / P.width);
    }
    uint32_t x = col + P.width * row;  // seed j + width * i
    for (uint32_t q = 0; q < kMT; q += 64) {
        for (uint32_t j = 0; j < 64; ++j) {
            const uint32_t i = q + j;
            if (i > 0 && i < kMT) x = 1812433253u * (x ^ (x >> 30)) + i;
            lds[wv][lane][j] = x;
        }
        wave_sync();
        for (uint32_t r = 0; r < 64; ++r) {
            const uint32_t sl = base + r;
            if (sl < P.n_slots && q + lane < kMT) P.ring[(size_t)sl * kRing + q + lane] = lds[wv][r][lane];
        }
        wave_sync();
    }
    if (valid) {
        P.rng_c[s] = kMT;   // cursor: next output is x[624]
        P.rng_g[s] = kMT;   // generated: x[0..623]
        P.state[s] = ST_REGEN | ST_RNGREQ;   // first twist by the k_refill right after
        P.req[s] = s;   // partition p = s / part_cap starts at p * part_cap: identity
        P.sample_k[s] = 0;
        P.depth[s] = 0;
        P.occ[s] = 0;
        P.c_seg[s] = 0;
        P.c_shadow[s] = 0;
        P.c_rej[s] = 0;
        P.c_stall[s] = 0;
        list[s] = s;
    }
    if (blockIdx.x == 0) {
        for (uint32_t p = threadIdx.x; p < P.n_part; p += kBlock) {
            const uint32_t lo = p * P.part_cap;
            const uint32_t c = lo < P.n_slots ? min(P.part_cap, P.n_slots - lo) : 0u;
            count[p] = c;
            count_other[p] = 0;
            req_count[p] = c;
            req_count[kMaxParts + p] = 0;
        }
    }
}

// =================================================================== k_trace ====
template <int SCN, int NL>
__global__ __launch_bounds__(kBlock) void k_trace(KParams P, const uint32_t* __restrict__ list,
                                                   const uint32_t* __restrict__ count, uint32_t* zero_count) {
    __shared__ f4 lds_tri[SCN == SCN_SPHERE ? 1 : 3 * kTriTile];
    __shared__ f4 lds_sph[SCN == SCN_TRI ? 1 : kSphTile];
    __shared__ int lds_sobj[SCN == SCN_TRI ? 1 : kSphTile];
    zero_parts(P, zero_count);
    const PartIter it = part_iter(P, count, kBlock);
    const int tid = threadIdx.x;
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        const bool valid = i < it.n;
        const uint32_t s = valid ? list[it.p * P.part_cap + i] : 0;
        const uint32_t st = valid ? P.state[s] : 0;
        const bool want = (st & ST_RAY) != 0;
        const uint32_t smask = (st >> ST_SHADOW_SHIFT) & ((1u << NL) - 1u);
        v3 o = mk(0, 0, 0), d = mk(0, 0, 0);
        if (want) {
            o = xyz(P.ray_o[s]);
            d = xyz(P.ray_d[s]);
        }
        v3 so[NL], sd[NL];
        float stmax[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            so[l] = mk(0, 0, 0), sd[l] = mk(0, 0, 0), stmax[l] = 0.0f;
            if (smask & (1u << l)) {
                const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                so[l] = xyz(a);
                stmax[l] = a.w;
                sd[l] = xyz(P.sh_d[(size_t)l * P.n_slots + s]);
            }
        }
        uint32_t occ = 0;
        float best_t = kINF, bu = 0.0f, bv = 0.0f;
        int best = -1;
        // mixed scenes: which primitive last wrote SurfaceInfo (position/ng/ns) and which
        // triangle last wrote dpdu/dpdv (spheres and boxes leave them untouched)
        int surf = -1, dp = -1;
        float surf_t = 0.0f, surf_u = 0.0f, surf_v = 0.0f, dp_u = 0.0f, dp_v = 0.0f, t1 = kINF;

        for (int sg = 0; sg < P.n_segs; ++sg) {
            const DSeg seg = P.segs[sg];
            if (SCN != SCN_SPHERE && seg.kind == SEG_TRI) {
                for (int tb = seg.first; tb < seg.first + seg.count; tb += kTriTile) {
                    const int nt = min(kTriTile, seg.first + seg.count - tb);
                    __syncthreads();
                    for (int q = tid; q < 3 * nt; q += kBlock) lds_tri[q] = P.tri[3 * (size_t)tb + q];
                    __syncthreads();
                    for (int k = 0; k < nt; ++k) {
                        const f4 A = lds_tri[3 * k], B = lds_tri[3 * k + 1], Cc = lds_tri[3 * k + 2];
                        const v3 v0 = xyz(A), e1 = xyz(B), e2 = xyz(Cc);
                        if (want) {
                            float t, u, v;
                            if (ray_tri(o, d, v0, e1, e2, t, u, v) && t < best_t) {
                                best_t = t, bu = u, bv = v, best = tb + k;
                                if (SCN == SCN_MIXED) surf = best, surf_t = t, surf_u = u, surf_v = v, dp = best, dp_u = u, dp_v = v;
                            }
                        }
                        if (B.w != 0.0f) {  // occluder (object without an area light)
#pragma unroll
                            for (int l = 0; l < NL; ++l) {
                                if ((smask & (1u << l)) && !(occ & (1u << l))) {
                                    float t, u, v;
                                    if (ray_tri(so[l], sd[l], v0, e1, e2, t, u, v) && t < stmax[l]) occ |= 1u << l;
                                }
                            }
                        }
                    }
                }
            } else if (SCN != SCN_TRI && seg.kind == SEG_SPHERE) {
                for (int tb = seg.first; tb < seg.first + seg.count; tb += kSphTile) {
                    const int nt = min(kSphTile, seg.first + seg.count - tb);
                    __syncthreads();
                    for (int q = tid; q < nt; q += kBlock) {
                        lds_sph[q] = P.sph[tb + q];
                        lds_sobj[q] = P.sph_obj[tb + q];
                    }
                    __syncthreads();
                    for (int k = 0; k < nt; ++k) {
                        const f4 S = lds_sph[k];
                        const v3 c = xyz(S);
                        if (want) {
                            float t;
                            if (sphere_hit(o, d, c, S.w, t) && t < best_t) {
                                best_t = t, bu = 0.0f, bv = 0.0f, best = (1 << 28) | (tb + k);
                                if (SCN == SCN_MIXED) surf = best, surf_t = t;
                            }
                        }
                        if (lds_sobj[k] & (1 << 30)) {
#pragma unroll
                            for (int l = 0; l < NL; ++l) {
                                if ((smask & (1u << l)) && !(occ & (1u << l))) {
                                    float t;
                                    if (sphere_hit(so[l], sd[l], c, S.w, t) && t < stmax[l]) occ |= 1u << l;
                                }
                            }
                        }
                    }
                }
            } else if (SCN == SCN_MIXED && seg.kind == SEG_BOX) {
                for (int b = seg.first; b < seg.first + seg.count; ++b) {
                    const v3 pmin = xyz(P.box[2 * b]), pmax = xyz(P.box[2 * b + 1]);
                    if (want) {
                        float t0, tt1;
                        if (box_hit(o, d, pmin, pmax, t0, tt1)) best_t = t0, t1 = tt1, best = (2 << 28) | b;
                    }
                    // BoxMesh::occluded returns true unconditionally (Src/primitive.h:266-268)
                    occ |= smask;
                }
            }
        }
        if (valid) {
            if (want) {
                P.hit[s] = make_float4(best_t, bu, bv, __int_as_float(best));
                if (SCN == SCN_MIXED) {
                    P.hit2[s] = make_float4(t1, __int_as_float(surf), __int_as_float(dp), surf_t);
                    P.hit3[s] = make_float4(surf_u, surf_v, dp_u, dp_v);
                }
            }
            if (smask) P.occ[s] = occ;
        }
    }
}

// ====================================================================== BVH trace ====
// Large triangle scenes (C4): closest hit and any-hit through the host-built BVH (bvh.h).
// Exactness: every node box is padded beyond the float error of a Moller-Trumbore hit, a
// child is entered when its box overlaps [0, best t] (inclusive: a later triangle at the
// same t with a lower index must still be found), and the closest hit is the
// lexicographic minimum of (t, original index) — the reference's in-order strict
// `t < best` scan over all triangles (Src/scene.cpp:190-200, primitive.cpp:83-131).
// Shadow rays test occluder triangles only and stop at the first hit (Scene::occluded).
// One ray per lane; the traversal stack lives in LDS (kBvhStack entries per thread).

template <bool ANY>
__device__ __forceinline__ bool bvh_leaf(const KParams& P, int first, int count, v3 o, v3 d, float tmax, float& bt,
                                         float& bu, float& bv, int& bk) {
    for (int i = first; i < first + count; ++i) {
        const f4 A = P.bvh_tri[3 * i], B = P.bvh_tri[3 * i + 1], C = P.bvh_tri[3 * i + 2];
        if (ANY && B.w == 0.0f) continue;   // area-light objects never occlude
        float t, u, v;
        if (!ray_tri(o, d, xyz(A), xyz(B), xyz(C), t, u, v)) continue;
        if (ANY) {
            if (t < tmax) return true;
        } else {
            const int k = __float_as_int(C.w);
            if (t < bt || (t == bt && k < bk)) bt = t, bu = u, bv = v, bk = k;
        }
    }
    return false;
}

// ANY: returns occluded; else fills (bt, bu, bv, bk) (bk = -1: miss).  Closest-hit rays
// descend into the nearer child first (entry distance) and stack the farther one, so the
// best t shrinks early and culls more of the tree; the result does not depend on the
// order (lexicographic (t, index) minimum over every triangle whose box overlaps).
// top: the first ntop nodes (the breadth-first top of the tree, host/bvh.cpp) in LDS.
template <bool ANY, typename SE>
__device__ bool bvh_trace(const KParams& P, const f4* top, int ntop, SE* stk, v3 o, v3 d, float tmax, float& bt,
                          float& bu, float& bv, int& bk) {
    const v3 inv = rcp3(d);
    int sp = 0;
    int node = 0;
    while (true) {
        f4 n0, n1, n2, n3;
        if (node < ntop) {
            const f4* N = top + 4 * node;
            n0 = N[0], n1 = N[1], n2 = N[2], n3 = N[3];
        } else {
            const f4* N = P.bvh_node + 4 * (size_t)node;
            n0 = N[0], n1 = N[1], n2 = N[2], n3 = N[3];
        }
        const float lim = ANY ? tmax : bt;
        const int lcount = __float_as_int(n1.w), rcount = __float_as_int(n3.w);
        const float el = lcount >= 0 ? bvh_enter(n0, n1, o, inv, lim) : __builtin_inff();
        const float er = rcount >= 0 ? bvh_enter(n2, n3, o, inv, lim) : __builtin_inff();
        const bool hl = el != __builtin_inff(), hr = er != __builtin_inff();
        // leaves first (either order gives the same result)
        if (hl && lcount > 0 && bvh_leaf<ANY>(P, __float_as_int(n0.w), lcount, o, d, tmax, bt, bu, bv, bk)) return true;
        if (hr && rcount > 0 && bvh_leaf<ANY>(P, __float_as_int(n2.w), rcount, o, d, tmax, bt, bu, bv, bk)) return true;
        const bool il = hl && lcount == 0, ir = hr && rcount == 0;
        int next = -1;
        if (il && ir) {
            const bool lfirst = ANY || el <= er;
            next = __float_as_int(lfirst ? n0.w : n2.w);
            stk[(sp++) * kBlock] = (SE)__float_as_int(lfirst ? n2.w : n0.w);
        } else if (il) {
            next = __float_as_int(n0.w);
        } else if (ir) {
            next = __float_as_int(n2.w);
        }
        if (next >= 0) {
            node = next;
        } else {
            if (sp == 0) break;
            node = (int)stk[(--sp) * kBlock];
        }
    }
    return false;
}

template <int NL, typename SE>
__global__ __launch_bounds__(kBlock) void k_trace_bvh(KParams P, const uint32_t* __restrict__ list,
                                                       const uint32_t* __restrict__ count, uint32_t* zero_count) {
    // LDS: the top min(bvh_nodes, kBvhTopNodes) nodes, then P.bvh_stack * kBlock stack
    // entries of SE (sized to the tree)
    extern __shared__ uint32_t bvh_stack_lds[];
    const int tid = threadIdx.x;
    const int ntop = P.bvh_nodes < (int)kBvhTopNodes ? P.bvh_nodes : (int)kBvhTopNodes;
    f4* top = reinterpret_cast<f4*>(bvh_stack_lds);
    for (int q = tid; q < 4 * ntop; q += kBlock) top[q] = P.bvh_node[q];
    SE* stack = reinterpret_cast<SE*>(bvh_stack_lds + 16 * ntop);
    __syncthreads();
    zero_parts(P, zero_count);
    const PartIter it = part_iter(P, count, kBlock);
    SE* stk = stack + tid;
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        if (i >= it.n) continue;
        const uint32_t s = list[it.p * P.part_cap + i];
        const uint32_t st = P.state[s];
        const uint32_t smask = (st >> ST_SHADOW_SHIFT) & ((1u << NL) - 1u);
        if (st & ST_RAY) {
            float bt = kINF, bu = 0.0f, bv = 0.0f;
            int bk = -1;
            (void)bvh_trace<false, SE>(P, top, ntop, stk, xyz(P.ray_o[s]), xyz(P.ray_d[s]), kINF, bt, bu, bv, bk);
            P.hit[s] = make_float4(bt, bu, bv, __int_as_float(bk));
        }
        if (smask) {
            uint32_t occ = 0;
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                if (!(smask & (1u << l))) continue;
                const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                float bt = kINF, bu, bv;
                int bk = -1;
                if (bvh_trace<true, SE>(P, top, ntop, stk, xyz(a), xyz(P.sh_d[(size_t)l * P.n_slots + s]), a.w, bt, bu, bv, bk))
                    occ |= 1u << l;
            }
            P.occ[s] = occ;
        }
    }
}

// ============================================================ two-level trace ====
// Large triangle scenes with small objects beside the big meshes (C4: the Cornell walls and
// blocks around a 51,200-triangle sphere): one wave's rays mostly bounce between the small
// objects, but a single lane whose segment passes the big mesh makes the whole wave walk
// its BVH (k_trace_bvh: lane utilisation 0.12).  Phase A (k_trace_2a) scans the small
// objects as k_trace_small does (LDS, in iteration order, strict t < best: the
// lexicographic (t, index) minimum among them), then queues only the rays whose segment
// [0, best t] (any-hit: [0, tmax], if not yet occluded) overlaps the BVH root; phase B
// (k_trace_deep) walks the BVH for the queued rays alone — full waves of deep rays — and
// merges with the same (t, index) order (bvh_leaf).  The result is the one-level trace's.
__device__ __forceinline__ bool plane_away_w(v3 o, v3 d, const DObjPlane& pl) {   // step_tri.hip plane_away
    const float oa = pl.axis == 0 ? o.x : (pl.axis == 1 ? o.y : o.z);
    const float da = pl.axis == 0 ? d.x : (pl.axis == 1 ? d.y : d.z);
    return pl.axis >= 0 && (oa - pl.c) * da >= 0.0f;
}

template <int NL>
__global__ __launch_bounds__(kBlock) void k_trace_2a(KParams P, const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ count, uint32_t* zero_count) {
    extern __shared__ __attribute__((aligned(16))) f4 lds_2a[];
    f4* ltri = lds_2a;
    DObjBox* lbox = reinterpret_cast<DObjBox*>(lds_2a + 3 * P.n_stri);
    DObjPlane* lpl = reinterpret_cast<DObjPlane*>(lbox + P.n_sobj);
    zero_parts(P, zero_count);
    const int tid = threadIdx.x, lane = tid & 63;
    for (int q = tid; q < 3 * P.n_stri; q += kBlock) ltri[q] = P.stri[q];
    for (int q = tid; q < P.n_sobj; q += kBlock) lbox[q] = P.sbox[q], lpl[q] = P.splane[q];
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
        if (want) {
            o = xyz(P.ray_o[s]);
            d = xyz(P.ray_d[s]);
        }
        v3 so[NL], sd[NL];
        float stmax[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            so[l] = mk(0, 0, 0), sd[l] = mk(0, 0, 0), stmax[l] = 0.0f;
            if (smask & (1u << l)) {
                const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                so[l] = xyz(a);
                stmax[l] = a.w;
                sd[l] = xyz(P.sh_d[(size_t)l * P.n_slots + s]);
            }
        }
        const v3 inv = rcp3(d);
        uint32_t occ = 0;
        float best_t = kINF, bu = 0.0f, bv = 0.0f;
        int best = -1;
        for (int ob = 0; ob < P.n_sobj; ++ob) {
            const DObjBox B = lbox[ob];
            const DObjPlane pl = lpl[ob];
            const int cnt = B.count_occ & 0x7fffffff;
            const bool occluder = B.count_occ < 0;
            const bool ne = want && !plane_away_w(o, d, pl) && box_overlap(o, inv, B, best_t);
            uint32_t nsm = 0;
            if (occluder) {
#pragma unroll
                for (int l = 0; l < NL; ++l)
                    if ((smask & ~occ & (1u << l)) && !plane_away_w(so[l], sd[l], pl) &&
                        box_overlap(so[l], rcp3(sd[l]), B, stmax[l]))
                        nsm |= 1u << l;
            }
            if (__ballot(ne || nsm) == 0) continue;
            for (int k = B.first; k < B.first + cnt; ++k) {
                const v3 v0 = xyz(ltri[3 * k]), e1 = xyz(ltri[3 * k + 1]);
                const f4 E2 = ltri[3 * k + 2];
                const v3 e2 = xyz(E2);
                if (ne) {
                    float t, u, v;
                    if (ray_tri(o, d, v0, e1, e2, t, u, v) && t < best_t)
                        best_t = t, bu = u, bv = v, best = __float_as_int(E2.w);
                }
#pragma unroll
                for (int l = 0; l < NL; ++l) {
                    if (nsm & ~occ & (1u << l)) {
                        float t, u, v;
                        if (ray_tri(so[l], sd[l], v0, e1, e2, t, u, v) && t < stmax[l]) occ |= 1u << l;
                    }
                }
            }
        }
        const bool dext = want && root_overlap(r0, r1, r2, r3, o, inv, best_t);
        uint32_t dsh = 0;
#pragma unroll
        for (int l = 0; l < NL; ++l)
            if ((smask & ~occ & (1u << l)) && root_overlap(r0, r1, r2, r3, so[l], rcp3(sd[l]), stmax[l])) dsh |= 1u << l;
        if (valid) {
            if (want) P.hit[s] = make_float4(best_t, bu, bv, __int_as_float(best));
            if (smask) P.occ[s] = occ;
        }
        wave_append(valid && dext, s * 8u, dq, P.deep_count + it.p, lane);
#pragma unroll
        for (int l = 0; l < NL; ++l)
            wave_append(valid && ((dsh >> l) & 1u), s * 8u + 1u + (uint32_t)l, dq + P.part_cap,
                        P.deep_count + 2 * kMaxParts + it.p, lane);
    }
}

// bvh_leaf for a leaf of at most kBvhLeaf triangles with every triangle's loads issued before
// the first test (one memory round trip per leaf instead of one per triangle); tests and
// updates in the same order as bvh_leaf.
template <bool ANY>
__device__ __forceinline__ bool bvh_leaf_batch(const KParams& P, int first, int count, v3 o, v3 d, float tmax,
                                               float& bt, float& bu, float& bv, int& bk) {
    f4 T[kBvhLeafTri][3];
#pragma unroll
    for (int q = 0; q < (int)kBvhLeafTri; ++q)
        if (q < count) T[q][0] = P.bvh_tri[3 * (first + q)], T[q][1] = P.bvh_tri[3 * (first + q) + 1],
                       T[q][2] = P.bvh_tri[3 * (first + q) + 2];
#pragma unroll
    for (int q = 0; q < (int)kBvhLeafTri; ++q) {
        if (q >= count) break;
        if (ANY && T[q][1].w == 0.0f) continue;   // area-light objects never occlude
        float t, u, v;
        if (!ray_tri(o, d, xyz(T[q][0]), xyz(T[q][1]), xyz(T[q][2]), t, u, v)) continue;
        if (ANY) {
            if (t < tmax) return true;
        } else {
            const int k = __float_as_int(T[q][2].w);
            if (t < bt || (t == bt && k < bk)) bt = t, bu = u, bv = v, bk = k;
        }
    }
    return false;
}

// Phase B: the queued rays walk the BVH's 4-wide form (bvh.h Bvh4Node: a step fetches four
// child boxes, the tree is about half as deep as the binary one), with dynamic ray fetch —
// a lane whose ray is done takes the next queued ray of its partition (one atomic per wave
// per refill, when at least 16 lanes are idle or the wave is empty), so lanes stay busy
// until the queue drains (a static assignment measured lane utilisation 0.095: most queued
// rays cross the mesh's box and leave after a few nodes, a few descend to the surface).
// One loop iteration = one node per active lane: the four children tested against [0, lim]
// (lim = best t, inclusive, for closest hits; tmax for shadow rays), leaf children first
// (bvh_leaf: the (t, index) order; shadow rays stop at the first occluder), then the nearest
// interior child that still overlaps [0, best t] is next and the other overlapping ones are
// stacked.  Exact for the same reason as bvh_trace: every triangle whose padded box overlaps
// [0, best t] is tested, whatever the order.
template <typename SE>
__global__ __launch_bounds__(kBlock, XRT_DEEP_WAVES) void k_trace_deep4(KParams P) {
    extern __shared__ uint32_t bvh_stack_lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int ntop = P.bvh4_nodes < (int)kBvhTopNodes ? P.bvh4_nodes : (int)kBvhTopNodes;
    f4* top = reinterpret_cast<f4*>(bvh_stack_lds);
    for (int q = tid; q < 8 * ntop; q += kBlock) top[q] = P.bvh4[q];
    SE* stk = reinterpret_cast<SE*>(bvh_stack_lds + 32 * ntop) + tid;
    __syncthreads();
    const uint32_t p = blockIdx.x % P.n_part;
    // extension rays first, then shadow rays (queued apart by phase A), so a wave's lanes
    // mostly run the same kind of walk (closest hit or any hit) at a time
    const uint32_t n_ext = P.deep_count[p];
    const uint32_t cnt = n_ext + P.deep_count[2 * kMaxParts + p];
    uint32_t* next_ctr = P.deep_count + kMaxParts + p;
    const uint32_t* dq = P.deep + (size_t)p * P.deep_cap;
    const uint32_t* dqs = dq + P.part_cap - n_ext;   // dqs[idx] for idx >= n_ext
#ifdef XRT_EXPERIMENTS
    if (blockIdx.x < P.n_part && tid == 0) atomicAdd(P.stats + 38, (unsigned long long)cnt);
    uint32_t nsteps = 0, niter = 0;
#endif
    bool active = false, drained = cnt == 0, any = false;
    uint32_t s = 0, l = 0;
    int node = 0, sp = 0, bk = -1;
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0), inv = mk(0, 0, 0);
    float tmax = 0.0f, bt = kINF, bu = 0.0f, bv = 0.0f;
    while (true) {
#ifdef XRT_EXPERIMENTS
        nsteps += active ? 1u : 0u;
        ++niter;
#endif
        const uint64_t idle = __ballot(!active);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (!drained && (nidle >= 16u || nidle == 64u)) {
            const int leader = __ffsll((unsigned long long)idle) - 1;
            uint32_t b = 0;
            if (lane == leader) b = atomicAdd(next_ctr, nidle);
            b = (uint32_t)__builtin_amdgcn_readlane((int)b, leader);
            if (b + nidle >= cnt) drained = true;
            if (!active) {
                const uint32_t idx = b + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                if (idx < cnt) {
                    const uint32_t e = idx < n_ext ? dq[idx] : dqs[idx];
                    s = e >> 3;
                    const uint32_t kind = e & 7u;
                    any = kind != 0;
                    if (!any) {
                        o = xyz(P.ray_o[s]), d = xyz(P.ray_d[s]);
                        const f4 h = P.hit[s];
                        bt = h.x, bu = h.y, bv = h.z, bk = __float_as_int(h.w);
                        tmax = kINF;
                    } else {
                        l = kind - 1u;
                        const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                        o = xyz(a), tmax = a.w;
                        d = xyz(P.sh_d[(size_t)l * P.n_slots + s]);
                        bt = kINF, bk = -1;
                    }
                    inv = rcp3(d);
                    node = 0, sp = 0;
                    active = true;
                }
            }
        }
        if (!__ballot(active)) break;
        if (!active) continue;
        f4 lo[4], hi[4];
        {
            const f4* N = node < ntop ? top + 8 * node : P.bvh4 + 8 * (size_t)node;
#pragma unroll
            for (int c = 0; c < 4; ++c) lo[c] = N[c], hi[c] = N[4 + c];
        }
        float e[4];
        {
            const float lim = any ? tmax : bt;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                e[c] = __float_as_int(hi[c].w) >= 0 ? bvh_enter(lo[c], hi[c], o, inv, lim) : __builtin_inff();
        }
        bool occluded = false;
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // leaves first (either order gives the same result)
            const int k = __float_as_int(hi[c].w);
            if (!occluded && k > 0 && e[c] != __builtin_inff())
                occluded = any ? bvh_leaf_batch<true>(P, __float_as_int(lo[c].w), k, o, d, tmax, bt, bu, bv, bk)
                               : bvh_leaf_batch<false>(P, __float_as_int(lo[c].w), k, o, d, tmax, bt, bu, bv, bk);
        }
        bool done = occluded;
        if (!done) {
            // interior children still overlapping [0, lim] (bt may have shrunk at the leaves:
            // e <= bt is the same test as a fresh one against the smaller limit)
            const float lim = any ? tmax : bt;
            int nx = -1;
            float en = __builtin_inff();
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (__float_as_int(hi[c].w) != 0 || !(e[c] <= lim)) continue;
                const int idx = __float_as_int(lo[c].w);
                if (nx < 0 || e[c] < en) {
                    if (nx >= 0) stk[(sp++) * kBlock] = (SE)nx;
                    nx = idx, en = e[c];
                } else {
                    stk[(sp++) * kBlock] = (SE)idx;
                }
            }
            if (nx >= 0) node = nx;
            else if (sp == 0) done = true;
            else node = (int)stk[(--sp) * kBlock];
        }
        if (done) {
            if (!any) P.hit[s] = make_float4(bt, bu, bv, __int_as_float(bk));
            else if (occluded) atomicOr(P.occ + s, 1u << l);
            active = false;
        }
    }
#ifdef XRT_EXPERIMENTS
    atomicAdd(P.stats + 39, (unsigned long long)nsteps);
    if (lane == 0) atomicAdd(P.stats + 37, (unsigned long long)niter), atomicMax(P.stats + 36, (unsigned long long)niter);
#endif
}

// Phase B with four lanes per ray ("quad"): lane q of a quad owns child q of the current
// node — loads its two float4, tests its box and, for a leaf child, that leaf's triangles.
// Each lane keeps its own best hit over the triangles it tested (bvh_leaf's (t, index) update
// from the ray's phase-A hit), and the quad shares only what steers the walk, by DPP
// quad_perm: the smallest t as the pruning limit (a 32-bit min per step), occlusion as an or,
// and the next node — the nearest overlapping interior child (key: entry distance with its
// two low bits replaced by the child slot; the order only steers the walk) — with the other
// overlapping ones pushed on one stack per quad.  When the walk ends the quad's closest hit
// is the minimum of the lanes' (t bits, index + 1) keys and the lane holding it writes its
// own (t, u, v, index).  A step costs one node fetch and at most one leaf per lane instead
// of four boxes and up to four leaves, so the longest walk of a launch — which bounds the
// launch when few rays are queued (a row shard of a multi-GPU frame) — takes fewer cycles.
// Exact for the same reason as k_trace_deep4: every triangle whose padded box overlaps
// [0, best t] is tested by some lane (each lane's limit is at least the quad's best t).
// Rays are fetched a quad at a time from the same partitioned queues and counters.
template <typename SE>
__global__ __launch_bounds__(kBlock, XRT_DEEP_WAVES) void k_trace_deep4q(KParams P) {
    extern __shared__ uint32_t bvh_stack_lds[];
    constexpr int kQuads = kBlock / 4;
    const int tid = threadIdx.x, lane = tid & 63, q = lane & 3;
    const int ntop = P.bvh4_nodes < (int)kBvhTopNodes ? P.bvh4_nodes : (int)kBvhTopNodes;
    f4* top = reinterpret_cast<f4*>(bvh_stack_lds);
    for (int i = tid; i < 8 * ntop; i += kBlock) top[i] = P.bvh4[i];
    SE* stk = reinterpret_cast<SE*>(bvh_stack_lds + 32 * ntop) + (tid >> 2);   // one stack per quad
    __syncthreads();
    const uint32_t p = blockIdx.x % P.n_part;
    // extension rays first, then shadow rays (queued apart by phase A), so a wave's lanes
    // mostly run the same kind of walk (closest hit or any hit) at a time
    const uint32_t n_ext = P.deep_count[p];
    const uint32_t cnt = n_ext + P.deep_count[2 * kMaxParts + p];
    uint32_t* next_ctr = P.deep_count + kMaxParts + p;
    const uint32_t* dq = P.deep + (size_t)p * P.deep_cap;
    const uint32_t* dqs = dq + P.part_cap - n_ext;   // dqs[idx] for idx >= n_ext
    constexpr uint64_t kLeads = 0x1111111111111111ull;   // lane 0 of every quad
#ifdef XRT_EXPERIMENTS
    if (blockIdx.x < P.n_part && tid == 0) atomicAdd(P.stats + 38, (unsigned long long)cnt);
    uint32_t nsteps = 0, niter = 0;
#endif
    bool active = false, drained = cnt == 0, any = false;
    uint32_t s = 0, l = 0;
    int node = 0, sp = 0, bk = -1;
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0), inv = mk(0, 0, 0);
    float tmax = 0.0f, bt = kINF, bu = 0.0f, bv = 0.0f;
    while (true) {
        const uint64_t idle = __ballot(!active) & kLeads;
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (!drained && (nidle >= 4u || nidle == 16u)) {
            const int leader = __ffsll((unsigned long long)idle) - 1;
            uint32_t b = 0;
            if (lane == leader) b = atomicAdd(next_ctr, nidle);
            b = (uint32_t)__builtin_amdgcn_readlane((int)b, leader);
            if (b + nidle >= cnt) drained = true;
            if (!active) {
                const uint32_t idx = b + (uint32_t)__popcll(idle & ((1ull << (lane & ~3)) - 1ull));
                if (idx < cnt) {
                    const uint32_t e = idx < n_ext ? dq[idx] : dqs[idx];
                    s = e >> 3;
                    const uint32_t kind = e & 7u;
                    any = kind != 0;
                    if (!any) {
                        o = xyz(P.ray_o[s]), d = xyz(P.ray_d[s]);
                        const f4 h = P.hit[s];
                        bt = h.x, bu = h.y, bv = h.z, bk = __float_as_int(h.w);
                        tmax = kINF;
                    } else {
                        l = kind - 1u;
                        const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                        o = xyz(a), tmax = a.w;
                        d = xyz(P.sh_d[(size_t)l * P.n_slots + s]);
                        bt = kINF, bk = -1;
                    }
                    inv = rcp3(d);
                    node = 0, sp = 0;
                    active = true;
                }
            }
        }
        if (!__ballot(active)) break;
#ifdef XRT_EXPERIMENTS
        ++niter;
        nsteps += (uint32_t)__popcll(__ballot(active) & kLeads);   // quads stepping (wave-uniform)
#endif
        if (!active) continue;
        // ---- one node: child q on lane q; lim = the quad's best t (closest hits) or tmax
        const f4* N = node < ntop ? top + 8 * node : P.bvh4 + 8 * (size_t)node;
        const f4 lo = N[q], hi = N[4 + q];
        const int cidx = __float_as_int(lo.w), ccnt = __float_as_int(hi.w);
        float lim = any ? tmax : __uint_as_float(group_min32<4>(__float_as_uint(bt)));   // t >= 0: bits order
        const float e = ccnt >= 0 ? bvh_enter(lo, hi, o, inv, lim) : __builtin_inff();
        bool done = false;
        if (any) {
            bool occ = false;
            if (ccnt > 0 && e != __builtin_inff()) occ = bvh_leaf_batch<true>(P, cidx, ccnt, o, d, tmax, bt, bu, bv, bk);
            done = group_or32<4>(occ ? 1u : 0u) != 0u;
            if (done && q == 0) atomicOr(P.occ + s, 1u << l);
        } else {
            if (ccnt > 0 && e != __builtin_inff()) {
                (void)bvh_leaf_batch<false>(P, cidx, ccnt, o, d, kINF, bt, bu, bv, bk);
                lim = __builtin_fminf(lim, bt);   // this lane's leaf may have closed in
            }
            lim = __uint_as_float(group_min32<4>(__float_as_uint(lim)));
        }
        if (!done) {
            const bool inner = ccnt == 0 && e <= lim;   // interior child still overlapping [0, lim]
            const uint32_t nkey = inner ? ((__float_as_uint(e) & ~3u) | (uint32_t)q) : ~0u;
            const uint32_t nmin = group_min32<4>(nkey);
            if (nmin != ~0u) {
                const bool nearest = nkey == nmin;
                const uint32_t m4 = (uint32_t)(__ballot(inner && !nearest) >> (lane & ~3)) & 0xfu;
                if (inner && !nearest) stk[(sp + __popc(m4 & ((1u << q) - 1u))) * kQuads] = (SE)cidx;
                sp += __popc(m4);
                node = (int)group_or32<4>(nearest ? (uint32_t)cidx : 0u);
            } else if (sp == 0) {
                done = true;
            } else {
                node = (int)stk[(--sp) * kQuads];
            }
        }
        if (done) {
            if (!any) {   // the quad's closest hit: the smallest (t bits, index + 1) of the lanes
                const uint64_t key = ((uint64_t)__float_as_uint(bt) << 32) | (uint32_t)(bk + 1);
                const uint64_t kmin = group_min64<4>(key);
                const uint32_t wm = (uint32_t)(__ballot(key == kmin) >> (lane & ~3)) & 0xfu;
                if (q == __builtin_ctz(wm)) P.hit[s] = make_float4(bt, bu, bv, __int_as_float(bk));
            }
            active = false;
        }
    }
#ifdef XRT_EXPERIMENTS
    if (lane == 0)
        atomicAdd(P.stats + 39, (unsigned long long)nsteps), atomicAdd(P.stats + 37, (unsigned long long)niter),
            atomicMax(P.stats + 36, (unsigned long long)niter);
#endif
}

// Small triangle scenes (<= kSmallTris triangles, e.g. the Cornell box): every triangle
// and the per-object boxes live in LDS for the whole launch; objects are visited in
// Scene iteration order and a wave skips an object none of its rays can hit (closest-hit
// rays are culled against the current best t, shadow rays against tmax; area-light
// objects are never occluders).  Inside an object the triangle order and the strict
// `t < best` update are the reference's, so results are identical to the linear scan.
template <int NL>
__global__ __launch_bounds__(kBlock) void k_trace_small(KParams P, const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count, uint32_t* zero_count) {
    extern __shared__ __attribute__((aligned(16))) f4 lds_small[];
    f4* ltri = lds_small;
    DObjBox* lbox = reinterpret_cast<DObjBox*>(lds_small + 3 * P.n_tris);
    zero_parts(P, zero_count);
    const int tid = threadIdx.x;
    for (int q = tid; q < 3 * P.n_tris; q += kBlock) ltri[q] = P.tri[q];
    for (int q = tid; q < P.n_objs; q += kBlock) lbox[q] = P.obj_box[q];
    __syncthreads();
    const PartIter it = part_iter(P, count, kBlock);
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        const bool valid = i < it.n;
        const uint32_t s = valid ? list[it.p * P.part_cap + i] : 0;
        const uint32_t st = valid ? P.state[s] : 0;
        const bool want = (st & ST_RAY) != 0;
        const uint32_t smask = (st >> ST_SHADOW_SHIFT) & ((1u << NL) - 1u);
        v3 o = mk(0, 0, 0), d = mk(0, 0, 0);
        if (want) {
            o = xyz(P.ray_o[s]);
            d = xyz(P.ray_d[s]);
        }
        v3 so[NL], sd[NL];
        float stmax[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            so[l] = mk(0, 0, 0), sd[l] = mk(0, 0, 0), stmax[l] = 0.0f;
            if (smask & (1u << l)) {
                const f4 a = P.sh_o[(size_t)l * P.n_slots + s];
                so[l] = xyz(a);
                stmax[l] = a.w;
                sd[l] = xyz(P.sh_d[(size_t)l * P.n_slots + s]);
            }
        }
        const v3 inv = rcp3(d);
        uint32_t occ = 0;
        float best_t = kINF, bu = 0.0f, bv = 0.0f;
        int best = -1;
        for (int ob = 0; ob < P.n_objs; ++ob) {
            const DObjBox B = lbox[ob];
            const int cnt = B.count_occ & 0x7fffffff;
            const bool occluder = B.count_occ < 0;
            const bool ne = want && box_overlap(o, inv, B, best_t);
            uint32_t nsm = 0;
            if (occluder) {
#pragma unroll
                for (int l = 0; l < NL; ++l)
                    if ((smask & ~occ & (1u << l)) && box_overlap(so[l], rcp3(sd[l]), B, stmax[l])) nsm |= 1u << l;
            }
            if (__ballot(ne || nsm) == 0) continue;
            for (int k = B.first; k < B.first + cnt; ++k) {
                const v3 v0 = xyz(ltri[3 * k]), e1 = xyz(ltri[3 * k + 1]), e2 = xyz(ltri[3 * k + 2]);
                if (ne) {
                    float t, u, v;
                    if (ray_tri(o, d, v0, e1, e2, t, u, v) && t < best_t) best_t = t, bu = u, bv = v, best = k;
                }
#pragma unroll
                for (int l = 0; l < NL; ++l) {
                    if (nsm & ~occ & (1u << l)) {
                        float t, u, v;
                        if (ray_tri(so[l], sd[l], v0, e1, e2, t, u, v) && t < stmax[l]) occ |= 1u << l;
                    }
                }
            }
        }
        if (valid) {
            if (want) P.hit[s] = make_float4(best_t, bu, bv, __int_as_float(best));
            if (smask) P.occ[s] = occ;
        }
    }
}

// ==================================================================== medium ====
// DensityGrid::getDensity = OpenVDB BoxSampler::wsSample (Src/grid.h:71-77): index-space
// position in double, floor, trilinear lerps a + float((b - a) * w) (z, then y, then x),
// background 0 outside the voxels.
__device__ __forceinline__ float grid_value(const DMedium& M, int i, int j, int k) {
    if (i < 0 || j < 0 || k < 0 || i >= M.nx || j >= M.ny || k >= M.nz) return 0.0f;
    return M.density[((size_t)k * M.ny + (size_t)j) * M.nx + (size_t)i];
}
__device__ __forceinline__ float vdb_lerp(float a, float b, double w) { return a + (float)((double)(b - a) * w); }
// sparse leaf bricks: one voxel (background 0 outside the grid and in inactive bricks)
__device__ __forceinline__ float brick_value(const DMedium& M, int i, int j, int k) {
    if (i < 0 || j < 0 || k < 0 || i >= M.nx || j >= M.ny || k >= M.nz) return 0.0f;
    const int b = M.brick_table[((k >> 3) * M.nby + (j >> 3)) * M.nbx + (i >> 3)];
    return b < 0 ? 0.0f : M.bricks[(size_t)b * 512 + (((k & 7) * 8 + (j & 7)) * 8 + (i & 7))];
}
// OpenVDB BoxSampler cell of a world position: index-space coordinates in double, the
// lower corner (i, j, k) and the fractional weights
struct VdbCell {
    double u, v, w;
    int i, j, k;
};
__device__ __forceinline__ VdbCell vdb_cell(const DMedium& M, v3 p) {
    const double inv = M.inv_voxel;
    const double xi = ((double)p.x - (double)M.origin[0]) * inv;
    const double yi = ((double)p.y - (double)M.origin[1]) * inv;
    const double zi = ((double)p.z - (double)M.origin[2]) * inv;
    const double fx = __builtin_floor(xi), fy = __builtin_floor(yi), fz = __builtin_floor(zi);
    VdbCell C;
    C.i = (int)fx, C.j = (int)fy, C.k = (int)fz;
    C.u = xi - fx, C.v = yi - fy, C.w = zi - fz;
    return C;
}
// dense grid, all eight corners inside: the x-neighbours are adjacent words, four dword-aligned
// dwordx2 loads, corners in the order d000 d001 d010 d011 d100 d101 d110 d111
__device__ __forceinline__ bool dense_interior(const DMedium& M, const VdbCell& C) {
    return !M.brick_table && C.i >= 0 && C.j >= 0 && C.k >= 0 && C.i + 1 < M.nx && C.j + 1 < M.ny && C.k + 1 < M.nz;
}
__device__ __forceinline__ void dense_corners(const DMedium& M, const VdbCell& C, float (&q)[8]) {
    if (M.corners) {
        const f4* r = reinterpret_cast<const f4*>(M.corners) +
                      2 * (((size_t)C.k * (M.ny - 1) + (size_t)C.j) * (M.nx - 1) + (size_t)C.i);
        const f4 a = r[0], b = r[1];
        q[0] = a.x, q[1] = a.y, q[2] = a.z, q[3] = a.w, q[4] = b.x, q[5] = b.y, q[6] = b.z, q[7] = b.w;
        return;
    }
    typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
    using g2 = __attribute__((address_space(1))) const f2u;
    const float* b = M.density + ((size_t)C.k * M.ny + (size_t)C.j) * M.nx + (size_t)C.i;
    const size_t sy = (size_t)M.nx, sz = (size_t)M.nx * M.ny;
    const f2u a = *(g2*)b, c = *(g2*)(b + sz), e = *(g2*)(b + sy), f = *(g2*)(b + sy + sz);
    q[0] = a.x, q[4] = a.y, q[1] = c.x, q[5] = c.y, q[2] = e.x, q[6] = e.y, q[3] = f.x, q[7] = f.y;
}
__device__ __forceinline__ float vdb_interp(const DMedium& M, const VdbCell& C, const float (&q)[8]) {
    const float g = vdb_lerp(vdb_lerp(vdb_lerp(q[0], q[1], C.w), vdb_lerp(q[2], q[3], C.w), C.v),
                             vdb_lerp(vdb_lerp(q[4], q[5], C.w), vdb_lerp(q[6], q[7], C.w), C.v), C.u);
    return M.multiplier * g;   // HeterogeneousMedium::getDensity (Src/medium.cpp:24-27)
}

__device__ float medium_density(const DMedium& M, v3 p) {
    const VdbCell C = vdb_cell(M, p);
    const int i = C.i, j = C.j, k = C.k;
    float q[8];
    if (M.brick_table) {
        // a cell inside one brick: one table lookup, x-neighbours adjacent in the brick
        if (i >= 0 && j >= 0 && k >= 0 && i + 1 < M.nx && j + 1 < M.ny && k + 1 < M.nz && (i & 7) != 7 &&
            (j & 7) != 7 && (k & 7) != 7) {
            const int b = M.brick_table[((k >> 3) * M.nby + (j >> 3)) * M.nbx + (i >> 3)];
            if (b < 0) {
                for (int c = 0; c < 8; ++c) q[c] = 0.0f;
            } else {
                const float* r = M.bricks + (size_t)b * 512 + (((k & 7) * 8 + (j & 7)) * 8 + (i & 7));
                q[0] = r[0], q[4] = r[1], q[2] = r[8], q[6] = r[9];
                q[1] = r[64], q[5] = r[65], q[3] = r[72], q[7] = r[73];
            }
        } else {
            q[0] = brick_value(M, i, j, k), q[1] = brick_value(M, i, j, k + 1);
            q[2] = brick_value(M, i, j + 1, k), q[3] = brick_value(M, i, j + 1, k + 1);
            q[4] = brick_value(M, i + 1, j, k), q[5] = brick_value(M, i + 1, j, k + 1);
            q[6] = brick_value(M, i + 1, j + 1, k), q[7] = brick_value(M, i + 1, j + 1, k + 1);
        }
    } else if (dense_interior(M, C)) {
        dense_corners(M, C, q);
    } else {
        q[0] = grid_value(M, i, j, k), q[1] = grid_value(M, i, j, k + 1);
        q[2] = grid_value(M, i, j + 1, k), q[3] = grid_value(M, i, j + 1, k + 1);
        q[4] = grid_value(M, i + 1, j, k), q[5] = grid_value(M, i + 1, j, k + 1);
        q[6] = grid_value(M, i + 1, j + 1, k), q[7] = grid_value(M, i + 1, j + 1, k + 1);
    }
    return vdb_interp(M, C, q);
}

// Medium::sampleWavelength + DiscreteEmpiricalDistribution1D (Src/medium.h:102-115,
// Src/sampler.h:53-94).  lower_bound past the end is UB in the reference; clamped to 2.
__device__ __forceinline__ uint32_t sample_wavelength(v3 thr, v3 albedo, Rng& rng, v3& pmf) {
    const v3 ta = thr * albedo;
    const float sum = ((0.0f + ta.x) + ta.y) + ta.z;
    const v3 q = div3s(ta, sum);   // ta.x / sum, ta.y / sum, ta.z / sum
    const float c1 = 0.0f + q.x;
    const float c2 = c1 + q.y;
    const float c3 = c2 + q.z;
    pmf = mk(c1 - 0.0f, c2 - c1, c3 - c2);
    const float u = rng.next();
    int x = 0;
    if (0.0f < u) {
        x = 1;
        if (c1 < u) {
            x = 2;
            if (c2 < u) x = (c3 < u) ? 4 : 3;
        }
    }
    if (x == 0) x = 1;
    if (x == 4) x = 3;
    return (uint32_t)(x - 1);
}

// HenyeyGreenstein::sampleDirection (Src/medium.h:37-67); getNext2D = (2nd, 1st draw)
__device__ void hg_sample(float g, v3 wo, Rng& rng, v3& wi) {
    const float d1 = rng.next();
    const float d2 = rng.next();
    const float u0 = d2, u1 = d1;
    float cosTheta;
    if (__builtin_fabs((double)g) < 1e-3) {
        cosTheta = 2.0f * u0 - 1.0f;
    } else {
        const float sqrTerm = (1.0f - g * g) / (1.0f - g + 2.0f * g * u0);
        cosTheta = (1.0f + g * g - sqrTerm * sqrTerm) / (2.0f * g);
    }
    const float sinTheta = __builtin_sqrtf(smax(1.0f - cosTheta * cosTheta, 0.0f));
    const float phi = 2.0f * kPI * u1;
    float sphi, cphi;
    glibc_sincosf(phi, sphi, cphi);
    const v3 wl = mk(cphi * sinTheta, cosTheta, sphi * sinTheta);
    v3 t, b;
    onb(wo, t, b);
    wi = local_to_world(wl, t, wo, b);
}

__device__ __forceinline__ v3 vexp(v3 a) { return mk(glibc_expf(a.x), glibc_expf(a.y), glibc_expf(a.z)); }
__device__ __forceinline__ bool isnan3(v3 a) {
    return __builtin_isnan(a.x) || __builtin_isnan(a.y) || __builtin_isnan(a.z);
}

// HeterogeneousMedium::sampleMedium — delta tracking with spectral MIS (Src/medium.cpp:
// 45-133), one collision per call: returns 0 = left the medium, 1 = real scattering,
// 2 = suspended because fewer than 8 RNG words remain (the slot resumes after the next
// refill), 3 = null collision (call again).  `t`, `tt` (throughput_tracking) and `sa`
// (sigma_a) carry the loop state.
__device__ __forceinline__ int delta_step(const KParams& P, v3 o, v3 d, v3 thr, float& t, float t1, v3& tt, v3& sa,
                                          Rng& rng, uint32_t g, v3& pos, v3& dir, v3& tm) {
    const DMedium& M = P.medium;
    const float majorant = M.majorant, invMajorant = M.inv_majorant;
    const v3 vmaj = mk(majorant, majorant, majorant);
    const v3 absorb = ld3(M.absorption), scatter = ld3(M.scattering);
    if (g - rng.c < 8u) return 2;
    v3 pmf;
    const uint32_t channel = sample_wavelength(thr * tt, (vmaj - sa) * invMajorant, rng, pmf);
    const float s = -glibc_logf(smax(1.0f - rng.next(), 0.0f)) * invMajorant;
    t += s;
    // the three outcomes share the transmittance and the throughput update: one expf and
    // one quotient per collision however the wave's lanes split (same operands per lane)
    int r = 0;
    float x, fe = 1.0f;   // the expf argument's distance; the majorant factor of the pdf
    v3 num = mk(0, 0, 0), Px = mk(1, 1, 1);
    if (t > t1 - kRAY_EPS) {
        pos = ray_at(o, d, t1 + kRAY_EPS);
        dir = d;
        x = s - (t - (t1 - kRAY_EPS));
    } else {
        const float density = medium_density(M, ray_at(o, d, t));
        const v3 sigma_s = scatter * density;
        sa = absorb * density;
        const v3 sigma_n = (vmaj - sa) - sigma_s;
        const v3 den = sigma_s + sigma_n;
        x = s, fe = majorant;
        // P_s = sigma_s / (sigma_s + sigma_n): the acceptance test reads one component
        r = rng.next() < comp(sigma_s, channel) / comp(den, channel) ? 1 : 3;
        if (r == 1) {
            pos = ray_at(o, d, t);
            hg_sample(M.g, d, rng, dir);
        }
        num = r == 1 ? sigma_s : sigma_n;
        Px = div3v(num, den);
    }
    const float e = glibc_expf(-majorant * x);   // vexp((-vmaj) * x): three equal arguments
    const v3 tr = mk(e, e, e);
    const v3 pdf = r == 0 ? pmf * tr : (pmf * (tr * fe)) * Px;
    tt = tt * div3s(r == 0 ? tr : tr * num, pdf.x + pdf.y + pdf.z);
    if (r != 3) tm = isnan3(tt) ? mk(0, 0, 0) : tt;
    return r;
}
// the whole walk (0, 1 or 2 as delta_step)
__device__ int delta_track(const KParams& P, v3 o, v3 d, v3 thr, float& t, float t1, v3& tt, v3& sa, Rng& rng,
                           uint32_t g, v3& pos, v3& dir, v3& tm) {
    for (;;) {
        const int r = delta_step(P, o, d, thr, t, t1, tt, sa, rng, g, pos, dir, tm);
        if (r != 3) return r;
    }
}

// HenyeyGreenstein::evaluate (Src/medium.h:29-34)
__device__ __forceinline__ float hg_eval(float g, v3 wo, v3 wi) {
    const float cosTheta = dot(wo, wi);
    const float denom = 1.0f + g * g - 2.0f * g * cosTheta;
    return kPI_MUL_4_INV * (1.0f - g * g) / (denom * __builtin_sqrtf(denom));
}

// HeterogeneousMedium::ratioTrackingTransmittance (Src/medium.h:360-386), resumable like
// delta_track: false = suspended (fewer than 8 RNG words left); `t`, `tr` carry the loop.
__device__ bool ratio_track(const KParams& P, v3 p1, v3 dn, float dist, float& t, v3& tr, Rng& rng, uint32_t g) {
    const DMedium& M = P.medium;
    const float majorant = M.majorant, invMajorant = M.inv_majorant;
    const v3 vmaj = mk(majorant, majorant, majorant);
    const v3 absorb = ld3(M.absorption), scatter = ld3(M.scattering);
    for (;;) {
        if (g - rng.c < 8u) return false;
        const float s = -glibc_logf(smax(1.0f - rng.next(), 0.0f)) * invMajorant;
        t += s;
        if (t > dist) return true;
        const float density = medium_density(M, ray_at(p1, dn, t));
        const v3 sigma_n = (vmaj - absorb * density) - scatter * density;
        tr = tr * (sigma_n * invMajorant);
    }
}

// VPT-NEE light sample at a scattering point and its resumption (defined with the fused
// schedule's scene traversal below)
template <int SCN>
__device__ int nee_medium(const KParams& P, const LScene& L, uint32_t s, v3 pos, v3 wo, v3 thr_m, v3& rad, Rng& rng,
                          uint32_t g, uint32_t& nsh);
__device__ int nee_resume(const KParams& P, uint32_t s, v3 thr_m, v3& rad, Rng& rng, uint32_t g);

// Homogeneous media (Src/medium.h:122-277): one free-flight sample per visit of the medium
// box, analytic transmittance exp(-sigma_t * t) (Medium::analyticTransmittance).  Same
// return contract as delta_track (0 = left the medium, 1 = scattering); never suspends
// (at most 4 draws).  t, t1: the box hit's entry / exit (IntersectInfo t, t1).
__device__ __forceinline__ v3 analytic_tr(float t, v3 sigma_t) { return vexp((-sigma_t) * t); }
__device__ int homog_track(const KParams& P, v3 o, v3 d, v3 thr, float t0, float t1, Rng& rng, v3& pos, v3& dir,
                           v3& tm) {
    const DMedium& M = P.medium;
    const v3 ss = ld3(M.scattering), st = ld3(M.sigma_t);
    const float distToSurface = t1 - t0;
    if (M.kind == XRT_MEDIUM_HOMOGENEOUS_MIS) {
        // HomogeneousMediumMIS::sampleMedium (Src/medium.h:154-191)
        v3 pmf;
        const uint32_t channel = sample_wavelength(thr, div3v(ss, st), rng, pmf);
        const float t = -glibc_logf(smax(1.0f - rng.next(), 0.0f)) / comp(st, channel);
        if (t > distToSurface - kRAY_EPS) {
            pos = ray_at(o, d, t1 + kRAY_EPS);
            dir = d;
            const v3 tr = analytic_tr(distToSurface, st);
            const v3 pdf = pmf * tr;
            tm = div3s(tr, pdf.x + pdf.y + pdf.z);
            return 0;
        }
        hg_sample(M.g, d, rng, dir);
        pos = ray_at(o, d, t0 + t);
        const v3 tr = analytic_tr(t, st);
        const v3 pdf = pmf * (st * tr);
        tm = div3s(tr * ss, pdf.x + pdf.y + pdf.z);
        return 1;
    }
    if (M.kind == XRT_MEDIUM_HOMOGENEOUS_ACHROMATIC) {
        // HomogeneousMediumAchromatic::sampleMedium (Src/medium.h:201-229)
        const float t = -glibc_logf(smax(1.0f - rng.next(), 0.0f)) / st.x;
        if (t > distToSurface - kRAY_EPS) {
            pos = ray_at(o, d, t1 + kRAY_EPS);
            dir = d;
            tm = mk(1.0f, 1.0f, 1.0f);
            return 0;
        }
        hg_sample(M.g, d, rng, dir);
        pos = ray_at(o, d, t0 + t);
        tm = div3v(ss, st);
        return 1;
    }
    // HomogeneousMediumNoMIS::sampleMedium (Src/medium.h:240-275)
    int channel = (int)(3.0f * rng.next());
    if (channel == 3) channel--;
    const float pmf_wavelength = 1.0f / 3.0f;
    const float sc = comp(st, (uint32_t)channel);
    const float t = -glibc_logf(smax(1.0f - rng.next(), 0.0f)) / sc;
    const float pdf_distance = sc * glibc_expf(-sc * t);
    if (t > distToSurface - kRAY_EPS) {
        pos = ray_at(o, d, t1 + kRAY_EPS);
        dir = d;
        const v3 tr = analytic_tr(distToSurface, st);
        const float p_surface = glibc_expf(-sc * distToSurface);
        tm = (tr * (1.0f / 3.0f)) / (pmf_wavelength * p_surface);
        return 0;
    }
    hg_sample(M.g, d, rng, dir);
    pos = ray_at(o, d, t0 + t);
    tm = ((analytic_tr(t, st) * (1.0f / 3.0f)) * ss) / (pmf_wavelength * pdf_distance);
    return 1;
}

// =================================================================== k_shade ====
template <int SCN, int INTEG>
__global__ __launch_bounds__(kBlock, XRT_SHADE_WAVES) void k_shade(KParams P, const uint32_t* __restrict__ list,
                                                   const uint32_t* __restrict__ count, uint32_t* __restrict__ out,
                                                   uint32_t* out_count, uint32_t* req_count) {
    __shared__ __attribute__((aligned(16))) uint32_t rbuf[kBlock / 64][kMT];   // wave_refill staging
    const PartIter it = part_iter(P, count, kBlock);
    const int tid = threadIdx.x, lane = tid & 63;
    // the two-level trace that follows appends to zeroed deep-queue counters (instead of a
    // memset launch per iteration); the previous iteration's deep walk is done by now
    if (P.two_level && P.deep_count && blockIdx.x == 0)
        for (uint32_t q = tid; q < 3 * kMaxParts; q += kBlock) P.deep_count[q] = 0;
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        const bool valid = i < it.n;
        const uint32_t s = valid ? list[it.p * P.part_cap + i] : 0;
        const uint32_t g = valid ? P.rng_g[s] : 0;
        Rng rng{P.ring + (size_t)s * kRing, valid ? P.rng_c[s] : 0};
        uint32_t st = valid ? P.state[s] : ST_DONE;
        // RNG words: below kRngMin the wave twists the slot's next block at the end of this
        // launch (wave_refill below; the block overwrites ring words < g - 624 <= c, all
        // drawn); below kRngVisit the slot sits this launch out
        const uint32_t avail = g - rng.c;
        const bool want_req = valid && avail < kRngMin;
        const bool go = valid && avail >= kRngVisit;
        if (go) {
            rng.prefetch(avail);
            uint32_t depth = P.depth[s];
            uint32_t k = P.sample_k[s];
            v3 thr = xyz(P.thr[s]), rad = xyz(P.rad[s]);
            v3 o = mk(0, 0, 0), d = mk(0, 0, 0);
            uint32_t nseg = 0, nsh = 0, nrej = 0, nstall = 0;
            bool finalize = false;

            // ---- 1. resolve the previous bounce's NEE with the shadow-ray results
            if (st & ST_NEE) {
                const uint32_t smask = (st >> ST_SHADOW_SHIFT) & 0xffu;
                const uint32_t occ = smask ? P.occ[s] : 0u;
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    // radiance += vis * fr * L * cos / pdf per light (Src/integrator.h:95-109)
                    for (int l = 0; l < P.n_lights; ++l) {
                        if (!(smask & (1u << l))) continue;
                        const v3 c = (occ & (1u << l)) ? mk(0, 0, 0) : xyz(P.sh_c[(size_t)l * P.n_slots + s]);
                        rad = rad + c;
                    }
                } else {
                    // L_light = 0 + vis*fr*L*cos/pdf; directL += L_light; radiance += thr*directL
                    // (Src/integrator.h:249-269)
                    v3 directL = mk(0, 0, 0);
                    for (int l = 0; l < P.n_lights; ++l) {
                        if (!(smask & (1u << l))) continue;
                        const v3 c = (occ & (1u << l)) ? mk(0, 0, 0) : xyz(P.sh_c[(size_t)l * P.n_slots + s]);
                        directL = directL + (mk(0, 0, 0) + c);
                    }
                    rad = rad + xyz(P.thr_prev[s]) * directL;
                }
                st &= ~(ST_NEE | (0xffu << ST_SHADOW_SHIFT));
                if (st & ST_END) finalize = true;
            }

            // ---- 2. shade the traced extension ray (or resume a suspended medium walk)
            if (vpt_family(INTEG) && (st & (ST_RAY | ST_MEDIUM | ST_NEEWALK))) {
                // VolumePathTracing::integrate loop body (Src/integrator.h:418-469);
                // VolumePathTracingNEE (:497-581)
                o = xyz(P.ray_o[s]);
                d = xyz(P.ray_d[s]);
                bool walk = false;
                float mt = 0.0f, mt1 = 0.0f;
                v3 tt = mk(1, 1, 1), sa = mk(0, 0, 0);
                if (INTEG == XRT_INTEGRATOR_VPT_NEE && (st & ST_NEEWALK)) {
                    // suspended NEE ratio tracking; the path ray after the scatter is stored
                    if (nee_resume(P, s, thr, rad, rng, g) == 0) {
                        st &= ~ST_NEEWALK;
                        if (depth < P.max_depth) st |= ST_RAY;
                        else finalize = true;
                    }
                } else if (st & ST_MEDIUM) {
                    st &= ~ST_MEDIUM;
                    const f4 m1 = P.med[s], m2 = P.med2[s];
                    mt = m1.x, mt1 = m1.y, sa = mk(m1.z, m1.w, m2.w), tt = xyz(m2);
                    walk = true;
                } else {
                    st &= ~ST_RAY;
                    ++nseg;
                    Surf S;
                    float t1;
                    const f4 h = P.hit[s];
                    const int obj = surface<SCN>(P, s, o, d, h, S, t1);
                    if (obj < 0) {
                        rad = rad + (thr * mk(0.0f, 0.0f, 0.0f)) * (float)(depth != 0);
                        finalize = true;
                    } else {
                        bool alive = true;
                        if (depth > 0) {
                            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
                            if (rng.next() >= p) alive = false, finalize = true;
                            else thr = thr / mk(p, p, p);
                        }
                        const DObj ob = P.objs[obj];
                        if (alive && ob.light >= 0) {
                            if (INTEG == XRT_INTEGRATOR_VPT || depth == 0)
                                rad = rad + thr * light_Le(P.lights[ob.light], S.ns, d);
                            alive = false, finalize = true;
                        }
                        if (alive) {
                            if (ob.medium >= 0) {
                                // sampleMedium entry (Src/medium.cpp:47-52): t = info.t
                                mt = h.x, mt1 = t1;
                                if (P.medium.kind == XRT_MEDIUM_HETEROGENEOUS)
                                    sa = ld3(P.medium.absorption) * medium_density(P.medium, ray_at(o, d, mt));
                                walk = true;
                            } else {
                                // neither light nor medium: the reference never advances this
                                // ray (endless loop); stop the path and count it.
                                ++nstall;
                                finalize = true;
                            }
                        }
                    }
                }
                if (walk) {
                    v3 pos, dir, tm;
                    const int r = P.medium.kind == XRT_MEDIUM_HETEROGENEOUS
                                      ? delta_track(P, o, d, thr, mt, mt1, tt, sa, rng, g, pos, dir, tm)
                                      : homog_track(P, o, d, thr, mt, mt1, rng, pos, dir, tm);
                    if (r == 2) {
                        st |= ST_MEDIUM;
                        P.med[s] = make_float4(mt, mt1, sa.x, sa.y);
                        P.med2[s] = make_float4(tt.x, tt.y, tt.z, sa.z);
                    } else {
                        int nr = 0;
                        if (INTEG == XRT_INTEGRATOR_VPT_NEE && r == 1) {
                            LScene Lg;   // the scene in global memory (linear scans, SCN_MIXED)
                            Lg.tri = P.tri, Lg.tng = P.tri_ng, Lg.nrm = P.tri_nrm, Lg.box = P.obj_box;
                            Lg.sph = P.sph, Lg.sobj = P.sph_obj, Lg.bx = P.box, Lg.obj = P.objs, Lg.light = P.lights;
                            nr = nee_medium<SCN>(P, Lg, s, pos, d, thr * tm, rad, rng, g, nsh);
                        }
                        o = pos;
                        d = dir;
                        thr = thr * tm;
                        if (r == 1) ++depth;
                        if (nr == 2) {
                            st |= ST_NEEWALK;   // resumes after the refill
                            P.ray_o[s] = pk(o);
                            P.ray_d[s] = pk(d);
                        } else if (depth < P.max_depth) {
                            st |= ST_RAY;
                            P.ray_o[s] = pk(o);
                            P.ray_d[s] = pk(d);
                        } else {
                            finalize = true;
                        }
                    }
                }
            } else if (st & ST_RAY) {
                st &= ~ST_RAY;
                ++nseg;
                o = xyz(P.ray_o[s]);
                d = xyz(P.ray_d[s]);
                Surf S;
                float t1;
                const int obj = surface<SCN>(P, s, o, d, P.hit[s], S, t1);
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    // DirectIntegrator::integrate (Src/integrator.h:82-119)
                    if (obj < 0) {
                        rad = mk((float)0.18, (float)0.18, (float)0.18);
                        finalize = true;
                    } else if (P.objs[obj].light >= 0) {
                        rad = light_Le(P.lights[P.objs[obj].light], S.ns, d);
                        finalize = true;
                    } else {
                        const DObj ob = P.objs[obj];
                        uint32_t smask = 0;
                        for (int l = 0; l < P.n_lights; ++l) {
                            v3 wi = mk(0, 0, 0);
                            float tmax = 0.0f, pdf = 0.0f;
                            const v3 L = light_sample(P.lights[l], S.pos, wi, pdf, tmax, rng);
                            if (pdf == 0.0f) continue;
                            const float bias = 0.01f;
                            const float cosv = smax(0.0f, dot(S.ng, wi));
                            const v3 fr = eval_bxdf(ob);
                            P.sh_o[(size_t)l * P.n_slots + s] = pk(S.pos + S.ng * bias, tmax - bias);
                            P.sh_d[(size_t)l * P.n_slots + s] = pk(wi);
                            P.sh_c[(size_t)l * P.n_slots + s] = pk(((fr * L) * cosv) / pdf);
                            smask |= 1u << l;
                            ++nsh;
                        }
                        if (smask) st |= ST_NEE | ST_END | (smask << ST_SHADOW_SHIFT);
                        else finalize = true;
                    }
                } else if (INTEG == XRT_INTEGRATOR_NORMAL) {
                    // NormalIntegrator::integrate (Src/integrator.h:28-37): 0.5 * (ns + 1)
                    if (obj >= 0) rad = normal_color(S.ns);
                    finalize = true;
                } else {
                    // GIIntegrator::integrate loop body (Src/integrator.h:214-284);
                    // IndirectIntegrator (Src/integrator.h:138-185): no light sampling, Le at
                    // every depth
                    if (obj < 0) {
                        rad = rad + thr * mk(0.0f, 0.0f, 0.0f);
                        finalize = true;
                    } else {
                        bool alive = true;
                        if (depth > 0) {
                            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
                            if (rng.next() >= p) alive = false, finalize = true;
                            else thr = thr / mk(p, p, p);
                        }
                        const DObj ob = P.objs[obj];
                        if (alive && ob.light >= 0) {
                            if (depth == 0 || INTEG == XRT_INTEGRATOR_INDIRECT)
                                rad = rad + thr * light_Le(P.lights[ob.light], S.ns, d);
                            alive = false, finalize = true;
                        }
                        if (alive) {
                            uint32_t smask = 0;
                            for (int l = 0; l < (INTEG == XRT_INTEGRATOR_GI ? P.n_lights : 0); ++l) {
                                v3 wi = mk(0, 0, 0);
                                float tmax = 0.0f, pdf = 0.0f;
                                const v3 L = light_sample(P.lights[l], S.pos, wi, pdf, tmax, rng);
                                if (pdf == 0.0f) continue;
                                const float bias = 0.01f;
                                const float cosv = smax(0.0f, dot(S.ng, wi));
                                const v3 fr = eval_bxdf(ob);
                                P.sh_o[(size_t)l * P.n_slots + s] = pk(S.pos + S.ng * bias, tmax - bias);
                                P.sh_d[(size_t)l * P.n_slots + s] = pk(wi);
                                P.sh_c[(size_t)l * P.n_slots + s] = pk(((fr * L) * cosv) / pdf);
                                smask |= 1u << l;
                                ++nsh;
                            }
                            if (smask) {
                                P.thr_prev[s] = pk(thr);
                                st |= ST_NEE | (smask << ST_SHADOW_SHIFT);
                            } else if (INTEG == XRT_INTEGRATOR_GI) {
                                rad = rad + thr * mk(0, 0, 0);   // radiance += thr * directL(=0)
                            }
                            // indirect: Object::sampleBxDF -> Lambert (no material: 0, no draws)
                            float pdf = 1.0f;
                            v3 nd = mk(0, 0, 0), fr = mk(0, 0, 0);
                            if (ob.material == 1) {
                                nd = lambert_sample(S, rng);
                                pdf = 1.0f / (2.0f * kPI);
                                fr = eval_bxdf(ob);
                            }
                            const float cosv = smax(0.0f, dot(nd, S.ng));
                            thr = thr * ((fr * cosv) / pdf);
                            o = S.pos + S.ng * 0.01f;
                            d = nd;
                            ++depth;
                            if (depth < P.max_depth) {
                                st |= ST_RAY;
                                P.ray_o[s] = pk(o);
                                P.ray_d[s] = pk(d);
                            } else if (smask) {
                                st |= ST_END;
                            } else {
                                finalize = true;
                            }
                        }
                    }
                }
            }

            // ---- 3. finish the sample, start the next one (Src/renderer.cpp:42-76)
            while (finalize) {
                finalize = false;
                if (st & ST_REGEN) {
                    st &= ~ST_REGEN;
                } else {
                    const v3 r = rad / 1.0f;   // integrate(...) / pdf, pdf = 1
                    if (__builtin_isnan(r.x) || __builtin_isnan(r.y) || __builtin_isnan(r.z) ||
                        __builtin_isinf(r.x) || __builtin_isinf(r.y) || __builtin_isinf(r.z) ||
                        r.x < 0.0f || r.y < 0.0f || r.z < 0.0f) {
                        ++nrej;
                    } else {
                        const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
                        float* px = P.fb + 3 * ((size_t)col + (size_t)P.width * row);
                        px[0] = px[0] + r.x, px[1] = px[1] + r.y, px[2] = px[2] + r.z;
                    }
                    ++k;
                }
                st &= ~(ST_END | ST_RAY);
                if (k >= P.spp) {
                    st = ST_DONE;
                    break;
                }
                // regenerate: jitter draws, camera ray
                const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
                const float u = div_w(P, (float)(int)col + rng.next());
                const float v = div_h(P, (float)(int)row + rng.next());
                camera_ray(P, u, v, o, d);
                thr = mk(1, 1, 1);
                rad = mk(0, 0, 0);
                depth = 0;
                if (!one_hit(INTEG) && P.max_depth == 0) {
                    finalize = true;   // the bounce loop never runs: radiance 0
                    continue;
                }
                st |= ST_RAY;
                P.ray_o[s] = pk(o);
                P.ray_d[s] = pk(d);
            }
            if (st & ST_REGEN) {   // very first sample of the slot
                st &= ~ST_REGEN;
                const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
                const float u = div_w(P, (float)(int)col + rng.next());
                const float v = div_h(P, (float)(int)row + rng.next());
                camera_ray(P, u, v, o, d);
                thr = mk(1, 1, 1);
                rad = mk(0, 0, 0);
                depth = 0;
                if (!one_hit(INTEG) && P.max_depth == 0) {
                    // degenerate: every sample is 0 — finish all of them here
                    while (true) {
                        ++k;
                        if (k >= P.spp) { st = ST_DONE; break; }
                        (void)rng.next(), (void)rng.next();
                    }
                } else {
                    st |= ST_RAY;
                    P.ray_o[s] = pk(o);
                    P.ray_d[s] = pk(d);
                }
            }
            P.state[s] = st;
            P.depth[s] = depth;
            P.sample_k[s] = k;
            P.thr[s] = pk(thr);
            P.rad[s] = pk(rad);
            P.rng_c[s] = rng.c;
            if (nseg) P.c_seg[s] += nseg;
            if (nsh) P.c_shadow[s] += nsh;
            if (nrej) P.c_rej[s] += nrej;
            if (nstall) P.c_stall[s] += nstall;
        }
        // ---- 4. compaction (ballot + prefix count, one atomic per wave), then the wave's
        // refills in-line, overlapping other waves' shading instead of a serial k_refill
        wave_append(valid && !(st & ST_DONE), s, out + it.p * P.part_cap, out_count + it.p, lane);
        wave_refill(P, want_req && !(st & ST_DONE), s, g, lane, rbuf[tid >> 6]);
    }
    (void)req_count;
}


// VolumePathTracingNEE's light sample at a scattering point (Src/integrator.h:539-560):
// sampleDirectionToLight (:586-602, Scene::sampleAreaLight Src/scene.cpp:182-188) and
// isVisible (:604-631) — the shadow ray's closest hit; a surface occludes, a medium
// attenuates by ratio tracking between the hit's t and t1.  Adds
// (thr * tm) * (transmittance * f * Le / pdf) to rad and returns 0, or returns 2 with the
// ratio tracking suspended (state in P.nee, resumed by nee_resume).  Media make a scene
// SCN_MIXED, so other scene kinds never get here.
template <int SCN>
__device__ int nee_medium(const KParams& P, const LScene& L, uint32_t s, v3 pos, v3 wo, v3 thr_m, v3& rad, Rng& rng,
                          uint32_t g, uint32_t& nsh) {
    if (SCN != SCN_MIXED) return 0;
    uint32_t li = (uint32_t)((float)P.n_lights * rng.next());   // size() * getNext1D(), truncated
    if (li == (uint32_t)P.n_lights) li--;
    const float choose = 1.0f / (float)P.n_lights;
    v3 wl = mk(0, 0, 0);
    float lpdf = 0.0f, dist = 0.0f;
    const v3 Le = light_sample(L.light[li], pos, wl, lpdf, dist, rng);
    const float pdf_dir = choose * lpdf;
    if (!(pdf_dir > 0.0f)) return 0;
    ++nsh;
    HitRec h;
    closest_l<SCN>(P, L, pos, wl, h);
    v3 tr = mk(1, 1, 1);
    const float f = hg_eval(P.medium.g, wo, wl);
    if (h.code >= 0) {
        const DObj ob = L.obj[hit_object(L, h)];
        if (ob.material != XRT_MAT_NONE) return 0;   // hasSurface(): occluded
        if (ob.medium >= 0 && P.medium.kind != XRT_MEDIUM_HETEROGENEOUS) {
            // HomogeneousMedium::transmittance (Src/medium.h:133-137)
            const v3 p1 = ray_at(pos, wl, h.t), p2 = ray_at(pos, wl, h.t1);
            tr = tr * analytic_tr(length(p1 - p2), ld3(P.medium.sigma_t));
        } else if (ob.medium >= 0) {
            const v3 p1 = ray_at(pos, wl, h.t), p2 = ray_at(pos, wl, h.t1);
            const float dist_end = length(p1 - p2);
            const v3 dn = normalize(p2 - p1);
            float t = 0.0f;
            if (!ratio_track(P, p1, dn, dist_end, t, tr, rng, g)) {
                const size_t n = P.n_slots;
                P.nee[s] = make_float4(p1.x, p1.y, p1.z, t);
                P.nee[n + s] = make_float4(dn.x, dn.y, dn.z, dist_end);
                P.nee[2 * n + s] = make_float4(tr.x, tr.y, tr.z, f);
                P.nee[3 * n + s] = make_float4(Le.x, Le.y, Le.z, pdf_dir);
                return 2;
            }
        }
    }
    rad = rad + thr_m * (((tr * f) * Le) / pdf_dir);
    return 0;
}

// resume a suspended NEE ratio tracking; thr_m = the path throughput after the scatter
__device__ int nee_resume(const KParams& P, uint32_t s, v3 thr_m, v3& rad, Rng& rng, uint32_t g) {
    const size_t n = P.n_slots;
    const f4 a = P.nee[s], b = P.nee[n + s], c = P.nee[2 * n + s], d = P.nee[3 * n + s];
    float t = a.w;
    v3 tr = xyz(c);
    if (!ratio_track(P, xyz(a), xyz(b), b.w, t, tr, rng, g)) {
        P.nee[s] = make_float4(a.x, a.y, a.z, t);
        P.nee[2 * n + s] = make_float4(tr.x, tr.y, tr.z, c.w);
        return 2;
    }
    rad = rad + thr_m * (((tr * c.w) * xyz(d)) / d.w);
    return 0;
}

// WV: waves per SIMD the register budget is sized for (XRT_KSTEP_WAVES; the volumetric
// integrators also at 2, for launches with too few live slots to fill more: no spills)
template <int SCN, int INTEG, int BS = kBlock, int WV = XRT_KSTEP_WAVES>
__global__ __launch_bounds__(BS, WV) void k_step(KParams P, const uint32_t* __restrict__ list,
                                                  const uint32_t* __restrict__ count, uint32_t* __restrict__ out,
                                                  uint32_t* out_count, uint32_t* zero_count, uint32_t* req_count,
                                                  uint32_t visits) {
    extern __shared__ __attribute__((aligned(16))) f4 lds_step[];
    char* lb = reinterpret_cast<char*>(lds_step);
    const int tid = threadIdx.x;
    const LScene L = load_lscene(P, lb, tid, BS);
    __syncthreads();
    zero_parts(P, zero_count);
    const int lane = tid & 63;
    const PartIter it = part_iter(P, count, BS);
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        const uint32_t s = i < it.n ? list[it.p * P.part_cap + i] : 0;
        uint32_t st = i < it.n ? P.state[s] : ST_DONE;
        bool want_req = false;
        uint32_t g = 0;
        if (!(st & ST_DONE)) {
        g = P.rng_g[s];
        Rng rng{P.ring + (size_t)s * kRing, P.rng_c[s]};
        uint32_t depth = P.depth[s];
        uint32_t k = P.sample_k[s];
        v3 thr = mk(1, 1, 1), rad = mk(0, 0, 0), o = mk(0, 0, 0), d = mk(0, 0, 0);
        if (!(st & ST_REGEN)) {
            thr = xyz(P.thr[s]), rad = xyz(P.rad[s]);
            o = xyz(P.ray_o[s]), d = xyz(P.ray_d[s]);
        }
        uint32_t nseg = 0, nsh = 0, nrej = 0, nstall = 0;
        const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
        float* px = P.fb + 3 * ((size_t)col + (size_t)P.width * row);
        v3 acc = mk(px[0], px[1], px[2]);   // the pixel's running sum, in registers this launch
        rng.prefetch(g - rng.c);
        // VPT family: one event per iteration (kVptEvents) — a trace + surface interaction, or
        // ONE delta-tracking collision of a walk that continues across iterations in
        // registers — so lanes whose walks end early start their next segment (or sample)
        // while the others keep colliding, instead of idling until the wave's longest walk
        // ends.  Each lane's own sequence of operations and draws is unchanged.
        constexpr bool EV = vpt_family(INTEG) && kVptEvents;
        bool walking = false;
        float mt = 0.0f, mt1 = 0.0f;
        v3 tt = mk(1, 1, 1), sa = mk(0, 0, 0);
        for (uint32_t vis = 0; vis < visits; ++vis) {
            if ((st & ST_DONE) || (!walking && g - rng.c < kRngVisit)) break;
            bool ended = false, trace = true;
            if (EV && walking) {
                trace = false;
            } else if (st & ST_REGEN) {
                // next sample: jitter draws + camera ray (Src/renderer.cpp:44-50)
                st &= ~ST_REGEN;
                const float u = div_w(P, (float)(int)col + rng.next());
                const float v = div_h(P, (float)(int)row + rng.next());
                camera_ray(P, u, v, o, d);
                thr = mk(1, 1, 1), rad = mk(0, 0, 0);
                depth = 0;
                if (!one_hit(INTEG) && P.max_depth == 0) ended = true, trace = false;
            } else if (vpt_family(INTEG) && (st & ST_MEDIUM)) {
                trace = false;
            } else if (INTEG == XRT_INTEGRATOR_VPT_NEE && (st & ST_NEEWALK)) {
                // the previous launch suspended this path's NEE ratio tracking
                trace = false;
                if (nee_resume(P, s, thr, rad, rng, g) == 0) {
                    st &= ~ST_NEEWALK;
                    if (depth >= P.max_depth) ended = true;
                    else trace = true;
                }
            }
            bool walk = EV && walking;
            if (!walk) mt = 0.0f, mt1 = 0.0f, tt = mk(1, 1, 1), sa = mk(0, 0, 0);
            if (vpt_family(INTEG) && (st & ST_MEDIUM)) {
                st &= ~ST_MEDIUM;
                const f4 m1 = P.med[s], m2 = P.med2[s];
                mt = m1.x, mt1 = m1.y, sa = mk(m1.z, m1.w, m2.w), tt = xyz(m2);
                walk = true;
            }
            if (trace) {
                ++nseg;
                HitRec h;
                closest_l<SCN>(P, L, o, d, h);
                Surf S;
                const int obj = surface_l<SCN>(L, o, d, h, S);
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    // DirectIntegrator::integrate (Src/integrator.h:82-119)
                    if (obj < 0) {
                        rad = mk((float)0.18, (float)0.18, (float)0.18);
                    } else if (L.obj[obj].light >= 0) {
                        rad = light_Le(L.light[L.obj[obj].light], S.ns, d);
                    } else {
                        const DObj& ob = L.obj[obj];
                        for (int l = 0; l < P.n_lights; ++l) {
                            v3 wi = mk(0, 0, 0);
                            float tmax = 0.0f, pdf = 0.0f;
                            const v3 Lv = light_sample(L.light[l], S.pos, wi, pdf, tmax, rng);
                            if (pdf == 0.0f) continue;
                            const float bias = 0.01f;
                            ++nsh;
                            const bool vis = !occluded_l<SCN>(P, L, S.pos + S.ng * bias, wi, tmax - bias);
                            const float cosv = smax(0.0f, dot(S.ng, wi));
                            const v3 fr = eval_bxdf(ob);
                            rad = rad + div3s(((fr * (float)vis) * Lv) * cosv, pdf);
                        }
                    }
                    ended = true;
                } else if (vpt_family(INTEG)) {
                    // VolumePathTracing::integrate loop body (Src/integrator.h:418-469);
                    // VolumePathTracingNEE (:497-581): Le only at depth 0
                    if (obj < 0) {
                        rad = rad + (thr * mk(0.0f, 0.0f, 0.0f)) * (float)(depth != 0);
                        ended = true;
                    } else {
                        bool alive = true;
                        if (depth > 0) {
                            const float pr = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
                            if (rng.next() >= pr) alive = false, ended = true;
                            else thr = div3s(thr, pr);   // thr / Vec3f(pr): one division when achromatic
                        }
                        const DObj& ob = L.obj[obj];
                        if (alive && ob.light >= 0) {
                            if (INTEG == XRT_INTEGRATOR_VPT || depth == 0)
                                rad = rad + thr * light_Le(L.light[ob.light], S.ns, d);
                            alive = false, ended = true;
                        }
                        if (alive) {
                            if (ob.medium >= 0) {
                                mt = h.t, mt1 = h.t1;
                                if (P.medium.kind == XRT_MEDIUM_HETEROGENEOUS)
                                    sa = ld3(P.medium.absorption) * medium_density(P.medium, ray_at(o, d, mt));
                                walk = true;
                            } else {
                                ++nstall;   // see k_shade: the reference never advances this ray
                                ended = true;
                            }
                        }
                    }
                } else if (INTEG == XRT_INTEGRATOR_NORMAL) {
                    // NormalIntegrator::integrate (Src/integrator.h:28-37): 0.5 * (ns + 1)
                    if (obj >= 0) rad = normal_color(S.ns);
                    ended = true;
                } else {
                    // GIIntegrator::integrate loop body (Src/integrator.h:214-284);
                    // IndirectIntegrator (Src/integrator.h:138-185): no light sampling, Le at
                    // every depth
                    if (obj < 0) {
                        rad = rad + thr * mk(0.0f, 0.0f, 0.0f);
                        ended = true;
                    } else {
                        bool alive = true;
                        if (depth > 0) {
                            const float pr = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
                            if (rng.next() >= pr) alive = false, ended = true;
                            else thr = thr / mk(pr, pr, pr);
                        }
                        const DObj& ob = L.obj[obj];
                        if (alive && ob.light >= 0) {
                            if (depth == 0 || INTEG == XRT_INTEGRATOR_INDIRECT)
                                rad = rad + thr * light_Le(L.light[ob.light], S.ns, d);
                            alive = false, ended = true;
                        }
                        if (alive) {
                            v3 directL = mk(0, 0, 0);
                            for (int l = 0; l < (INTEG == XRT_INTEGRATOR_GI ? P.n_lights : 0); ++l) {
                                v3 L_light = mk(0, 0, 0);
                                v3 wi = mk(0, 0, 0);
                                float tmax = 0.0f, pdf = 0.0f;
                                const v3 Lv = light_sample(L.light[l], S.pos, wi, pdf, tmax, rng);
                                if (pdf == 0.0f) continue;
                                const float bias = 0.01f;
                                ++nsh;
                                const bool vis = !occluded_l<SCN>(P, L, S.pos + S.ng * bias, wi, tmax - bias);
                                const float cosv = smax(0.0f, dot(S.ng, wi));
                                const v3 fr = eval_bxdf(ob);
                                L_light = L_light + (((fr * (float)vis) * Lv) * cosv) / pdf;
                                directL = directL + L_light;
                            }
                            if (INTEG == XRT_INTEGRATOR_GI) rad = rad + thr * directL;
                            float pdf = 1.0f;
                            v3 nd = mk(0, 0, 0), fr = mk(0, 0, 0);
                            if (ob.material == 1) {
                                nd = lambert_sample(S, rng);
                                pdf = 1.0f / (2.0f * kPI);
                                fr = eval_bxdf(ob);
                            }
                            const float cosv = smax(0.0f, dot(nd, S.ng));
                            thr = thr * ((fr * cosv) / pdf);
                            o = S.pos + S.ng * 0.01f;
                            d = nd;
                            ++depth;
                            if (depth >= P.max_depth) ended = true;
                        }
                    }
                }
            }
            if (vpt_family(INTEG) && walk) {
                v3 pos, dir, tm;
                const int r = P.medium.kind != XRT_MEDIUM_HETEROGENEOUS
                                  ? homog_track(P, o, d, thr, mt, mt1, rng, pos, dir, tm)
                              : EV ? delta_step(P, o, d, thr, mt, mt1, tt, sa, rng, g, pos, dir, tm)
                                   : delta_track(P, o, d, thr, mt, mt1, tt, sa, rng, g, pos, dir, tm);
                walking = EV && r == 3;   // null collision: the walk goes on next iteration
                if (r == 3) {
                } else if (r == 2) {
                    st |= ST_MEDIUM;
                    P.med[s] = make_float4(mt, mt1, sa.x, sa.y);
                    P.med2[s] = make_float4(tt.x, tt.y, tt.z, sa.z);
                } else {
                    // VolumePathTracingNEE: light sample at a scattering event, before the
                    // ray advances (Src/integrator.h:537-572)
                    const int nr = (INTEG == XRT_INTEGRATOR_VPT_NEE && r == 1)
                                       ? nee_medium<SCN>(P, L, s, pos, d, thr * tm, rad, rng, g, nsh)
                                       : 0;
                    o = pos, d = dir;
                    thr = thr * tm;
                    if (r == 1) ++depth;
                    if (nr == 2) st |= ST_NEEWALK;   // resumes at the next launch (RNG words ran out)
                    else if (depth >= P.max_depth) ended = true;
                }
            }
            // finish the sample (Src/renderer.cpp:55-75) and start the next one right away:
            // its jitter draws are still in the prefetch buffer (a segment draws <= 13 of the
            // >= 16 words it starts with), so the next segment opens with the trace while
            // the words it needs next are loading.
            while (ended) {
                ended = false;
                const v3 r = rad / 1.0f;
                if (__builtin_isnan(r.x) || __builtin_isnan(r.y) || __builtin_isnan(r.z) || __builtin_isinf(r.x) ||
                    __builtin_isinf(r.y) || __builtin_isinf(r.z) || r.x < 0.0f || r.y < 0.0f || r.z < 0.0f) {
                    ++nrej;
                } else {
                    acc = acc + r;
                }
                ++k;
                if (k >= P.spp) {
                    st = ST_DONE;
                } else if (!one_hit(INTEG) && P.max_depth == 0) {
                    (void)rng.next(), (void)rng.next();   // the next sample's jitter; radiance 0
                    rad = mk(0, 0, 0);
                    ended = true;
                } else {
                    const float u = div_w(P, (float)(int)col + rng.next());
                    const float v = div_h(P, (float)(int)row + rng.next());
                    camera_ray(P, u, v, o, d);
                    thr = mk(1, 1, 1), rad = mk(0, 0, 0);
                    depth = 0;
                }
            }
            if (!EV || rng.nb < kVptEventPrefetch) rng.prefetch(g - rng.c);
        }
        if (EV && walking) {   // the launch ended mid-walk: resume it like a suspended one
            st |= ST_MEDIUM;
            P.med[s] = make_float4(mt, mt1, sa.x, sa.y);
            P.med2[s] = make_float4(tt.x, tt.y, tt.z, sa.z);
        }
        px[0] = acc.x, px[1] = acc.y, px[2] = acc.z;
        // RNG refill (words ahead < rng_keep <= 624): twisted by this wave below
        want_req = !(st & (ST_DONE | ST_RNGREQ)) && g - rng.c < P.rng_keep;
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
        if (nstall) P.c_stall[s] += nstall;
        }
        // live list of the next round (partitioned, one atomic per wave), then the wave's
        // refills in-line (as k_step_merged: no k_refill launch between step launches)
        wave_append(!(st & ST_DONE), s, out + it.p * P.part_cap, out_count + it.p, lane);
        if (kstep_refill_off(P, BS)) {   // wave_refill staging: the wave's kMT words after the scene
            uint32_t* rbuf = reinterpret_cast<uint32_t*>(lb + kstep_refill_off(P, BS)) + (tid >> 6) * kMT;
            wave_refill(P, want_req, s, g, lane, rbuf);
        } else {
            // sphere-BVH scenes: twisted from global memory (L2), no LDS buffer beside the
            // scene's ~45 KB (3 blocks per CU instead of 2)
            uint32_t gn = g;
            wave_refill(want_req, s, gn, P.ring, lane);
            if (want_req) P.rng_g[s] = gn;
        }
    }
    (void)req_count;
}

// ======================================================= cooperative triangle trace ====
// For triangle scenes the rays of a wave are incoherent after the first bounce: tracing one
// ray per lane, a wave pays for every object any of its 64 rays needs (measured on C2:
// ~29 triangle tests per wave per trace while a ray needs ~5).  The cooperative trace
// instead culls each ray against the object boxes, lays the (ray, triangle) pairs that
// survive out in one flat index space (exclusive scan over the lanes; each lane writes its
// pairs into an LDS list, 512 per chunk) and tests 64 pairs per pass — every lane busy.  Results are merged per ray in LDS: closest hit = atomicMin
// of (t bits << 32 | triangle index), i.e. smallest t and, on a tie, the triangle the
// reference's in-order `t < best` loop keeps (triangles are packed in Scene iteration
// order); then the owner lane recomputes u, v of its winner with the same Moller-Trumbore
// ops.  Shadow rays set an occlusion flag.  Requires n_objs <= 32 (object masks).
struct CoopWave {
    f4 ro[64];                     // ray origin, w = tmax (shadow rays)
    f4 rd[64];
    unsigned long long best[64];   // closest: packed (t, tri); shadow: != 0 occluded
    uint32_t pair[512];            // expanded pairs of the current chunk: owner << 24 | tri
};
constexpr int kCoopMaxObjs = 32;
constexpr uint32_t kCoopCap = 512;

template <bool SHADOW>
__device__ __forceinline__ unsigned long long coop_trace(const KParams& P, const LScene& L, CoopWave& W, int lane,
                                                         bool want, v3 o, v3 d, float tmax) {
    uint32_t m = 0, n = 0;
    if (want) {
        const v3 inv = rcp3(d);
        for (int ob = 0; ob < P.n_objs; ++ob) {
            const DObjBox B = L.box[ob];
            if (SHADOW && B.count_occ >= 0) continue;   // area-light objects never occlude
            if (box_overlap(o, inv, B, SHADOW ? tmax : kINF)) m |= 1u << ob, n += B.count_occ & 0x7fffffff;
        }
    }
    uint32_t incl = n;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
    }
    const uint32_t total = __shfl(incl, 63);
    const uint32_t pre = incl - n;
    W.ro[lane] = make_float4(o.x, o.y, o.z, tmax);
    W.rd[lane] = make_float4(d.x, d.y, d.z, 0.0f);
    W.best[lane] = SHADOW ? 0ull : ~0ull;
    for (uint32_t c0 = 0; c0 < total; c0 += kCoopCap) {
        // expand this lane's pairs that fall into the chunk [c0, c0 + kCoopCap)
        if (n && pre < c0 + kCoopCap && pre + n > c0) {
            uint32_t pos = pre, mm = m;
            while (mm) {
                const int ob = __builtin_ctz(mm);
                mm &= mm - 1;
                const DObjBox B = L.box[ob];
                const uint32_t c = B.count_occ & 0x7fffffff;
                const uint32_t lo = max(pos, c0), hi = min(pos + c, c0 + kCoopCap);
                for (uint32_t q = lo; q < hi; ++q) W.pair[q - c0] = ((uint32_t)lane << 24) | (B.first + (q - pos));
                pos += c;
            }
        }
        wave_sync();
        const uint32_t cnt = min(kCoopCap, total - c0);
        for (uint32_t j = lane; j < cnt; j += 64) {
            const uint32_t e = W.pair[j];
            const int r = (int)(e >> 24), k = (int)(e & 0xffffffu);
            const f4 A = W.ro[r];
            float t, u, v;
            if (ray_tri(xyz(A), xyz(W.rd[r]), xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u,
                        v)) {
                if (SHADOW) {
                    if (t < A.w) W.best[r] = 1ull;
                } else {
                    atomicMin(&W.best[r], ((unsigned long long)__float_as_uint(t) << 32) | (uint32_t)k);
                }
            }
        }
        wave_sync();
    }
    return W.best[lane];
}

__device__ __forceinline__ void coop_closest(const KParams& P, const LScene& L, CoopWave& W, int lane, bool want, v3 o,
                                             v3 d, HitRec& h) {
    const unsigned long long b = coop_trace<false>(P, L, W, lane, want, o, d, kINF);
    h.t = kINF, h.u = h.v = 0.0f, h.code = -1, h.surf = -1, h.dp = -1, h.t1 = kINF;
    h.st = h.su = h.sv = h.du = h.dv = 0.0f;
    if (want && b != ~0ull) {
        const int k = (int)(uint32_t)b;
        float t, u, v;
        (void)ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v);
        h.t = t, h.u = u, h.v = v, h.code = k;
    }
}

// k_step for triangle scenes (GI / Direct) with cooperative traces: the same per-slot
// sequence as k_step, arranged so every trace is reached by the whole wave (per-lane
// activity flags instead of divergent control flow around the traces).
template <int INTEG>
__global__ __launch_bounds__(kBlock, XRT_STEP_WAVES) void k_step_tri(const KParams* __restrict__ Pp,
                                                                      const uint32_t* __restrict__ list,
                                                                      const uint32_t* __restrict__ count,
                                                                      uint32_t* __restrict__ out, uint32_t* out_count,
                                                                      uint32_t* zero_count, uint32_t* req_count,
                                                                      uint32_t visits) {
    // KParams lives in device memory here (one copy per render): fields are fetched with
    // scalar loads when needed instead of pinning ~150 SGPRs of kernel arguments
    const KParams& P = *Pp;
    extern __shared__ __attribute__((aligned(16))) f4 lds_step[];
    char* lb = reinterpret_cast<char*>(lds_step);
    const StepLayout Lo = step_layout(P);
    LScene L;
    L.tri = reinterpret_cast<const f4*>(lb + Lo.tri);
    L.tng = reinterpret_cast<const f4*>(lb + Lo.tng);
    L.nrm = reinterpret_cast<const f4*>(lb + Lo.nrm);
    L.box = reinterpret_cast<const DObjBox*>(lb + Lo.box);
    L.sph = reinterpret_cast<const f4*>(lb + Lo.sph);
    L.bx = reinterpret_cast<const f4*>(lb + Lo.bx);
    L.obj = reinterpret_cast<const DObj*>(lb + Lo.obj);
    L.light = reinterpret_cast<const DLight*>(lb + Lo.light);
    L.sobj = reinterpret_cast<const int*>(lb + Lo.sobj);
    const int tid = threadIdx.x, lane = tid & 63;
    CoopWave& W = reinterpret_cast<CoopWave*>(lb + ((Lo.total + 15u) & ~15u))[tid >> 6];
    lds_copy(const_cast<f4*>(L.tri), P.tri, 3 * P.n_tris, tid);
    lds_copy(const_cast<f4*>(L.tng), P.tri_ng, P.n_tris, tid);
    lds_copy(const_cast<f4*>(L.nrm), P.tri_nrm, 3 * P.n_tris, tid);
    lds_copy(const_cast<DObjBox*>(L.box), P.obj_box, P.n_objs, tid);
    lds_copy(const_cast<DObj*>(L.obj), P.objs, P.n_objs, tid);
    lds_copy(const_cast<DLight*>(L.light), P.lights, P.n_lights, tid);
    __syncthreads();
    zero_parts(P, zero_count);
    const PartIter it = part_iter(P, count, kBlock);
    for (uint32_t base = it.first; base < it.n; base += it.stride) {
        const uint32_t i = base + tid;
        const uint32_t s = i < it.n ? list[it.p * P.part_cap + i] : 0;
        uint32_t st = i < it.n ? P.state[s] : ST_DONE;
        const bool live = !(st & ST_DONE);
        uint32_t g = 0, depth = 0, k = 0;
        Rng rng{P.ring + (size_t)s * kRing, 0};
        v3 thr = mk(1, 1, 1), rad = mk(0, 0, 0), o = mk(0, 0, 0), d = mk(0, 0, 0), acc = mk(0, 0, 0);
        const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
        float* px = P.fb + 3 * ((size_t)col + (size_t)P.width * row);
        if (live) {
            g = P.rng_g[s];
            rng.c = P.rng_c[s];
            depth = P.depth[s];
            k = P.sample_k[s];
            if (!(st & ST_REGEN)) {
                thr = xyz(P.thr[s]), rad = xyz(P.rad[s]);
                o = xyz(P.ray_o[s]), d = xyz(P.ray_d[s]);
            }
            acc = mk(px[0], px[1], px[2]);
            rng.prefetch(g - rng.c);
        }
        uint32_t nseg = 0, nsh = 0, nrej = 0;
        for (uint32_t vis = 0; vis < visits; ++vis) {
            const bool act = live && !(st & ST_DONE) && g - rng.c >= kRngVisit;
            if (!__ballot(act)) break;
            if (act && (st & ST_REGEN)) {
                // first sample of the slot: jitter draws + camera ray (Src/renderer.cpp:44-50)
                st &= ~ST_REGEN;
                const float u = div_w(P, (float)(int)col + rng.next());
                const float v = div_h(P, (float)(int)row + rng.next());
                camera_ray(P, u, v, o, d);
                thr = mk(1, 1, 1), rad = mk(0, 0, 0);
                depth = 0;
            }
            bool ended = false, alive = false;
            if (!one_hit(INTEG) && P.max_depth == 0) ended = act;   // bounce loop never runs
            const bool ext = act && !ended;
            HitRec h;
            coop_closest(P, L, W, lane, ext, o, d, h);
            // SurfaceInfo of a triangle hit: position, face normal; the shading normal (for
            // Le) and the dpdu/dpdv frame (for the BSDF) are rebuilt from (tri, u, v) where used
            Surf S;
            S.pos = S.ng = S.ns = S.dpdu = S.dpdv = mk(0, 0, 0);
            int obj = -1;
            const int hk = h.code;
            const float hu = h.u, hv = h.v;
            if (ext) {
                ++nseg;
                if (hk >= 0) {
                    S.pos = ray_at(o, d, h.t);
                    S.ng = xyz(L.tng[hk]);
                    obj = __float_as_int(L.tri[3 * hk].w);
                }
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    // DirectIntegrator::integrate (Src/integrator.h:82-119)
                    if (obj < 0) {
                        rad = mk((float)0.18, (float)0.18, (float)0.18);
                        ended = true;
                    } else if (L.obj[obj].light >= 0) {
                        rad = light_Le(L.light[L.obj[obj].light], tri_ns_l(L, hk, hu, hv), d);
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
                            const float pr = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
                            if (rng.next() >= pr) alive = false, ended = true;
                            else thr = thr / mk(pr, pr, pr);
                        }
                        if (alive && L.obj[obj].light >= 0) {
                            if (depth == 0)
                                rad = rad + thr * light_Le(L.light[L.obj[obj].light], tri_ns_l(L, hk, hu, hv), d);
                            alive = false, ended = true;
                        }
                    }
                }
            }
            // next-event estimation: one cooperative shadow trace per light, in light order
            v3 directL = mk(0, 0, 0);
            for (int l = 0; l < P.n_lights; ++l) {
                v3 wi = mk(0, 0, 0), Lv = mk(0, 0, 0);
                float tmax = 0.0f, pdf = 0.0f;
                if (alive) Lv = light_sample(L.light[l], S.pos, wi, pdf, tmax, rng);
                const bool sh = alive && pdf != 0.0f;
                const float bias = 0.01f;
                const bool occ = coop_trace<true>(P, L, W, lane, sh, S.pos + S.ng * bias, wi, tmax - bias) != 0;
                if (sh) {
                    ++nsh;
                    const float cosv = smax(0.0f, dot(S.ng, wi));
                    const v3 fr = eval_bxdf(L.obj[obj]);
                    const v3 c = (((fr * (float)!occ) * Lv) * cosv) / pdf;
                    if (INTEG == XRT_INTEGRATOR_DIRECT) {
                        rad = rad + c;
                    } else {
                        const v3 L_light = mk(0, 0, 0) + c;
                        directL = directL + L_light;
                    }
                }
            }
            if (alive) {
                if (INTEG == XRT_INTEGRATOR_DIRECT) {
                    ended = true;
                } else {
                    rad = rad + thr * directL;
                    const DObj& ob = L.obj[obj];
                    float pdf = 1.0f;
                    v3 nd = mk(0, 0, 0), fr = mk(0, 0, 0);
                    if (ob.material == 1) {
                        v3 dpdu, dpdv;
                        onb(tri_ns_l(L, hk, hu, hv), dpdu, dpdv);
                        nd = lambert_sample_f(S.ng, dpdu, dpdv, rng);
                        pdf = 1.0f / (2.0f * kPI);
                        fr = eval_bxdf(ob);
                    }
                    const float cosv = smax(0.0f, dot(nd, S.ng));
                    thr = thr * ((fr * cosv) / pdf);
                    o = S.pos + S.ng * 0.01f;
                    d = nd;
                    ++depth;
                    if (depth >= P.max_depth) ended = true;
                }
            }
            // finish the sample and start the next one (see k_step)
            while (ended) {
                ended = false;
                const v3 r = rad / 1.0f;
                if (__builtin_isnan(r.x) || __builtin_isnan(r.y) || __builtin_isnan(r.z) || __builtin_isinf(r.x) ||
                    __builtin_isinf(r.y) || __builtin_isinf(r.z) || r.x < 0.0f || r.y < 0.0f || r.z < 0.0f) {
                    ++nrej;
                } else {
                    acc = acc + r;
                }
                ++k;
                if (k >= P.spp) {
                    st = ST_DONE;
                } else if (!one_hit(INTEG) && P.max_depth == 0) {
                    (void)rng.next(), (void)rng.next();
                    rad = mk(0, 0, 0);
                    ended = true;
                } else {
                    const float u = div_w(P, (float)(int)col + rng.next());
                    const float v = div_h(P, (float)(int)row + rng.next());
                    camera_ray(P, u, v, o, d);
                    thr = mk(1, 1, 1), rad = mk(0, 0, 0);
                    depth = 0;
                }
            }
            if (act) rng.prefetch(g - rng.c);
        }
        bool want_req = false;
        if (live) {
            px[0] = acc.x, px[1] = acc.y, px[2] = acc.z;
            want_req = !(st & (ST_DONE | ST_RNGREQ)) && g - rng.c < P.rng_keep;   // twisted below
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
        wave_append(live && !(st & ST_DONE), s, out + it.p * P.part_cap, out_count + it.p, lane);
        // the wave's refills in-line through its trace scratch (idle now)
        static_assert(sizeof(CoopWave) >= kMT * sizeof(uint32_t), "refill staging");
        wave_refill(P, want_req, s, g, lane, reinterpret_cast<uint32_t*>(&W));
    }
    (void)req_count;
}

// ================================================================== k_finish ====
// Image::operator/=(Vec3f(n_samples)) over this shard's pixels + counter reduction.
__global__ __launch_bounds__(kBlock) void k_finish(KParams P) {
    __shared__ unsigned long long red[6][kBlock / 64];
    unsigned long long a[6] = {0, 0, 0, 0, 0, 0};
    const float n = (float)P.spp;
    for (uint32_t s = blockIdx.x * kBlock + threadIdx.x; s < P.n_slots; s += gridDim.x * kBlock) {
        const uint32_t col = s % P.width, row = P.shard_index + P.shard_count * (s / P.width);
        float* px = P.fb + 3 * ((size_t)col + (size_t)P.width * row);
        px[0] = px[0] / n, px[1] = px[1] / n, px[2] = px[2] / n;
        a[0] += P.c_seg[s];
        a[1] += P.c_shadow[s];
        a[2] += P.rng_c[s] - kMT;
        a[3] += P.c_rej[s];
        a[4] += P.c_stall[s];
        a[5] += P.rng_g[s] / kMT - 1u;   // twists: k_seed leaves g = kMT, every twist adds kMT
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        unsigned long long v = a[q];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
        if (lane == 0) red[q][wv] = v;
    }
    __syncthreads();
    if (threadIdx.x < 6) {   // stats[0..4], twists to stats[7] (5, 6: experiment counters)
        unsigned long long v = 0;
        for (int w = 0; w < kBlock / 64; ++w) v += red[threadIdx.x][w];
        atomicAdd(P.stats + (threadIdx.x < 5 ? threadIdx.x : 7u), v);
    }
}

// ============================================================== self-tests ====
__global__ __launch_bounds__(kBlock) void k_test_rng(const uint32_t* seeds, uint32_t n_seeds, uint32_t skip,
                                                      uint32_t n, float* out, uint32_t* rings) {
    const int lane = threadIdx.x & 63;
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    const bool valid = s < n_seeds;
    uint32_t* ring = rings + (size_t)s * kRing;
    if (valid) {
        uint32_t x = seeds[s];
        ring[0] = x;
        for (uint32_t i = 1; i < kMT; ++i) {
            x = 1812433253u * (x ^ (x >> 30)) + i;
            ring[i] = x;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    uint32_t g = kMT;
    Rng rng{ring, kMT};
    // consume skip + n draws, refilling cooperatively like k_shade does
    const uint32_t total = skip + n;
    for (uint32_t done = 0; done < total;) {
        wave_refill(valid && (g - rng.c) < kRngMin, s, g, rings, lane);
        const uint32_t chunk = min(32u, total - done);   // < kRngMin: never reads past g
        if (valid) {
            for (uint32_t q = 0; q < chunk; ++q) {
                const uint32_t idx = done + q;
                const float f = rng.next();
                if (idx >= skip) out[(size_t)s * n + (idx - skip)] = f;
            }
        }
        done += chunk;
    }
}

__global__ void k_test_trig(const float* x, uint32_t n, float* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        out[2 * i] = glibc_sinf(x[i]);
        out[2 * i + 1] = glibc_cosf(x[i]);
    }
}

// every float r in [0,1) with bit pattern in [first, first+count) that the sampler can
// produce (r * 2^32 integral): phi = 2*PI*r -> (sin, cos); others -> NaN marker in out_r
__global__ void k_test_trig_domain(uint32_t first, uint32_t count, float* out_sin, float* out_cos, float* out_r) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float r = __uint_as_float(first + i);
    const double sc = (double)r * 4294967296.0;
    const bool reach = r >= 0.0f && r < 1.0f && sc == __builtin_floor(sc);
    const float phi = kPI_MUL_2 * r;
    out_r[i] = reach ? r : __builtin_nanf("");
    out_sin[i] = glibc_sinf(phi);
    out_cos[i] = glibc_cosf(phi);
}

// fast-division self-test over every 32-bit pattern in [first, first + count): mode 0 checks
// rcp_rn(b) against 1.0f / b; mode 1 checks div_const(x, c, rc) against x / c.  Counts
// mismatches (NaN == NaN) and records the first 16.
__global__ void k_test_fastdiv(uint32_t mode, float c, float rc, uint32_t first, uint32_t count,
                               unsigned long long* nbad, uint32_t* bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float x = __uint_as_float(first + i);
    float f, r;
    if (mode == 0) {
        f = rcp_rn(x);
        r = 1.0f / x;
    } else {
        f = div_const(x, c, rc);
        r = x / c;
    }
    const bool same = __float_as_uint(f) == __float_as_uint(r) || (f != f && r != r);
    if (!same) {
        const unsigned long long k = atomicAdd(nbad, 1ull);
        if (k < 16) bad[k] = first + i;
    }
}

__global__ void k_test_logexp(const float* x, uint32_t n, float* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        out[2 * i] = glibc_logf(x[i]);
        out[2 * i + 1] = glibc_expf(x[i]);
    }
}

__global__ void k_test_powf(const float* x, uint32_t n, float y, float* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = glibc_powf(x[i], y);
}

// ===================================================================== output ====
// Image::gammaCorrection (Src/image.h:80-90: pow(c, 1.0f / gamma) per channel) followed by
// writePPM's quantisation (:92-114: std::clamp(static_cast<uint32_t>(255.0f * c), 0u, 255u)),
// the float -> uint32 conversion as GCC emits it on x86-64 (a 64-bit truncating convert,
// INT64_MIN for NaN and out-of-range values, low 32 bits kept).  One thread per channel.
__global__ void k_tonemap(const float* __restrict__ rgb, uint32_t n, float inv_gamma, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = 255.0f * glibc_powf(rgb[i], inv_gamma);
    const int64_t q = (v >= -0x1p63f && v < 0x1p63f) ? (int64_t)v : INT64_MIN;
    const uint32_t u = (uint32_t)(uint64_t)q;
    out[i] = (uint8_t)(u < 255u ? u : 255u);
}

// ================================================================== launchers ====
}  // namespace xrt

#include "launch.h"

namespace xrt {

hipError_t launch_seed(const KParams& P, uint32_t* list, uint32_t* count, uint32_t* count_other,
                       uint32_t* req_count, hipStream_t st) {
    const uint32_t blocks = (P.n_slots + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_seed, dim3(blocks), dim3(kBlock), 0, st, P, list, count, count_other, req_count);
    return hipGetLastError();
}


template <int SCN>
static hipError_t trace_nl(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* zero,
                           uint32_t blocks, hipStream_t st) {
    if (P.n_lights <= 1)
        hipLaunchKernelGGL((k_trace<SCN, 1>), dim3(blocks), dim3(kBlock), 0, st, P, list, count, zero);
    else
        hipLaunchKernelGGL((k_trace<SCN, kMaxLights>), dim3(blocks), dim3(kBlock), 0, st, P, list, count, zero);
    return hipGetLastError();
}

// Phase B of the two-level trace (P.two_level): the 4-wide BVH walk of the rays phase A
// queued.  Persistent: up to 2048 blocks (8 per CU), each serving partition blockIdx % n_part.
// A no-op for every other trace.
hipError_t launch_trace_deep(const KParams& P, hipStream_t st) {
    if (!(P.bvh_node && P.scene_kind == SCN_TRI && P.two_level)) return hipSuccess;
    if (!P.bvh4 || P.bvh4_stack <= 0 || P.bvh4_stack > kBvh4Stack) return hipErrorInvalidValue;
    const uint32_t db = P.n_part * std::max<uint32_t>(1u, std::min<uint32_t>(2048u / P.n_part,
                                                                            (P.deep_cap + kBlock - 1) / kBlock));
    const bool small4 = P.bvh4_nodes <= 0x10000;
    const size_t ntop4 = std::min<size_t>((size_t)P.bvh4_nodes, kBvhTopNodes);
    const size_t lds4 = ntop4 * 8 * sizeof(f4) + (size_t)P.bvh4_stack * kBlock * (small4 ? sizeof(uint16_t) : sizeof(uint32_t));
    if (P.deep_quad) {   // four lanes per ray: one stack per quad
        const size_t lds4q = ntop4 * 8 * sizeof(f4) +
                             (size_t)P.bvh4_stack * (kBlock / 4) * (small4 ? sizeof(uint16_t) : sizeof(uint32_t));
        if (small4) hipLaunchKernelGGL((k_trace_deep4q<uint16_t>), dim3(db), dim3(kBlock), lds4q, st, P);
        else hipLaunchKernelGGL((k_trace_deep4q<uint32_t>), dim3(db), dim3(kBlock), lds4q, st, P);
        return hipGetLastError();
    }
    if (small4) hipLaunchKernelGGL((k_trace_deep4<uint16_t>), dim3(db), dim3(kBlock), lds4, st, P);
    else hipLaunchKernelGGL((k_trace_deep4<uint32_t>), dim3(db), dim3(kBlock), lds4, st, P);
    return hipGetLastError();
}

hipError_t launch_trace(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* zero,
                        uint32_t blocks, hipStream_t st, bool zero_deep) {
    if (P.bvh_node && P.scene_kind == SCN_TRI) {
        if (P.bvh_stack <= 0 || P.bvh_stack > kBvhStack) return hipErrorInvalidValue;
        // node indices below 2^16: 16-bit stack entries, half the LDS per thread
        const bool small = P.bvh_nodes <= 0x10000;
        const size_t ntop = std::min<size_t>((size_t)P.bvh_nodes, kBvhTopNodes);
        const size_t lds = ntop * 4 * sizeof(f4) + (size_t)P.bvh_stack * kBlock * (small ? sizeof(uint16_t) : sizeof(uint32_t));
        const bool nl1 = P.n_lights <= 1;
        if (P.two_level) {
            if (!P.deep || !P.deep_count) return hipErrorInvalidValue;
            hipError_t e = zero_deep ? hipMemsetAsync(P.deep_count, 0, 3 * kMaxParts * sizeof(uint32_t), st)   // counts,
                                     : hipSuccess;                                                        // fetch counters
            if (e != hipSuccess) return e;
            const size_t lds_a = (size_t)P.n_stri * 3 * sizeof(f4) + (size_t)P.n_sobj * (sizeof(DObjBox) + sizeof(DObjPlane));
            if (P.sstep)
                e = launch_trace_2a_coop(P, list, count, zero, blocks, st);
            else if (nl1)
                hipLaunchKernelGGL((k_trace_2a<1>), dim3(blocks), dim3(kBlock), lds_a, st, P, list, count, zero);
            else
                hipLaunchKernelGGL((k_trace_2a<kMaxLights>), dim3(blocks), dim3(kBlock), lds_a, st, P, list, count, zero);
            if (e == hipSuccess) e = hipGetLastError();
            return e;   // phase B: launch_trace_deep
        }
        if (small && nl1)
            hipLaunchKernelGGL((k_trace_bvh<1, uint16_t>), dim3(blocks), dim3(kBlock), lds, st, P, list, count, zero);
        else if (small)
            hipLaunchKernelGGL((k_trace_bvh<kMaxLights, uint16_t>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                               zero);
        else if (nl1)
            hipLaunchKernelGGL((k_trace_bvh<1, uint32_t>), dim3(blocks), dim3(kBlock), lds, st, P, list, count, zero);
        else
            hipLaunchKernelGGL((k_trace_bvh<kMaxLights, uint32_t>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                               zero);
        return hipGetLastError();
    }
    if (P.small_tri) {
        const size_t lds = (size_t)P.n_tris * 3 * sizeof(f4) + (size_t)P.n_objs * sizeof(DObjBox);
        if (P.n_lights <= 1)
            hipLaunchKernelGGL((k_trace_small<1>), dim3(blocks), dim3(kBlock), lds, st, P, list, count, zero);
        else
            hipLaunchKernelGGL((k_trace_small<kMaxLights>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                               zero);
        return hipGetLastError();
    }
    switch (P.scene_kind) {
        case SCN_TRI: return trace_nl<SCN_TRI>(P, list, count, zero, blocks, st);
        case SCN_SPHERE: return trace_nl<SCN_SPHERE>(P, list, count, zero, blocks, st);
        default: return trace_nl<SCN_MIXED>(P, list, count, zero, blocks, st);
    }
}

template <int SCN>
static hipError_t shade_i(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* out,
                          uint32_t* out_count, uint32_t* req_count, uint32_t blocks, hipStream_t st) {
    if (P.integrator == XRT_INTEGRATOR_DIRECT)
        hipLaunchKernelGGL((k_shade<SCN, XRT_INTEGRATOR_DIRECT>), dim3(blocks), dim3(kBlock), 0, st, P, list,
                           count, out, out_count, req_count);
    else if (P.integrator == XRT_INTEGRATOR_VPT)
        hipLaunchKernelGGL((k_shade<SCN, XRT_INTEGRATOR_VPT>), dim3(blocks), dim3(kBlock), 0, st, P, list, count,
                           out, out_count, req_count);
    else if (P.integrator == XRT_INTEGRATOR_INDIRECT)
        hipLaunchKernelGGL((k_shade<SCN, XRT_INTEGRATOR_INDIRECT>), dim3(blocks), dim3(kBlock), 0, st, P, list, count,
                           out, out_count, req_count);
    else if (P.integrator == XRT_INTEGRATOR_NORMAL)
        hipLaunchKernelGGL((k_shade<SCN, XRT_INTEGRATOR_NORMAL>), dim3(blocks), dim3(kBlock), 0, st, P, list, count,
                           out, out_count, req_count);
    else if (P.integrator == XRT_INTEGRATOR_VPT_NEE)
        hipLaunchKernelGGL((k_shade<SCN, XRT_INTEGRATOR_VPT_NEE>), dim3(blocks), dim3(kBlock), 0, st, P, list, count,
                           out, out_count, req_count);
    else
        hipLaunchKernelGGL((k_shade<SCN, XRT_INTEGRATOR_GI>), dim3(blocks), dim3(kBlock), 0, st, P, list, count,
                           out, out_count, req_count);
    return hipGetLastError();
}

hipError_t launch_shade(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* out,
                        uint32_t* out_count, uint32_t* req_count, uint32_t blocks, hipStream_t st) {
    switch (P.scene_kind) {
        case SCN_TRI: return shade_i<SCN_TRI>(P, list, count, out, out_count, req_count, blocks, st);
        case SCN_SPHERE: return shade_i<SCN_SPHERE>(P, list, count, out, out_count, req_count, blocks, st);
        default: return shade_i<SCN_MIXED>(P, list, count, out, out_count, req_count, blocks, st);
    }
}

size_t step_lds_bytes(const KParams& P) {
    if (P.scene_kind == SCN_TRI && !P.small_tri) return 0;   // needs the per-object boxes
    if (P.n_tris > 65536 || P.n_sph > 65536 || P.n_box > 65536 || P.n_objs > 65536) return 0;
    const size_t total = step_layout(P).total;
    return total <= kStepLds ? (total + 15) / 16 * 16 : 0;
}

// k_step's dynamic LDS: the scene carve, plus each wave's refill staging buffer where the
// in-line refill is staged through LDS (kstep_refill_off).  The staging sits outside the
// kStepLds scene budget (at most 64 KiB + 10 KiB per 256-thread block, within gfx950's
// 160 KiB per workgroup).
static size_t kstep_lds_bytes(const KParams& P, int bs) {
    const size_t off = kstep_refill_off(P, bs);
    return off ? off + (size_t)(bs / 64) * kMT * 4 : step_lds_bytes(P);
}

template <int SCN>
static hipError_t step_i(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* out,
                         uint32_t* out_count, uint32_t* zero, uint32_t* req_count, uint32_t visits, uint32_t blocks,
                         uint64_t live, hipStream_t st) {
    // Sphere-BVH scenes (C3) keep ~45 KB of BVH and spheres in LDS, so 256-thread blocks stop
    // at 3 per CU (3 waves per SIMD); 512-thread blocks share one copy between 8 waves
    // (4 waves per SIMD, the VGPR limit).  Same partitions, same results.
    if (SCN == SCN_SPHERE && P.n_snode > 0 && kStepBlock512 && P.integrator == XRT_INTEGRATOR_DIRECT) {
        // the grid must stay a multiple of n_part (part_iter: block b serves partition b % n_part
        // and chunk b / n_part of gridDim / n_part chunks)
        const uint32_t chunks = std::max(1u, blocks / P.n_part);
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_DIRECT, 512>), dim3(P.n_part * ((chunks + 1) / 2)), dim3(512),
                           kstep_lds_bytes(P, 512), st, P, list, count, out, out_count, zero, req_count, visits);
        return hipGetLastError();
    }
    const size_t lds = kstep_lds_bytes(P, kBlock);
    if (P.integrator == XRT_INTEGRATOR_DIRECT)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_DIRECT>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                           out, out_count, zero, req_count, visits);
    // volumetric walks with fewer live slots than 2 waves per SIMD hold (a row shard of a
    // multi-GPU frame, a frame's tail): the 2-wave build, whose registers hold the walk without
    // spilling (C5 shard 0 of 8: 43.9 -> 41.9 ms; a full frame stays at 4 waves per SIMD)
    else if (P.integrator == XRT_INTEGRATOR_VPT && live < kVptLowLive)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_VPT, kBlock, 2>), dim3(blocks), dim3(kBlock), lds, st, P, list,
                           count, out, out_count, zero, req_count, visits);
    else if (P.integrator == XRT_INTEGRATOR_VPT_NEE && live < kVptLowLive)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_VPT_NEE, kBlock, 2>), dim3(blocks), dim3(kBlock), lds, st, P,
                           list, count, out, out_count, zero, req_count, visits);
    else if (P.integrator == XRT_INTEGRATOR_VPT)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_VPT>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                           out, out_count, zero, req_count, visits);
    else if (P.integrator == XRT_INTEGRATOR_INDIRECT)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_INDIRECT>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                           out, out_count, zero, req_count, visits);
    else if (P.integrator == XRT_INTEGRATOR_NORMAL)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_NORMAL>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                           out, out_count, zero, req_count, visits);
    else if (P.integrator == XRT_INTEGRATOR_VPT_NEE)
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_VPT_NEE>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                           out, out_count, zero, req_count, visits);
    else
        hipLaunchKernelGGL((k_step<SCN, XRT_INTEGRATOR_GI>), dim3(blocks), dim3(kBlock), lds, st, P, list, count,
                           out, out_count, zero, req_count, visits);
    return hipGetLastError();
}

bool use_step_tri(const KParams& P) {
    return P.scene_kind == SCN_TRI && P.small_tri && P.n_objs <= kCoopMaxObjs &&
           (P.integrator == XRT_INTEGRATOR_GI || P.integrator == XRT_INTEGRATOR_DIRECT) && !exp_env("XRT_NO_COOP") &&
           ((step_layout(P).total + 15u) & ~15u) + (kBlock / 64) * sizeof(CoopWave) <= kStepLds;
}

hipError_t launch_step(const KParams& P, const KParams* dP, const uint32_t* list, const uint32_t* count, uint32_t* out,
                       uint32_t* out_count, uint32_t* zero, uint32_t* req_count, uint32_t visits, uint32_t blocks,
                       uint64_t live, hipStream_t st) {
    if (!step_lds_bytes(P)) return hipErrorInvalidValue;
    if (P.n_part == 0 || blocks % P.n_part != 0) return hipErrorInvalidValue;   // part_iter's grid contract
    if (use_step_tri(P)) {
        const size_t lds = ((step_layout(P).total + 15u) & ~15u) + (kBlock / 64) * sizeof(CoopWave);
        if (P.integrator == XRT_INTEGRATOR_DIRECT)
            hipLaunchKernelGGL((k_step_tri<XRT_INTEGRATOR_DIRECT>), dim3(blocks), dim3(kBlock), lds, st, dP, list,
                               count, out, out_count, zero, req_count, visits);
        else
            hipLaunchKernelGGL((k_step_tri<XRT_INTEGRATOR_GI>), dim3(blocks), dim3(kBlock), lds, st, dP, list, count,
                               out, out_count, zero, req_count, visits);
        return hipGetLastError();
    }
    switch (P.scene_kind) {
        case SCN_TRI: return step_i<SCN_TRI>(P, list, count, out, out_count, zero, req_count, visits, blocks, live, st);
        case SCN_SPHERE: return step_i<SCN_SPHERE>(P, list, count, out, out_count, zero, req_count, visits, blocks, live, st);
        default: return step_i<SCN_MIXED>(P, list, count, out, out_count, zero, req_count, visits, blocks, live, st);
    }
}

// ------------------------------------------------------------------ ray queries ----
// Scene::intersect / Scene::occluded for caller rays (xrt_query): the rays become the slots
// of a one-partition list, launch_trace (the render's own trace kernels, BVHs included)
// writes the hit records, and k_query_out rebuilds IntersectInfo with the shading code's
// surface() — the same records the integrators read.
__global__ __launch_bounds__(kBlock) void k_query_in(KParams P, const float* __restrict__ rays,
                                                     const float* __restrict__ tmax, int mode, uint32_t* list,
                                                     uint32_t* count) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s == 0) count[0] = P.n_slots;
    if (s >= P.n_slots) return;
    const float* r = rays + 6 * (size_t)s;
    list[s] = s;
    P.occ[s] = 0;
    if (mode == XRT_QUERY_INTERSECT) {
        P.ray_o[s] = make_float4(r[0], r[1], r[2], 0.0f);
        P.ray_d[s] = make_float4(r[3], r[4], r[5], 0.0f);
        P.state[s] = ST_RAY;
    } else {
        P.sh_o[s] = make_float4(r[0], r[1], r[2], tmax ? tmax[s] : kINF);
        P.sh_d[s] = make_float4(r[3], r[4], r[5], 0.0f);
        P.state[s] = 1u << ST_SHADOW_SHIFT;
    }
}

template <int SCN>
__global__ __launch_bounds__(kBlock) void k_query_out(KParams P, int mode, xrt_hit* __restrict__ out) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= P.n_slots) return;
    xrt_hit q;
    memset(&q, 0, sizeof(q));
    q.object = -1, q.primitive = -1;
    if (mode != XRT_QUERY_INTERSECT) {
        q.hit = P.occ[s] & 1u;
        q.t = q.t1 = kINF;
        out[s] = q;
        return;
    }
    const v3 o = xyz(P.ray_o[s]), d = xyz(P.ray_d[s]);
    const f4 h = P.hit[s];
    Surf S;
    float t1;
    const int obj = surface<SCN>(P, s, o, d, h, S, t1);
    // the triangle that last wrote barycentric (with dpdu / dpdv; spheres and boxes leave
    // both untouched), and its (u, v)
    int surf = SCN == SCN_SPHERE ? -1 : __float_as_int(h.w);
    float su = h.y, sv = h.z;
    if (SCN == SCN_MIXED && surf >= 0) {
        const f4 h2 = P.hit2[s], h3 = P.hit3[s];
        surf = __float_as_int(h2.z), su = h3.z, sv = h3.w;
    }
    q.hit = obj >= 0;
    q.object = obj;
    q.primitive = (surf >= 0 && (surf >> 28) == SEG_TRI) ? (surf & 0x0fffffff) : -1;   // global; host makes it local
    q.t = obj >= 0 ? h.x : kINF;
    q.t1 = t1;
    const v3 f[5] = {S.pos, S.ng, S.ns, S.dpdu, S.dpdv};
    float* dst[5] = {q.position, q.ng, q.ns, q.dpdu, q.dpdv};
    for (int k = 0; k < 5; ++k) dst[k][0] = f[k].x, dst[k][1] = f[k].y, dst[k][2] = f[k].z;
    if (q.primitive >= 0) q.barycentric[0] = su, q.barycentric[1] = sv;
    out[s] = q;
}

hipError_t launch_query(const KParams& P, const float* rays, const float* tmax, int mode, uint32_t* list,
                        uint32_t* count, uint32_t* zero, xrt_hit* out, hipStream_t st) {
    const uint32_t blocks = (P.n_slots + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_query_in, dim3(blocks), dim3(kBlock), 0, st, P, rays, tmax, mode, list, count);
    hipError_t e = hipGetLastError();
    // the caller's directions need not be unit vectors, so |det| is not bounded by det_bounded's
    // |e1| |e2|: phase A takes the per-lane test (IEEE-exact reciprocal) instead of the pair passes
    KParams Q = P;
    Q.sstep = nullptr;
    if (e == hipSuccess) e = launch_trace(Q, list, count, zero, blocks, st);
    if (e == hipSuccess) e = launch_trace_deep(Q, st);
    if (e != hipSuccess) return e;
    switch (P.scene_kind) {
        case SCN_TRI: hipLaunchKernelGGL(k_query_out<SCN_TRI>, dim3(blocks), dim3(kBlock), 0, st, P, mode, out); break;
        case SCN_SPHERE: hipLaunchKernelGGL(k_query_out<SCN_SPHERE>, dim3(blocks), dim3(kBlock), 0, st, P, mode, out); break;
        default: hipLaunchKernelGGL(k_query_out<SCN_MIXED>, dim3(blocks), dim3(kBlock), 0, st, P, mode, out); break;
    }
    return hipGetLastError();
}

hipError_t launch_finish(const KParams& P, hipStream_t st) {
    const uint32_t blocks = std::min<uint32_t>((P.n_slots + kBlock - 1) / kBlock, 2048u);
    hipLaunchKernelGGL(k_finish, dim3(blocks), dim3(kBlock), 0, st, P);
    return hipGetLastError();
}

hipError_t launch_test_rng(const uint32_t* seeds, uint32_t n_seeds, uint32_t skip, uint32_t n, float* out,
                           uint32_t* rings, hipStream_t st) {
    const uint32_t blocks = (n_seeds + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_test_rng, dim3(blocks), dim3(kBlock), 0, st, seeds, n_seeds, skip, n, out, rings);
    return hipGetLastError();
}

hipError_t launch_test_trig(const float* x, uint32_t n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_test_trig, dim3((n + 255) / 256), dim3(256), 0, st, x, n, out);
    return hipGetLastError();
}

hipError_t launch_test_trig_domain(uint32_t first, uint32_t count, float* s, float* c, float* r, hipStream_t st) {
    hipLaunchKernelGGL(k_test_trig_domain, dim3((count + 255) / 256), dim3(256), 0, st, first, count, s, c, r);
    return hipGetLastError();
}

hipError_t launch_test_fastdiv(uint32_t mode, float c, float rc, uint32_t first, uint32_t count,
                               unsigned long long* nbad, uint32_t* bad, hipStream_t st) {
    hipLaunchKernelGGL(k_test_fastdiv, dim3((count + 255) / 256), dim3(256), 0, st, mode, c, rc, first, count, nbad,
                       bad);
    return hipGetLastError();
}

hipError_t launch_test_logexp(const float* x, uint32_t n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_test_logexp, dim3((n + 255) / 256), dim3(256), 0, st, x, n, out);
    return hipGetLastError();
}

hipError_t launch_test_powf(const float* x, uint32_t n, float y, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_test_powf, dim3((n + 255) / 256), dim3(256), 0, st, x, n, y, out);
    return hipGetLastError();
}

hipError_t launch_tonemap(const float* rgb, uint32_t n, float inv_gamma, uint8_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_tonemap, dim3((n + 255) / 256), dim3(256), 0, st, rgb, n, inv_gamma, out);
    return hipGetLastError();
}

}  // namespace xrt
