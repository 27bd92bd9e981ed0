// lscene.h — the LDS-resident scene of the fused schedules (k_step, k_pixel): its carve
// (step_layout, path_common.h), the copy into LDS at the start of a launch, and the per-lane
// Scene::intersect / Scene::occluded restatements over it (object order, exact BVHs).
#pragma once
#include "path_common.h"

namespace xrt {

// Conservative ray/box overlap on [0, tlim] (boxes padded far beyond a hit's float error)
__device__ __forceinline__ bool bvh_box(const f4& mn, const f4& mx, v3 o, v3 inv, float tlim) {
    const float tx0 = (mn.x - o.x) * inv.x, tx1 = (mx.x - o.x) * inv.x;
    const float ty0 = (mn.y - o.y) * inv.y, ty1 = (mx.y - o.y) * inv.y;
    const float tz0 = (mn.z - o.z) * inv.z, tz1 = (mx.z - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
    return !(tn > tf);
}

struct HitRec {
    float t, u, v;
    int code;           // winner: (kind << 28) | index, -1 miss
    int surf, dp;       // mixed scenes: last SurfaceInfo / dpdu writer
    float st, su, sv, du, dv, t1;
};

// Sphere scenes (C3): stackless traversal of the threaded BVH (bvh.h SkipNode) in LDS.
// Same exactness argument as the triangle BVH: boxes are the spheres' bounds padded far
// beyond the float error of Sphere::intersect's hit point, a box is entered when it
// overlaps [0, best t] (inclusive), and the closest hit is the lexicographic minimum of
// (t, original index) — the reference's in-order strict `t < best` scan over the objects
// (Src/scene.cpp:190-200, primitive.h:106-124).  Any-hit for shadow rays skips spheres of
// area-light objects (Scene::occluded, Src/scene.cpp:202-211).
template <bool ANY>
__device__ __forceinline__ bool sphere_bvh(const LScene& L, v3 o, v3 d, float tmax, float& bt, int& bk) {
    const v3 inv = rcp3(d);
    int i = 0;
    while (i < L.n_snode) {
        const f4 a = L.snode[2 * i], b = L.snode[2 * i + 1];
        if (!bvh_box(a, b, o, inv, ANY ? tmax : bt)) {
            i = __float_as_int(a.w);
            continue;
        }
        const int leaf = __float_as_int(b.w);
        if (leaf >= 0) {
            const int first = leaf & 0xffffff, end = first + (leaf >> 24);
            for (int j = first; j < end; ++j) {
                const int kw = L.sbk[j];
                if (ANY && !(kw & (1 << 30))) continue;
                const f4 S = L.ssph[j];
                float t;
                const bool hit = sphere_hit(o, d, xyz(S), S.w, t);
                if (ANY) {
                    if (hit && t < tmax) return true;
                } else {
                    const int k = kw & 0x3fffffff;
                    const bool upd = hit && (t < bt || (t == bt && k < bk));
                    bt = upd ? t : bt;
                    bk = upd ? k : bk;
                }
            }
        }
        ++i;
    }
    return false;
}

// Scene::intersect over the LDS scene (Src/scene.cpp:190-200)
template <int SCN>
__device__ __forceinline__ void closest_l(const KParams& P, const LScene& L, v3 o, v3 d, HitRec& h) {
    h.t = kINF, h.u = h.v = 0.0f, h.code = -1, h.surf = -1, h.dp = -1, h.t1 = kINF;
    h.st = h.su = h.sv = h.du = h.dv = 0.0f;
    if (SCN == SCN_TRI) {
        const v3 inv = rcp3(d);
        for (int ob = 0; ob < P.n_objs; ++ob) {
            const DObjBox B = L.box[ob];
            const bool ne = box_overlap(o, inv, B, h.t);
            if (!ne) continue;
            const int end = B.first + (B.count_occ & 0x7fffffff);
            for (int k = B.first; k < end; ++k) {
                float t, u, v;
                if (ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v) &&
                    t < h.t)
                    h.t = t, h.u = u, h.v = v, h.code = k;
            }
        }
    } else if (SCN == SCN_SPHERE) {
        if (L.n_snode > 0) {
            float bt = kINF;
            int bk = -1;
            (void)sphere_bvh<false>(L, o, d, kINF, bt, bk);
            if (bk >= 0) h.t = bt, h.code = (1 << 28) | bk;
            return;
        }
        for (int k = 0; k < P.n_sph; ++k) {
            const f4 S = L.sph[k];
            float t;
            if (sphere_hit(o, d, xyz(S), S.w, t) && t < h.t) h.t = t, h.code = (1 << 28) | k;
        }
    } else {
        for (int sg = 0; sg < P.n_segs; ++sg) {
            const DSeg seg = P.segs[sg];
            if (seg.kind == SEG_TRI) {
                for (int k = seg.first; k < seg.first + seg.count; ++k) {
                    float t, u, v;
                    if (ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v) &&
                        t < h.t)
                        h.t = t, h.u = u, h.v = v, h.code = k, h.surf = k, h.st = t, h.su = u, h.sv = v, h.dp = k,
                        h.du = u, h.dv = v;
                }
            } else if (seg.kind == SEG_SPHERE) {
                for (int k = seg.first; k < seg.first + seg.count; ++k) {
                    const f4 S = L.sph[k];
                    float t;
                    if (sphere_hit(o, d, xyz(S), S.w, t) && t < h.t)
                        h.t = t, h.u = h.v = 0.0f, h.code = (1 << 28) | k, h.surf = h.code, h.st = t;
                }
            } else {
                for (int b = seg.first; b < seg.first + seg.count; ++b) {
                    float t0, t1;
                    if (box_hit(o, d, xyz(L.bx[2 * b]), xyz(L.bx[2 * b + 1]), t0, t1))
                        h.t = t0, h.t1 = t1, h.code = (2 << 28) | b;
                }
            }
        }
    }
}

// Scene::occluded over the LDS scene (Src/scene.cpp:202-211): area-light objects skipped
template <int SCN>
__device__ __forceinline__ bool occluded_l(const KParams& P, const LScene& L, v3 o, v3 d, float tmax) {
    if (SCN == SCN_TRI) {
        const v3 inv = rcp3(d);
        for (int ob = 0; ob < P.n_objs; ++ob) {
            const DObjBox B = L.box[ob];
            const bool ne = B.count_occ < 0 && box_overlap(o, inv, B, tmax);
            if (!ne) continue;
            const int end = B.first + (B.count_occ & 0x7fffffff);
            for (int k = B.first; k < end; ++k) {
                float t, u, v;
                if (ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v) &&
                    t < tmax)
                    return true;
            }
        }
        return false;
    } else {
        if (SCN == SCN_SPHERE && L.n_snode > 0) {
            float bt = kINF;
            int bk = -1;
            return sphere_bvh<true>(L, o, d, tmax, bt, bk);
        }
        for (int sg = 0; sg < P.n_segs; ++sg) {
            const DSeg seg = P.segs[sg];
            if (SCN == SCN_MIXED && seg.kind == SEG_TRI) {
                for (int k = seg.first; k < seg.first + seg.count; ++k) {
                    if (L.tri[3 * k + 1].w == 0.0f) continue;
                    float t, u, v;
                    if (ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v) &&
                        t < tmax)
                        return true;
                }
            } else if (seg.kind == SEG_SPHERE) {
                for (int k = seg.first; k < seg.first + seg.count; ++k) {
                    if (!(L.sobj[k] & (1 << 30))) continue;
                    const f4 S = L.sph[k];
                    float t;
                    if (sphere_hit(o, d, xyz(S), S.w, t) && t < tmax) return true;
                }
            } else if (SCN == SCN_MIXED && seg.kind == SEG_BOX) {
                return true;   // BoxMesh::occluded (Src/primitive.h:266-268)
            }
        }
        return false;
    }
}

// IntersectInfo::surfaceInfo from a hit record (see surface<>)
template <int SCN>
__device__ __forceinline__ int surface_l(const LScene& L, v3 o, v3 d, const HitRec& h, Surf& S) {
    S.pos = S.ng = S.ns = S.dpdu = S.dpdv = mk(0, 0, 0);
    if (h.code < 0) return -1;
    int surf = h.code, dp = (SCN == SCN_TRI) ? h.code : -1;
    float st = h.t, su = h.u, sv = h.v, du = h.u, dv = h.v;
    if (SCN == SCN_MIXED) surf = h.surf, dp = h.dp, st = h.st, su = h.su, sv = h.sv, du = h.du, dv = h.dv;
    if (surf >= 0) {
        const int kind = surf >> 28, idx = surf & 0x0fffffff;
        S.pos = ray_at(o, d, st);
        if (kind == SEG_TRI) {
            S.ng = xyz(L.tng[idx]);
            S.ns = tri_ns_l(L, idx, su, sv);
        } else {
            S.ng = normalize(ray_at(o, d, st) - xyz(L.sph[idx]));
            S.ns = S.ng;
        }
    }
    if (dp >= 0) onb(tri_ns_l(L, dp & 0x0fffffff, du, dv), S.dpdu, S.dpdv);
    const int kind = h.code >> 28, idx = h.code & 0x0fffffff;
    if (kind == SEG_TRI) return __float_as_int(L.tri[3 * idx].w);
    if (kind == SEG_SPHERE) return L.sobj[idx] & 0x3fffffff;
    return __float_as_int(L.bx[2 * idx].w);
}

// object index of a hit record (see surface_l)
__device__ __forceinline__ int hit_object(const LScene& L, const HitRec& h) {
    const int kind = h.code >> 28, idx = h.code & 0x0fffffff;
    if (kind == SEG_TRI) return __float_as_int(L.tri[3 * idx].w);
    if (kind == SEG_SPHERE) return L.sobj[idx] & 0x3fffffff;
    return __float_as_int(L.bx[2 * idx].w);
}

// ---- packet traversal (k_pixel) ----
// The rays of a k_pixel wave are coherent: 64 camera rays through one pixel, and their shadow
// rays toward one light.  These forms walk the scene once per wave at a wave-uniform position
// (node / object index in SGPRs, node words broadcast from LDS, loop control in SALU) and
// enter a node when any active lane's segment overlaps it; a lane tests a leaf's primitives
// only when its own segment overlaps the leaf's box.  A lane that does not overlap a node does
// not overlap any node below it (children's padded boxes lie inside the parent's), so each
// lane tests exactly the primitives, in exactly the order, of its own per-lane walk
// (sphere_bvh / closest_l / occluded_l): same hits, same ties.  Every lane of the wave must
// call them (ballots); `active` says which lanes have a ray.
__device__ __forceinline__ int wave_uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

template <bool ANY>
__device__ __forceinline__ bool sphere_bvh_wave(const LScene& L, v3 o, v3 d, float tmax, float& bt, int& bk,
                                                bool active) {
    const v3 inv = rcp3(d);
    bool occ = false;
    int i = 0;
    while (i < L.n_snode) {
        const f4 a = L.snode[2 * i], b = L.snode[2 * i + 1];
        const bool ov = active && !occ && bvh_box(a, b, o, inv, ANY ? tmax : bt);
        if (__ballot(ov) == 0ull) {
            i = wave_uniform(__float_as_int(a.w));
            continue;
        }
        const int leaf = wave_uniform(__float_as_int(b.w));
        if (leaf >= 0) {
            const int first = leaf & 0xffffff, end = first + (leaf >> 24);
            for (int j = first; j < end; ++j) {
                const int kw = wave_uniform(L.sbk[j]);
                if (ANY && !(kw & (1 << 30))) continue;
                const f4 S = L.ssph[j];
                float t = 0.0f;
                const bool hit = ov && sphere_hit(o, d, xyz(S), S.w, t);
                if (ANY) {
                    occ = occ || (hit && t < tmax);
                } else {
                    const int k = kw & 0x3fffffff;
                    const bool upd = hit && (t < bt || (t == bt && k < bk));
                    bt = upd ? t : bt;
                    bk = upd ? k : bk;
                }
            }
            if (ANY && __ballot(active && !occ) == 0ull) return occ;
        }
        ++i;
    }
    return occ;
}

// Scene::intersect for a coherent wave (closest_l's result for every active lane)
template <int SCN>
__device__ __forceinline__ void closest_w(const KParams& P, const LScene& L, v3 o, v3 d, HitRec& h, bool active) {
    if (SCN == SCN_SPHERE && L.n_snode > 0) {
        h.t = kINF, h.u = h.v = 0.0f, h.code = -1, h.surf = -1, h.dp = -1, h.t1 = kINF;
        h.st = h.su = h.sv = h.du = h.dv = 0.0f;
        float bt = kINF;
        int bk = -1;
        (void)sphere_bvh_wave<false>(L, o, d, kINF, bt, bk, active);
        if (bk >= 0) h.t = bt, h.code = (1 << 28) | bk;
    } else if (SCN == SCN_TRI) {
        h.t = kINF, h.u = h.v = 0.0f, h.code = -1, h.surf = -1, h.dp = -1, h.t1 = kINF;
        h.st = h.su = h.sv = h.du = h.dv = 0.0f;
        const v3 inv = rcp3(d);
        for (int ob = 0; ob < P.n_objs; ++ob) {
            const DObjBox B = L.box[ob];
            const bool ne = active && box_overlap(o, inv, B, h.t);
            if (__ballot(ne) == 0ull) continue;
            const int first = wave_uniform(B.first), end = first + wave_uniform(B.count_occ & 0x7fffffff);
            for (int k = first; k < end; ++k) {
                float t, u, v;
                if (ne && ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v) &&
                    t < h.t)
                    h.t = t, h.u = u, h.v = v, h.code = k;
            }
        }
    } else {
        if (active) closest_l<SCN>(P, L, o, d, h);
    }
}

// Scene::occluded for a coherent wave (occluded_l's result for every active lane)
template <int SCN>
__device__ __forceinline__ bool occluded_w(const KParams& P, const LScene& L, v3 o, v3 d, float tmax, bool active) {
    if (SCN == SCN_SPHERE && L.n_snode > 0) {
        float bt = kINF;
        int bk = -1;
        return sphere_bvh_wave<true>(L, o, d, tmax, bt, bk, active);
    } else if (SCN == SCN_TRI) {
        const v3 inv = rcp3(d);
        bool occ = false;
        for (int ob = 0; ob < P.n_objs; ++ob) {
            const DObjBox B = L.box[ob];
            const bool ne = active && !occ && B.count_occ < 0 && box_overlap(o, inv, B, tmax);
            if (__ballot(ne) == 0ull) continue;
            const int first = wave_uniform(B.first), end = first + wave_uniform(B.count_occ & 0x7fffffff);
            for (int k = first; k < end; ++k) {
                float t, u, v;
                if (ne && !occ && ray_tri(o, d, xyz(L.tri[3 * k]), xyz(L.tri[3 * k + 1]), xyz(L.tri[3 * k + 2]), t, u, v) &&
                    t < tmax)
                    occ = true;
            }
        }
        return occ;
    } else {
        bool occ = false;
        if (active) occ = occluded_l<SCN>(P, L, o, d, tmax);
        return occ;
    }
}

// k_step's in-line refill staging (wave_refill through LDS, one kMT-word buffer per wave)
// sits in the dynamic LDS right after the scene carve; returns its byte offset, or 0 where
// the refill twists from L2 instead (XRT_KSTEP_LDS_REFILL: sphere scenes keep their blocks
// per CU).  The same function sizes the launch (kstep_lds_bytes) and carves the kernel's LDS.
__host__ __device__ inline uint32_t kstep_refill_off(const KParams& P, int bs) {
    (void)bs;
    if (XRT_KSTEP_LDS_REFILL == 0 || (XRT_KSTEP_LDS_REFILL == 2 && P.scene_kind == SCN_SPHERE)) return 0;
    return (step_layout(P).total + 15u) & ~15u;
}

// Copy the scene into the block's LDS carve at `lb` (step_layout) and point an LScene at
// it.  Sphere-BVH scenes keep the BVH, the spheres in leaf order and their index words in
// LDS; the original-order sphere / object tables (read once per hit) stay in global memory.
// Every thread of the block calls it; the caller barriers before the first trace.
// bvh_lds = false (k_pixel): the sphere BVH, leaf-order spheres and index words are read
// from global memory (L1 / L2) and take no LDS.
__device__ inline LScene load_lscene(const KParams& P, char* lb, int tid, int bs, bool bvh_lds = true) {
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
    lds_copy(const_cast<f4*>(L.tri), P.tri, 3 * P.n_tris, tid, bs);
    lds_copy(const_cast<f4*>(L.tng), P.tri_ng, P.n_tris, tid, bs);
    lds_copy(const_cast<f4*>(L.nrm), P.tri_nrm, 3 * P.n_tris, tid, bs);
    if (P.scene_kind == SCN_TRI) lds_copy(const_cast<DObjBox*>(L.box), P.obj_box, P.n_objs, tid, bs);
    lds_copy(const_cast<f4*>(L.bx), P.box, 2 * P.n_box, tid, bs);
    lds_copy(const_cast<DLight*>(L.light), P.lights, P.n_lights, tid, bs);
    if (P.scene_kind == SCN_SPHERE && P.n_snode > 0 && !bvh_lds) {
        L.snode = P.snode, L.ssph = P.ssph, L.sbk = P.sbk;
        L.n_snode = P.n_snode;
        L.sph = P.sph, L.sobj = P.sph_obj, L.obj = P.objs;
    } else if (P.scene_kind == SCN_SPHERE && P.n_snode > 0) {
        L.snode = reinterpret_cast<const f4*>(lb + Lo.snode);
        L.ssph = reinterpret_cast<const f4*>(lb + Lo.ssph);
        L.sbk = reinterpret_cast<const int*>(lb + Lo.sbk);
        L.n_snode = P.n_snode;
        lds_copy(const_cast<f4*>(L.snode), P.snode, 2 * P.n_snode, tid, bs);
        lds_copy(const_cast<f4*>(L.ssph), P.ssph, P.n_sph, tid, bs);
        lds_copy(const_cast<int*>(L.sbk), P.sbk, P.n_sph, tid, bs);
        L.sph = P.sph, L.sobj = P.sph_obj, L.obj = P.objs;
    } else {
        lds_copy(const_cast<f4*>(L.sph), P.sph, P.n_sph, tid, bs);
        lds_copy(const_cast<DObj*>(L.obj), P.objs, P.n_objs, tid, bs);
        lds_copy(const_cast<int*>(L.sobj), P.sph_obj, P.n_sph, tid, bs);
    }
    return L;
}

}  // namespace xrt
