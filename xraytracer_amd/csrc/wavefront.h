// wavefront.h — device data layout of the MI355X wavefront path tracer, shared by the
// kernels (wavefront.hip) and the host orchestration (xrt_api.cpp).
//
// HBM layout (DESIGN.md §Data layout):
//   scene  : triangles as 3 float4 per triangle {(v0, obj), (e1 = v1-v0, occluder), (e2 = v2-v0, 0)}
//            in Scene::m_objects order, plus per-triangle ng and vertex normals read only
//            at shading; spheres {(c, r)}; boxes {pmin, pmax}; object and light tables.
//   slots  : one path slot per pixel of this shard; all per-slot state is SoA (float4 /
//            uint32 arrays indexed by slot) so a wave's loads are coalesced.
//   RNG    : per slot a 1248-word ring (two 624-word mt19937 blocks) + cursor/generated
//            counters.  k_seed writes each slot's seeded state and one k_refill launch
//            twists its first block; after that every schedule twists a slot's next block
//            in-line, at the end of the launch in which it runs low, one whole wave per
//            ring (wave_refill: k_shade, k_step, k_step_tri, k_step_merged).  k_pixel keeps
//            its pixel's stream in LDS and generates it as it goes (pixel.hip).
#pragma once
#include <stdint.h>

#include "tuning.h"
#include "xrt.h"

#ifndef __HIPCC__
struct float4_ { float x, y, z, w; };
#endif

namespace xrt {

constexpr int kMaxLights = 4;        // shadow rays in flight per slot (one per area light)
constexpr uint32_t kMT = 624;        // mt19937 state words
constexpr uint32_t kRing = 1248;     // ring words per slot
constexpr uint32_t kRngMin = 64;     // request a refill when fewer words than this remain
constexpr uint32_t kRngVisit = 16;   // a slot visit needs at least this many (max draws of a
                                     // GI/Direct visit with kMaxLights lights is 13; VPT walks
                                     // suspend themselves below 8)
constexpr uint32_t kMaxParts = XRT_MAX_PARTS;   // live-list partitions (counters per list)
constexpr uint32_t kPartMinSlots = XRT_PART_MIN;   // ... of at least this many slots each
constexpr uint32_t kStepVisits = 32; // fused schedule: path segments per slot per k_step
constexpr uint32_t kMergedVisits = 64; // merged-trace schedule: segments per slot per launch (at most;
                                       // clamped so a launch's draws fit one refill block)
constexpr uint32_t kMergedLive64 = 160000;  // merged-trace schedule: live slots for 64 slots per wave
constexpr uint32_t kMergedLive32 = XRT_LIVE32;   // ... and for 32 (below: 16 slots, 4 lanes each)
constexpr uint32_t kBvhLive64 = XRT_BVH_LIVE64;   // two-level merged schedule: 64 slots per wave above this
constexpr uint32_t kBvhLive32 = XRT_BVH_LIVE32;   // ... 32 above this, else 16
constexpr uint32_t kMergedLive16 = XRT_LIVE16;   // ... and for 16 (below: 4 slots, 16 lanes each)
constexpr bool kVptEvents = XRT_VPT_EVENTS != 0;   // VPT k_step: one event (trace or collision) per iteration
constexpr uint32_t kVptEventVisits = XRT_VPT_EV_VISITS;   // ... events per slot per launch
constexpr uint32_t kVptEventDraws = XRT_VPT_EV_DRAWS;     // ... draws of an event for the refill threshold (a
                                           // collision draws <= 5; a lane with fewer words left stops early)
constexpr uint32_t kVptEventPrefetch = XRT_VPT_EV_PF;
constexpr uint64_t kVptLowLive = XRT_VPT_LOW_LIVE;          // ... below this many live slots: the 2-wave k_step build     // ... reload the 8-word RNG window below this many
constexpr bool kStepBlock512 = XRT_KSTEP_512 != 0;   // k_step of sphere-BVH scenes in 512-thread blocks
constexpr uint32_t kVisitDraws = 13; // max RNG draws of one GI/Direct segment (4 lights)
// fused schedule: a slot's ring is twisted at the end of a step launch when fewer than
// visits * 13 + kRngVisit words are left, so a GI/Direct slot never waits for words
// (KParams::rng_keep)

// slot state bits
enum : uint32_t {
    ST_RAY = 1u,      // extension ray pending (shade -> trace) / hit record valid (trace -> shade)
    ST_NEE = 2u,      // NEE contributions pending resolution (after the shadow rays are traced)
    ST_END = 4u,      // path ends after the NEE resolve
    ST_REGEN = 8u,    // slot must start its next sample
    ST_DONE = 16u,    // all samples of this pixel are done
    ST_MEDIUM = 32u,  // VPT delta-tracking loop suspended (resumes after an RNG refill)
    ST_RNGREQ = 64u,  // slot's first twist is pending (k_seed sets it, the seeding k_refill clears it)
    ST_NEEWALK = 128u,// VPT-NEE: the light sample's ratio tracking is suspended (state in KParams::nee)
    ST_SHADOW_SHIFT = 8u  // bits 8..15: which lights have a shadow ray in flight
};

enum : int { SEG_TRI = 0, SEG_SPHERE = 1, SEG_BOX = 2 };
enum : int { SCN_TRI = 0, SCN_SPHERE = 1, SCN_MIXED = 2 };  // trace kernel specialisations
// integrators that trace exactly one ray per sample (Direct, Normal): no bounce loop, so
// maxDepth 0 does not zero their samples
constexpr bool one_hit(int integ) { return integ == XRT_INTEGRATOR_DIRECT || integ == XRT_INTEGRATOR_NORMAL; }
// volumetric integrators (VolumePathTracing and its NEE variant): delta tracking through media
constexpr bool vpt_family(int integ) { return integ == XRT_INTEGRATOR_VPT || integ == XRT_INTEGRATOR_VPT_NEE; }

struct DSeg {   // a run of consecutive objects of one kind, in iteration order
    int kind, first, count, pad;
};

struct DObj {
    int kind, material, light, medium;
    float fr[3];   // Lambert::evaluateBxDF = albedo / PI (material 1), computed once on the host
    float pad;     // with the same correctly rounded float division; 0 for other materials
};

// Mesh object culling record for small triangle scenes: the object's triangle range and
// an AABB of its vertices grown by a margin far larger than the float error of the
// Moller-Trumbore test, so skipping an object whose box the ray misses never changes a
// hit decision.
struct DObjBox {
    float bmin[3];
    int first;
    float bmax[3];
    int count_occ;   // triangle count | (occluder << 31)
};
// Per-object record of the merged-trace triangle kernel (step_tri.hip), passed by value
// as a kernel argument so the object loop reads it with scalar loads: the culling box
// (DObjBox's, margin included), the triangle range, whether it occludes (no area light),
// and magic = ceil(2^32 / count) for the pair -> (ray rank, triangle) split.
struct StepObj {
    float bmin[3];
    int first;
    float bmax[3];
    uint32_t count;
    uint32_t magic;
    uint32_t occluder;
    int axis;      // DObjPlane of the object
    float plane;
};
// Axis-aligned plane of a mesh object whose every vertex has the same coordinate `c` on
// axis `axis` (-1: no such plane).  Every Moller-Trumbore test of such an object by a ray
// whose origin lies on one side of the plane and whose direction does not point back at it
// returns t <= 0 (or |det| < eps), so the merged-trace kernels skip the object for that ray
// without a box test (plane_away, step_tri.hip; the argument is in DESIGN.md §3).
struct DObjPlane {
    int axis;
    float c;
};
constexpr int kMergedMaxObjs = 32;
struct StepObjs {
    StepObj o[kMergedMaxObjs];
    int n;
};
constexpr uint32_t kBvhLeaf = 4;      // sphere BVH (C3): primitives per leaf (at most)
constexpr uint32_t kBvhLeafTri = XRT_BVH_LEAF;   // triangle BVH (C4): triangles per leaf (at most)
constexpr int kBvhMaxDepth = 48;      // BVH build: depth bound (SAH above max - 24 levels, median below)
constexpr int kBvhStack = 24;         // k_trace_bvh: LDS traversal stack entries per thread (> tree depth)
constexpr int kBvh4Stack = 48;        // k_trace_deep4: LDS stack entries per lane (>= 3 * 4-wide depth + 1)
constexpr int kSphBvhMin = 16;        // sphere scenes with at least this many spheres get a skip-link BVH
constexpr int kSmallTris = 1024;   // scenes up to this size keep every triangle in LDS
constexpr int kLargeObjTris = 256;  // two-level trace: mesh objects above this go into the BVH
constexpr int kSmallObjs = 256;
constexpr unsigned kStepLds = 64u * 1024u;   // LDS budget of the fused schedule (k_step)
constexpr int kStatsPix = 8;                // KParams::stats words 8..14: k_pixel path counters (xrt_stats pix_*)
constexpr int kStatsPhase = 40;              // KParams::stats words 40..47: XRT_PHASE_CLOCK builds' phase cycles
constexpr int kStatsWork = 32;               // KParams::stats word k_pixel counts the pixels taken in
constexpr unsigned kPixLds = 160u * 1024u;   // k_pixel: scene + per-wave stream windows (gfx950: 160 KiB per workgroup)

struct DLight {  // e1/e2/Ng precomputed on the host with the reference constructor's ops
    int kind;
    float v0[3], v1[3], v2[3], e1[3], e2[3], Ng[3], center[3], radius, Le[3];
};

struct DMedium {
    const float* density;  // [nz][ny][nx]
    int nx, ny, nz;
    float origin[3], voxel_size;
    float absorption[3], scattering[3], multiplier, g;
    float majorant, inv_majorant;
    int kind;              // XRT_MEDIUM_* (0 heterogeneous: delta / ratio tracking)
    float sigma_t[3];      // homogeneous kinds: sigma_a + sigma_s (HomogeneousMedium ctor)
    double inv_voxel;      // 1.0 / (double)voxel_size, once on the host (same IEEE quotient)
    // sparse leaf bricks (xrt_set_medium_bricks): table[(bz*nby + by)*nbx + bx] -> brick or -1;
    // null for the dense grid
    const int* brick_table;
    const float* bricks;
    int nbx, nby, nbz;
    // dense grid: every cell's eight corner values in BoxSampler's order (d000 d001 d010 d011
    // d100 d101 d110 d111), 32 B per cell [(k * (ny-1) + j) * (nx-1) + i], so an interior
    // lookup is one 32-byte load instead of four rows of the grid; null when not built
    const float* corners;
};

#ifdef __HIPCC__
using f4 = float4;
#else
using f4 = float4_;
#endif

struct KParams {
    // ---- scene
    const f4* tri;      // [3 * n_tris]
    const f4* tri_ng;   // [n_tris]
    const f4* tri_nrm;  // [3 * n_tris]
    const f4* sph;      // [n_sph] (center, radius)
    const int* sph_obj; // [n_sph] object index; bit 30 set = occluder
    const f4* box;      // [2 * n_box] (pmin, obj) (pmax, 0)
    const DObj* objs;
    const DLight* lights;
    const DSeg* segs;
    const DObjBox* obj_box;   // per object, for the small-scene trace path (n_objs entries)
    const DObjPlane* obj_plane;   // per object, small triangle scenes (n_objs entries)
    const f4* bvh_node;       // large triangle scenes: BvhNode array (4 f4 each, bvh.h), else null
    const f4* bvh_tri;        // triangles in BVH leaf order, as `tri` but e2.w = original index
    int bvh_stack;            // k_trace_bvh: LDS stack entries per thread (tree depth + 1 <= kBvhStack)
    int bvh_nodes;            // BvhNode count
    // two-level trace of large triangle scenes (C4): objects of at most kLargeObjTris
    // triangles are scanned directly (k_trace_2a: LDS, culling boxes and planes); only rays
    // whose segment reaches the BVH over the large objects' triangles are queued for it
    // (k_trace_deep)
    const f4* stri;           // small objects' triangles, as bvh_tri (e2.w = original index)
    const DObjBox* sbox;      // their culling boxes (first / count into stri)
    const DObjPlane* splane;
    int n_stri, n_sobj, two_level;
    const struct StepObjs* sstep;   // HOST pointer (launch_trace passes it by value): the small objects as
                                    // merged-trace records when n_sobj <= kMergedMaxObjs, else null
    const f4* bvh4;           // the BVH's 4-wide form (bvh.h Bvh4Node, 8 f4 each) for k_trace_deep4
    int bvh4_nodes, bvh4_stack;   // node count; LDS stack entries per lane (3 * depth + 1)
    int deep_quad;                // k_trace_deep4q (four lanes per ray) instead of k_trace_deep4
    uint32_t* deep;           // queued rays (slot * 8 + kind: 0 extension, 1 + l shadow ray l), per partition:
                              // extension rays from the start, shadow rays from entry part_cap on
    uint32_t* deep_count;     // [kMaxParts] extension-ray counts, [kMaxParts] fetch counters,
                              // [kMaxParts] shadow-ray counts (queued from dq + part_cap)
    uint32_t deep_cap;        // entries per partition
    const f4* snode;          // sphere scenes: threaded BVH (bvh.h SkipNode, 2 f4 each), else null
    const f4* ssph;           // spheres in BVH leaf order (center, radius)
    const int* sbk;           // per ssph entry: original sphere index | (occluder << 30)
    int n_snode;
    float sph_pad;            // the sphere BVH's box margin (1e-4 scene diagonal + 1e-4)
    const f4* sblk;           // per 64 ssph entries: a ball (center, radius) holding each member's ball of radius |r| + sph_pad
    int n_segs, n_lights, n_tris, n_sph, n_box, scene_kind, n_objs, small_tri;
    int det_bounded;   // every triangle has |e1| |e2| < 2^120 (ray_tri_nb's Newton reciprocal, xrt_api.cpp)
    DMedium medium;
    // ---- camera (row-major c2w) + PinholeCamera scale / aspect
    float c2w[16];
    float scale, aspect;
    float raspect;               // RN(1 / aspect)
    float fw, fh, rw, rh;        // (float)width, (float)height and their RN reciprocals
    uint32_t cdiv;               // bit 0/1/2: x / width, height, aspect may use div_const (host-proven)
    // ---- render
    int integrator;
    uint32_t max_depth, width, height, spp, shard_index, shard_count, n_slots;
    uint32_t n_part, part_cap;   // live-list partitions: n_part (<= kMaxParts) of part_cap slots
    uint32_t rng_keep;           // fused schedule refill threshold (words ahead)
    uint32_t spw_req;            // merged schedule: requested slots per wave (0 = by live count)
    uint32_t rflags;             // xrt_render_params.flags
    uint32_t lds_max;            // the device's LDS bytes per workgroup (hipDeviceAttributeMaxSharedMemoryPerBlock)
    uint4* camlist;              // speculative starts (spec.hip): per slot the pixel's camera-ray triangle list
    // ---- slot state (SoA)
    f4 *ray_o, *ray_d, *thr, *rad, *thr_prev;
    f4 *hit;     // t, u, v, code(bits)        code: -1 miss, (kind << 28) | prim
    f4 *hit2;    // t1, surf code, dp code, surf t   (mixed scenes / boxes)
    f4 *hit3;    // surf u, surf v, dp u, dp v
    f4 *sh_o;    // [kMaxLights][n_slots] origin, tmax
    f4 *sh_d;    // [kMaxLights][n_slots] direction
    f4 *sh_c;    // [kMaxLights][n_slots] unoccluded contribution
    f4 *med;     // VPT suspended delta-tracking state: t, t1, ...
    f4 *med2;
    f4 *nee;     // VPT-NEE suspended ratio tracking, 4 x [n_slots]: (p1, t) (dir, dist) (tr, f) (Le, pdf)
    uint32_t *state, *sample_k, *depth, *occ;
    uint32_t *rng_c, *rng_g, *ring;
    uint32_t *req;             // refill request list (slots)
    uint32_t *c_seg, *c_shadow, *c_rej, *c_stall;
    float* fb;                 // [height][width][3]
    unsigned long long* stats; // device reduction target: seg, shadow, draws, rej, stall
};

}  // namespace xrt
