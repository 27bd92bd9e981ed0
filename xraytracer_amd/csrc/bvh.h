// bvh.h — host-side bounding volume hierarchy over a scene's primitives (triangles of
// large triangle scenes, C4), consumed by k_trace_bvh (wavefront.hip).
//
// The reference scans every primitive (Scene::intersect, Src/scene.cpp:190-200); the
// hierarchy only decides which primitives a ray needs to be tested against, and the
// device keeps the reference's result: closest hit = smallest t, ties to the lowest
// primitive index (the in-order strict `t < best` scan), any-hit for shadow rays.  Node
// boxes are padded by a margin far above the float error of a Moller-Trumbore hit
// position, so a box test never rejects a hit the linear scan accepts.
#pragma once
#include <stdint.h>

#include <vector>

namespace xrt {

// Binary BVH node holding both children's boxes (64 bytes = 4 float4), so one node fetch
// tests both children: {lmin, left}, {lmax, lcount}, {rmin, right}, {rmax, rcount}.
// A child with count > 0 is a leaf of `count` primitives starting at `index` of the
// reordered primitive array; count == 0 is an interior node at `index`; count == -1 is an
// empty slot (a one-leaf tree's right child).
constexpr uint32_t kBvhTopNodes = 64;   // leading nodes (breadth-first) the BVH trace keeps in LDS

struct BvhNode {
    float lmin[3];
    int32_t left;
    float lmax[3];
    int32_t lcount;
    float rmin[3];
    int32_t right;
    float rmax[3];
    int32_t rcount;
};

struct BvhBuild {
    std::vector<BvhNode> nodes;      // nodes[0] is the root
    std::vector<uint32_t> order;     // reordered primitive array: order[i] = original index
    int depth = 0;                   // deepest node (traversal stack bound)
};

// Threaded ("skip-link") form of a BvhBuild for stackless traversal: nodes in depth-first
// order, one box each; a ray that overlaps node i continues at i + 1 (its first child, or
// the next subtree after a leaf), a ray that misses it jumps to `skip` (the node after
// i's whole subtree).  leaf = -1 for an interior node, else (count << 24) | first.
struct SkipNode {
    float bmin[3];
    int32_t skip;
    float bmax[3];
    int32_t leaf;
};
std::vector<SkipNode> thread_bvh(const BvhBuild& b);

// 4-wide form of a BvhBuild (two-level trace, k_trace_deep_pt): each binary node absorbs
// its interior children (largest box first) until it has four children, so a traversal
// step fetches four child boxes (128 bytes) and the tree is about half as deep.  Child c:
// bmin[c], bmax[c]; count[c] > 0: a leaf of count[c] primitives from index[c] (the same
// reordered primitive array), 0: the interior node index[c], -1: empty.  Stored as 8 float4
// {bmin, index} x 4, {bmax, count} x 4; the first kBvhTopNodes (breadth-first) come first.
struct Bvh4Node {
    float lo[4][4];   // bmin xyz, index (int bits)
    float hi[4][4];   // bmax xyz, count (int bits)
};
// `depth`: the deepest node (a traversal pushes at most 3 children per level)
std::vector<Bvh4Node> collapse_bvh4(const BvhBuild& b, int& depth);

// prim_min / prim_max: n boxes (3 floats each).  Binned SAH, leaves of <= leaf_max
// primitives, median split below max_depth - 8 levels of headroom; margin pads every box.
BvhBuild build_bvh(const float* prim_min, const float* prim_max, uint32_t n, uint32_t leaf_max, float margin,
                   int max_depth);

}  // namespace xrt
