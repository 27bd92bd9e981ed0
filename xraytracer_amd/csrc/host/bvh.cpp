// bvh.cpp — binned-SAH BVH build on the host (see bvh.h).
#include "../bvh.h"

#include <algorithm>
#include <cfloat>
#include <cstring>

namespace xrt {

namespace {

struct Ref {
    float mn[3], mx[3], c[3];
    uint32_t idx;
};

struct Box {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const float* a, const float* b) {
        for (int q = 0; q < 3; ++q) mn[q] = std::min(mn[q], a[q]), mx[q] = std::max(mx[q], b[q]);
    }
    void grow(const Box& o) { grow(o.mn, o.mx); }
    float area() const {
        if (mx[0] < mn[0]) return 0.0f;
        const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

struct Builder {
    std::vector<Ref> refs;
    BvhBuild out;
    uint32_t leaf_max;
    float margin;
    int max_depth;

    Box bounds(uint32_t lo, uint32_t hi) const {
        Box b;
        for (uint32_t i = lo; i < hi; ++i) b.grow(refs[i].mn, refs[i].mx);
        return b;
    }

    uint32_t split(uint32_t lo, uint32_t hi, int depth) {
        const uint32_t n = hi - lo;
        Box cb;
        for (uint32_t i = lo; i < hi; ++i) cb.grow(refs[i].c, refs[i].c);
        int axis = 0;
        for (int q = 1; q < 3; ++q)
            if (cb.mx[q] - cb.mn[q] > cb.mx[axis] - cb.mn[axis]) axis = q;
        const float ext = cb.mx[axis] - cb.mn[axis];
        auto median = [&]() {
            const uint32_t mid = lo + n / 2;
            std::nth_element(refs.begin() + lo, refs.begin() + mid, refs.begin() + hi,
                             [axis](const Ref& a, const Ref& b) { return a.c[axis] < b.c[axis]; });
            return mid;
        };
        if (!(ext > 0.0f) || depth >= max_depth - 24) return median();
        constexpr int kBins = 16;
        Box bb[kBins];
        uint32_t bc[kBins] = {0};
        auto bin_of = [&](const Ref& r) {
            int b = (int)((r.c[axis] - cb.mn[axis]) / ext * kBins);
            return std::min(std::max(b, 0), kBins - 1);
        };
        for (uint32_t i = lo; i < hi; ++i) {
            const int b = bin_of(refs[i]);
            bb[b].grow(refs[i].mn, refs[i].mx);
            ++bc[b];
        }
        float best = FLT_MAX;
        int best_b = -1;
        for (int s = 1; s < kBins; ++s) {
            Box l, r;
            uint32_t nl = 0, nr = 0;
            for (int b = 0; b < s; ++b) l.grow(bb[b]), nl += bc[b];
            for (int b = s; b < kBins; ++b) r.grow(bb[b]), nr += bc[b];
            if (!nl || !nr) continue;
            const float cost = l.area() * nl + r.area() * nr;
            if (cost < best) best = cost, best_b = s;
        }
        if (best_b < 0) return median();
        const auto it = std::partition(refs.begin() + lo, refs.begin() + hi,
                                       [&](const Ref& r) { return bin_of(r) < best_b; });
        const uint32_t mid = (uint32_t)(it - refs.begin());
        return (mid == lo || mid == hi) ? median() : mid;
    }

    void set_child(float* cmn, float* cmx, int32_t& index, int32_t& count, uint32_t lo, uint32_t hi, int depth) {
        const Box b = bounds(lo, hi);
        for (int q = 0; q < 3; ++q) cmn[q] = b.mn[q] - margin, cmx[q] = b.mx[q] + margin;
        if (hi - lo <= leaf_max) {
            index = (int32_t)lo;
            count = (int32_t)(hi - lo);
            out.depth = std::max(out.depth, depth);
        } else {
            index = (int32_t)node(lo, hi, depth);
            count = 0;
        }
    }

    uint32_t node(uint32_t lo, uint32_t hi, int depth) {
        const uint32_t id = (uint32_t)out.nodes.size();
        out.nodes.push_back(BvhNode{});
        out.depth = std::max(out.depth, depth);
        const uint32_t mid = split(lo, hi, depth);
        BvhNode nd{};
        set_child(nd.lmin, nd.lmax, nd.left, nd.lcount, lo, mid, depth + 1);
        set_child(nd.rmin, nd.rmax, nd.right, nd.rcount, mid, hi, depth + 1);
        out.nodes[id] = nd;
        return id;
    }
};

}  // namespace

BvhBuild build_bvh(const float* prim_min, const float* prim_max, uint32_t n, uint32_t leaf_max, float margin,
                   int max_depth) {
    Builder B;
    B.leaf_max = std::max<uint32_t>(1u, leaf_max);
    B.margin = margin;
    B.max_depth = max_depth;
    B.refs.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        Ref& r = B.refs[i];
        for (int q = 0; q < 3; ++q) {
            r.mn[q] = prim_min[3 * i + q], r.mx[q] = prim_max[3 * i + q];
            r.c[q] = 0.5f * (r.mn[q] + r.mx[q]);
        }
        r.idx = i;
    }
    if (n <= B.leaf_max) {
        BvhNode root{};
        B.set_child(root.lmin, root.lmax, root.left, root.lcount, 0, n, 1);
        if (n == 0) root.lcount = -1;
        root.right = 0, root.rcount = -1;
        for (int q = 0; q < 3; ++q) root.rmin[q] = FLT_MAX, root.rmax[q] = -FLT_MAX;
        B.out.nodes.push_back(root);
    } else {
        B.node(0, n, 0);
    }
    B.out.order.resize(n);
    for (uint32_t i = 0; i < n; ++i) B.out.order[i] = B.refs[i].idx;
    // Renumber so the first kBvhTopNodes nodes in breadth-first order come first (the
    // trace kernel keeps them in LDS); the rest keep their depth-first order.  Traversal
    // results do not depend on node numbering.
    std::vector<BvhNode>& nodes = B.out.nodes;
    const size_t nn = nodes.size();
    std::vector<int32_t> remap(nn, -1);
    std::vector<uint32_t> order;
    order.reserve(nn);
    if (nn) order.push_back(0), remap[0] = 0;
    for (size_t head = 0; head < order.size() && order.size() < std::min<size_t>(nn, kBvhTopNodes); ++head) {
        const BvhNode& nd = nodes[order[head]];
        for (int c = 0; c < 2; ++c) {
            const int32_t idx = c ? nd.right : nd.left, cnt = c ? nd.rcount : nd.lcount;
            if (cnt == 0 && order.size() < std::min<size_t>(nn, kBvhTopNodes)) {
                remap[(size_t)idx] = (int32_t)order.size();
                order.push_back((uint32_t)idx);
            }
        }
    }
    for (size_t i = 0; i < nn; ++i)
        if (remap[i] < 0) remap[i] = (int32_t)order.size(), order.push_back((uint32_t)i);
    std::vector<BvhNode> out(nn);
    for (size_t i = 0; i < nn; ++i) {
        BvhNode nd = nodes[order[i]];
        if (nd.lcount == 0) nd.left = remap[(size_t)nd.left];
        if (nd.rcount == 0) nd.right = remap[(size_t)nd.right];
        out[i] = nd;
    }
    nodes.swap(out);
    return std::move(B.out);
}

namespace {
void emit_child(const BvhBuild& b, std::vector<SkipNode>& out, const float* mn, const float* mx, int32_t index,
                int32_t count) {
    if (count < 0) return;   // empty slot
    const size_t me = out.size();
    SkipNode s{};
    for (int q = 0; q < 3; ++q) s.bmin[q] = mn[q], s.bmax[q] = mx[q];
    s.leaf = count > 0 ? (int32_t)(((uint32_t)count << 24) | (uint32_t)index) : -1;
    out.push_back(s);
    if (count == 0) {
        const BvhNode& n = b.nodes[(size_t)index];
        emit_child(b, out, n.lmin, n.lmax, n.left, n.lcount);
        emit_child(b, out, n.rmin, n.rmax, n.right, n.rcount);
    }
    out[me].skip = (int32_t)out.size();
}
}  // namespace

std::vector<SkipNode> thread_bvh(const BvhBuild& b) {
    std::vector<SkipNode> out;
    if (b.nodes.empty()) return out;
    const BvhNode& r = b.nodes[0];
    emit_child(b, out, r.lmin, r.lmax, r.left, r.lcount);
    emit_child(b, out, r.rmin, r.rmax, r.right, r.rcount);
    return out;
}

namespace {
struct Child {
    const float* mn;
    const float* mx;
    int32_t index, count;
};
float child_area(const Child& c) {
    const float dx = c.mx[0] - c.mn[0], dy = c.mx[1] - c.mn[1], dz = c.mx[2] - c.mn[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}
}  // namespace

std::vector<Bvh4Node> collapse_bvh4(const BvhBuild& b, int& depth) {
    std::vector<Bvh4Node> out;
    depth = 0;
    if (b.nodes.empty()) return out;
    // breadth-first over binary interior nodes that become 4-wide nodes
    std::vector<std::pair<uint32_t, int>> queue{{0u, 0}};   // (binary node, depth)
    std::vector<std::vector<Child>> kids;
    for (size_t head = 0; head < queue.size(); ++head) {
        const BvhNode& n = b.nodes[queue[head].first];
        std::vector<Child> ch;
        if (n.lcount >= 0) ch.push_back(Child{n.lmin, n.lmax, n.left, n.lcount});
        if (n.rcount >= 0) ch.push_back(Child{n.rmin, n.rmax, n.right, n.rcount});
        while (ch.size() < 4) {   // open the interior child with the largest box
            int best = -1;
            for (size_t c = 0; c < ch.size(); ++c)
                if (ch[c].count == 0 && (best < 0 || child_area(ch[c]) > child_area(ch[(size_t)best]))) best = (int)c;
            if (best < 0) break;
            const BvhNode& m = b.nodes[(size_t)ch[(size_t)best].index];
            ch.erase(ch.begin() + best);
            if (m.lcount >= 0) ch.push_back(Child{m.lmin, m.lmax, m.left, m.lcount});
            if (m.rcount >= 0) ch.push_back(Child{m.rmin, m.rmax, m.right, m.rcount});
        }
        depth = std::max(depth, queue[head].second);
        for (Child& c : ch)
            if (c.count == 0) {   // becomes the 4-wide node numbered queue.size()
                queue.push_back({(uint32_t)c.index, queue[head].second + 1});
                c.index = (int32_t)(queue.size() - 1);
            }
        kids.push_back(std::move(ch));
    }
    out.resize(kids.size());
    for (size_t i = 0; i < kids.size(); ++i) {
        Bvh4Node& nd = out[i];
        for (int c = 0; c < 4; ++c) {
            const bool has = (size_t)c < kids[i].size();
            int32_t index = has ? kids[i][(size_t)c].index : 0, count = has ? kids[i][(size_t)c].count : -1;
            for (int q = 0; q < 3; ++q) {
                nd.lo[c][q] = has ? kids[i][(size_t)c].mn[q] : FLT_MAX;
                nd.hi[c][q] = has ? kids[i][(size_t)c].mx[q] : -FLT_MAX;
            }
            std::memcpy(&nd.lo[c][3], &index, 4);
            std::memcpy(&nd.hi[c][3], &count, 4);
        }
    }
    return out;
}

}  // namespace xrt
