// bvh_visits.cpp — CPU experiment: node / primitive tests per ray for the C3 sphere scene
// under the device's skip-link traversal versus an ordered (near-child-first, stack)
// traversal of the same binary BVH.  Not part of the product; decides which traversal the
// sphere path should use.  Build: g++ -O2 -std=c++17 -Ixraytracer_amd/csrc
//   tools/bvh_visits.cpp xraytracer_amd/csrc/host/bvh.cpp -o /tmp/bvh_visits
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "bvh.h"

using namespace xrt;
struct V { float x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V norm(V a) { float l = std::sqrt(dot(a, a)); return {a.x / l, a.y / l, a.z / l}; }

static bool sph(V o, V d, V c, float r, float& t) {
    V L = sub(o, c);
    float b = 2 * dot(d, L), cc = dot(L, L) - r * r, disc = b * b - 4 * cc;
    if (disc < 0) return false;
    float s = std::sqrt(disc), t0 = (-b - s) / 2, t1 = (-b + s) / 2;
    if (t0 < 0) t0 = t1;
    if (t0 < 0) return false;
    t = t0;
    return true;
}
static bool box(const float* mn, const float* mx, V o, V inv, float tl, float& tn) {
    float a[3] = {o.x, o.y, o.z}, iv[3] = {inv.x, inv.y, inv.z}, n = 0, f = tl;
    for (int q = 0; q < 3; ++q) {
        float t0 = (mn[q] - a[q]) * iv[q], t1 = (mx[q] - a[q]) * iv[q];
        n = std::fmax(n, std::fmin(t0, t1)), f = std::fmin(f, std::fmax(t0, t1));
    }
    tn = n;
    return !(n > f);
}

struct Cnt { double nodes = 0, prims = 0, rays = 0; };

int main() {
    std::vector<V> c;
    std::vector<float> r;
    for (int iz = 0; iz < 25; ++iz)
        for (int ix = 0; ix < 40; ++ix) c.push_back({-19.5f + ix, 0, -2.0f - iz}), r.push_back(0.4f);
    c.push_back({0, 10, -12}), r.push_back(2);
    const uint32_t n = (uint32_t)c.size();
    std::vector<float> mn(3 * n), mx(3 * n);
    for (uint32_t k = 0; k < n; ++k) {
        float cc[3] = {c[k].x, c[k].y, c[k].z};
        for (int q = 0; q < 3; ++q) mn[3 * k + q] = cc[q] - r[k] - 1e-3f, mx[3 * k + q] = cc[q] + r[k] + 1e-3f;
    }
    BvhBuild B = build_bvh(mn.data(), mx.data(), n, 4, 1e-3f, 48);
    std::vector<SkipNode> T = thread_bvh(B);
    printf("nodes binary %zu skip %zu depth %d\n", B.nodes.size(), T.size(), B.depth);

    auto skip = [&](V o, V d, float tmax, bool any, Cnt& C) {
        V inv{1 / d.x, 1 / d.y, 1 / d.z};
        float bt = any ? tmax : INFINITY, tn;
        int i = 0;
        C.rays++;
        while (i < (int)T.size()) {
            C.nodes++;
            if (!box(T[i].bmin, T[i].bmax, o, inv, bt, tn)) { i = T[i].skip; continue; }
            if (T[i].leaf >= 0) {
                int f = T[i].leaf & 0xffffff, e = f + (T[i].leaf >> 24);
                for (int j = f; j < e; ++j) {
                    C.prims++;
                    uint32_t k = B.order[j];
                    float t;
                    if (any && k == n - 1) continue;
                    if (sph(o, d, c[k], r[k], t) && t < bt) {
                        if (any) return;
                        bt = t;
                    }
                }
            }
            ++i;
        }
    };
    // ordered: node fetch tests both children, near first, far pushed with its entry t
    auto ordered = [&](V o, V d, float tmax, bool any, Cnt& C) {
        V inv{1 / d.x, 1 / d.y, 1 / d.z};
        float bt = any ? tmax : INFINITY;
        struct E { int idx, cnt; float tn; } st[64];
        int sp = 0;
        C.rays++;
        E cur{0, 0, 0};
        for (;;) {
            if (cur.cnt > 0) {
                for (int j = cur.idx; j < cur.idx + cur.cnt; ++j) {
                    C.prims++;
                    uint32_t k = B.order[j];
                    float t;
                    if (any && k == n - 1) continue;
                    if (sph(o, d, c[k], r[k], t) && t < bt) {
                        if (any) return;
                        bt = t;
                    }
                }
            } else {
                C.nodes++;
                const BvhNode& N = B.nodes[cur.idx];
                float tl, tr;
                bool hl = N.lcount >= 0 && box(N.lmin, N.lmax, o, inv, bt, tl);
                bool hr = N.rcount >= 0 && box(N.rmin, N.rmax, o, inv, bt, tr);
                E L{N.left, N.lcount, tl}, R{N.right, N.rcount, tr};
                if (hl && hr) {
                    if (tr < tl) std::swap(L, R);
                    st[sp++] = R, cur = L;
                    continue;
                }
                if (hl) { cur = L; continue; }
                if (hr) { cur = R; continue; }
            }
            for (;;) {
                if (!sp) return;
                cur = st[--sp];
                if (cur.tn <= bt) break;
            }
        }
    };
    const int W = 320, H = 180;
    const float tf = std::tan(30 * M_PI / 180), asp = (float)W / H;
    std::mt19937 g(1);
    std::uniform_real_distribution<float> U(0, 1);
    Cnt ps, po, ss, so;
    std::vector<double> rowS(H), rowO(H), rowSS(H), rowSO(H);
    double hits = 0;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            V o{0, 4, 8};
            V d = norm({(2 * (x + 0.5f) / W - 1) * asp * tf, (1 - 2 * (y + 0.5f) / H) * tf, -1});
            { Cnt a, b; skip(o, d, 0, false, a); ordered(o, d, 0, false, b); ps.nodes += a.nodes, ps.prims += a.prims, ps.rays++; po.nodes += b.nodes, po.prims += b.prims, po.rays++;
              rowS[y] = std::max(rowS[y], a.nodes + 4 * a.prims), rowO[y] = std::max(rowO[y], 2 * b.nodes + 4 * b.prims); }
            // closest hit by brute force for the shadow origin
            float bt = INFINITY;
            for (uint32_t k = 0; k < n; ++k) { float t; if (sph(o, d, c[k], r[k], t) && t < bt) bt = t; }
            if (!std::isfinite(bt)) continue;
            hits++;
            V p{o.x + bt * d.x, o.y + bt * d.y, o.z + bt * d.z};
            float u1 = U(g), u2 = U(g), zz = 1 - 2 * u1, rr = std::sqrt(std::fmax(0.f, 1 - zz * zz)), ph = 2 * M_PI * u2;
            V q{2 * rr * std::cos(ph), 10 + 2 * rr * std::sin(ph), -12 + 2 * zz};
            V sd = sub(q, p);
            float dist = std::sqrt(dot(sd, sd));
            sd = norm(sd);
            V so_{p.x + 1e-3f * sd.x, p.y + 1e-3f * sd.y, p.z + 1e-3f * sd.z};
            { Cnt a, b; skip(so_, sd, dist * 0.999f, true, a); ordered(so_, sd, dist * 0.999f, true, b); ss.nodes += a.nodes, ss.prims += a.prims, ss.rays++; so.nodes += b.nodes, so.prims += b.prims, so.rays++;
              rowSS[y] = std::max(rowSS[y], a.nodes + 4 * a.prims), rowSO[y] = std::max(rowSO[y], 2 * b.nodes + 4 * b.prims); }
        }
    for (int y = 0; y < H; y += 6) printf("row %3d max cost primary skip %5.0f ordered %5.0f | shadow skip %5.0f ordered %5.0f\n", y, rowS[y], rowO[y], rowSS[y], rowSO[y]);
    printf("primary rays %.0f (hit %.0f)\n", ps.rays, hits);
    printf("primary skip:    nodes %.1f prims %.1f per ray\n", ps.nodes / ps.rays, ps.prims / ps.rays);
    printf("primary ordered: nodes %.1f (x2 boxes) prims %.1f per ray\n", po.nodes / po.rays, po.prims / po.rays);
    printf("shadow  skip:    nodes %.1f prims %.1f per ray\n", ss.nodes / ss.rays, ss.prims / ss.rays);
    printf("shadow  ordered: nodes %.1f (x2 boxes) prims %.1f per ray\n", so.nodes / so.rays, so.prims / so.rays);
}
