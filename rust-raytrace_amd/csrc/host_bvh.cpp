// Sphere BVH builder (host).  The reference has no acceleration structure: its
// Scene::intersect (scene.rs:247-249) tests every object.  The BVH only decides
// which spheres a ray is TESTED against; the leaf test is the reference's
// exact f64 quadratic and the winner is chosen by (NaN, t, object id) exactly
// as min_by_key does, so the result is identical whenever the culling is
// conservative ("BVH exactness").  Conservative here:
//   * each sphere's box is [c - r, c + r] widened by `pad` and rounded OUTWARD
//     to f32 (so it contains every point the f64 test can report as a hit);
//   * the traversal (trace_common.hpp, box_hit) widens every slab interval by
//     a relative 1e-5, covering f32 rounding of the ray and of the slab math.
// Binned SAH (16 bins) with leaves of <= 4 spheres; median split below depth
// 40 keeps the depth (and the per-lane traversal stack) bounded.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "bvh_build.hpp"

namespace rtamd {
namespace {

float down(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) > x) f = std::nextafter(f, -FLT_MAX);
    return f;
}
float up(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) < x) f = std::nextafter(f, FLT_MAX);
    return f;
}

struct Box {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL};
    double hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    double area() const {
        double d[3];
        for (int a = 0; a < 3; ++a) d[a] = std::max(0.0, hi[a] - lo[a]);
        return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct Prim {
    Box box;
    double c[3];
    int32_t idx;
};

constexpr int kBins = 16;
constexpr int kSahDepth = 40;

struct Builder {
    std::vector<Prim>& prims;
    std::vector<BvhNodeHost>& nodes;
    double pad;
    int leaf_max;

    Box bounds(int b, int e) const {
        Box r;
        for (int i = b; i < e; ++i) r.grow(prims[i].box);
        return r;
    }

    // Returns the encoded child pointer for prims[b, e).
    int32_t build(int b, int e, int depth) {
        const int n = e - b;
        if (n <= leaf_max) return ~((b << 3) | (n - 1));
        Box cb;                         // centroid bounds
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) { cb.lo[a] = std::min(cb.lo[a], prims[i].c[a]); cb.hi[a] = std::max(cb.hi[a], prims[i].c[a]); }
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (cb.hi[a] - cb.lo[a] > cb.hi[axis] - cb.lo[axis]) axis = a;
        int mid = -1;
        const double ext = cb.hi[axis] - cb.lo[axis];
        if (depth < kSahDepth && ext > 0) {
            // binned SAH over all three axes
            double best = HUGE_VAL;
            int best_axis = -1, best_bin = -1;
            for (int a = 0; a < 3; ++a) {
                const double ea = cb.hi[a] - cb.lo[a];
                if (!(ea > 0)) continue;
                Box bb[kBins];
                int bc[kBins] = {0};
                for (int i = b; i < e; ++i) {
                    int k = static_cast<int>((prims[i].c[a] - cb.lo[a]) / ea * kBins);
                    k = std::min(kBins - 1, std::max(0, k));
                    bb[k].grow(prims[i].box);
                    ++bc[k];
                }
                Box lb[kBins], rb[kBins];
                int lc[kBins], rc[kBins];
                Box acc;
                int cnt = 0;
                for (int k = 0; k < kBins; ++k) { acc.grow(bb[k]); cnt += bc[k]; lb[k] = acc; lc[k] = cnt; }
                acc = Box();
                cnt = 0;
                for (int k = kBins - 1; k >= 0; --k) { acc.grow(bb[k]); cnt += bc[k]; rb[k] = acc; rc[k] = cnt; }
                for (int k = 0; k < kBins - 1; ++k) {
                    if (lc[k] == 0 || rc[k + 1] == 0) continue;
                    const double cost = lb[k].area() * lc[k] + rb[k + 1].area() * rc[k + 1];
                    if (cost < best) { best = cost; best_axis = a; best_bin = k; }
                }
            }
            if (best_axis >= 0) {
                const int a = best_axis;
                const double ea = cb.hi[a] - cb.lo[a];
                auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim& p) {
                    int k = static_cast<int>((p.c[a] - cb.lo[a]) / ea * kBins);
                    k = std::min(kBins - 1, std::max(0, k));
                    return k <= best_bin;
                });
                mid = static_cast<int>(it - prims.begin());
                if (mid == b || mid == e) mid = -1;
            }
        }
        if (mid < 0) {                  // median split (also for coincident centroids)
            mid = b + n / 2;
            std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e,
                             [&](const Prim& p, const Prim& q) {
                                 return p.c[axis] < q.c[axis] || (p.c[axis] == q.c[axis] && p.idx < q.idx);
                             });
        }
        const int32_t self = static_cast<int32_t>(nodes.size());
        nodes.emplace_back();
        const Box l = bounds(b, mid), r = bounds(mid, e);
        const int32_t c0 = build(b, mid, depth + 1);
        const int32_t c1 = build(mid, e, depth + 1);
        BvhNodeHost& nd = nodes[self];
        for (int a = 0; a < 3; ++a) {
            nd.lo0[a] = down(l.lo[a]); nd.hi0[a] = up(l.hi[a]);
            nd.lo1[a] = down(r.lo[a]); nd.hi1[a] = up(r.hi[a]);
        }
        nd.c0 = c0;
        nd.c1 = c1;
        return self;
    }
};

}  // namespace

BvhResult build_sphere_bvh(const std::vector<double>& cx, const std::vector<double>& cy, const std::vector<double>& cz,
                           const std::vector<double>& radius, double pad, int leaf_max) {
    BvhResult res;
    const size_t n = cx.size();
    if (n == 0) { res.root = 0; return res; }
    std::vector<Prim> prims(n);
    for (size_t i = 0; i < n; ++i) {
        Prim& p = prims[i];
        const double c[3] = {cx[i], cy[i], cz[i]};
        const double r = std::fabs(radius[i]);
        for (int a = 0; a < 3; ++a) {
            p.c[a] = c[a];
            // a NaN radius/centre never produces a hit (disc > 0 is false): any box works
            p.box.lo[a] = std::isfinite(c[a] - r) ? c[a] - r - pad : -HUGE_VAL;
            p.box.hi[a] = std::isfinite(c[a] + r) ? c[a] + r + pad : HUGE_VAL;
            if (!std::isfinite(p.c[a])) p.c[a] = 0.0;
        }
        p.idx = static_cast<int32_t>(i);
    }
    leaf_max = std::min(8, std::max(1, leaf_max));
    res.nodes.reserve(2 * n / leaf_max + 2);
    Builder bld{prims, res.nodes, pad, leaf_max};
    res.root = bld.build(0, static_cast<int>(n), 0);
    // Renumber breadth-first so the top levels are a prefix of the array: the
    // traversal kernels keep the first nodes that fit in LDS.
    if (res.root >= 0 && !res.nodes.empty()) {
        std::vector<int32_t> order, remap(res.nodes.size(), -1);
        order.reserve(res.nodes.size());
        order.push_back(res.root);
        for (size_t h = 0; h < order.size(); ++h) {
            const BvhNodeHost& nd = res.nodes[order[h]];
            if (nd.c0 >= 0) order.push_back(nd.c0);
            if (nd.c1 >= 0) order.push_back(nd.c1);
        }
        for (size_t k = 0; k < order.size(); ++k) remap[order[k]] = static_cast<int32_t>(k);
        std::vector<BvhNodeHost> bfs(order.size());
        for (size_t k = 0; k < order.size(); ++k) {
            bfs[k] = res.nodes[order[k]];
            if (bfs[k].c0 >= 0) bfs[k].c0 = remap[bfs[k].c0];
            if (bfs[k].c1 >= 0) bfs[k].c1 = remap[bfs[k].c1];
        }
        res.nodes.swap(bfs);
        res.root = 0;
    }
    res.order.resize(n);
    for (size_t i = 0; i < n; ++i) res.order[i] = prims[i].idx;
    return res;
}

// Collapse: each 4-wide node takes the two children of a binary node and
// repeatedly opens the inner child with the largest box area until it has 4
// children or only leaves.  Child boxes are the binary tree's f32 boxes
// unchanged (so the culling stays conservative), numbered breadth-first.
Bvh4Result collapse_bvh4(const BvhResult& b2) {
    Bvh4Result out;
    out.root = b2.root;
    if (b2.nodes.empty() || b2.root < 0) return out;
    struct Ref {
        int32_t ptr;
        float lo[3], hi[3];
    };
    auto area = [](const Ref& r) {
        const double dx = r.hi[0] - r.lo[0], dy = r.hi[1] - r.lo[1], dz = r.hi[2] - r.lo[2];
        return dx * dy + dy * dz + dz * dx;
    };
    auto children = [&](int32_t node, Ref& a, Ref& b) {
        const BvhNodeHost& nd = b2.nodes[node];
        a.ptr = nd.c0; b.ptr = nd.c1;
        for (int k = 0; k < 3; ++k) { a.lo[k] = nd.lo0[k]; a.hi[k] = nd.hi0[k]; b.lo[k] = nd.lo1[k]; b.hi[k] = nd.hi1[k]; }
    };
    struct Node4 {
        Ref c[4];
        int n;
    };
    std::vector<Node4> nodes;
    std::vector<int32_t> queue{b2.root};       // binary node of each 4-wide node, breadth-first
    for (size_t h = 0; h < queue.size(); ++h) {
        Node4 nd{};
        children(queue[h], nd.c[0], nd.c[1]);
        nd.n = 2;
        while (nd.n < 4) {
            int best = -1;
            double best_area = -1.0;
            for (int k = 0; k < nd.n; ++k)
                if (nd.c[k].ptr >= 0 && area(nd.c[k]) > best_area) { best = k; best_area = area(nd.c[k]); }
            if (best < 0) break;
            Ref a, b;
            children(nd.c[best].ptr, a, b);
            nd.c[best] = a;
            nd.c[nd.n++] = b;
        }
        for (int k = 0; k < nd.n; ++k)
            if (nd.c[k].ptr >= 0) {
                const int32_t binary = nd.c[k].ptr;
                nd.c[k].ptr = static_cast<int32_t>(queue.size());   // its 4-wide index
                queue.push_back(binary);
            }
        nodes.push_back(nd);
    }
    const int32_t N = static_cast<int32_t>(nodes.size());
    out.n_nodes = N;
    out.root = 0;
    out.planes.assign(static_cast<size_t>(kBvh4Planes) * N, DevBvh4Plane{});
    for (int32_t i = 0; i < N; ++i) {
        const Node4& nd = nodes[i];
        for (int k = 0; k < 4; ++k) {
            const bool used = k < nd.n;
            for (int a = 0; a < 3; ++a) {
                out.planes[static_cast<size_t>(2 * a) * N + i].f[k] = used ? nd.c[k].lo[a] : 0.0f;
                out.planes[static_cast<size_t>(2 * a + 1) * N + i].f[k] = used ? nd.c[k].hi[a] : 0.0f;
            }
            out.planes[static_cast<size_t>(6) * N + i].i[k] = used ? nd.c[k].ptr : kBvh4Empty;
        }
    }
    return out;
}

// Quantise the 4-wide tree (DevQNode4).  Per node and axis, the frame step is
// the smallest power of two s = 2^e (e >= -100) for which the node's f32 box
// [L, H] spans at most 255 steps from m = floor(L / s) and m fits 24 bits
// signed; child bounds round outward to whole steps: lo' = floor(lo / s) * s,
// hi' = ceil(hi / s) * s.  Every quantity is a power-of-two multiple of an f32,
// so the double arithmetic here is exact, and so is the device's decode
// fma(q, s, m * s) = (m + q) * s (an integer below 2^24 times a power of two
// in the normal range).
std::vector<DevQNode4> quantize_bvh4(const Bvh4Result& b4) {
    const int32_t N = b4.n_nodes;
    if (N <= 0 || N >= 0x8000 || b4.root != 0) return {};
    std::vector<DevQNode4> out(static_cast<size_t>(N));
    for (int32_t i = 0; i < N; ++i) {
        DevQNode4& q = out[i];
        std::memset(&q, 0, sizeof q);
        const DevBvh4Plane& ch = b4.planes[static_cast<size_t>(6) * N + i];
        bool used[4];
        int32_t first_leaf = INT32_MAX;
        for (int k = 0; k < 4; ++k) {
            used[k] = ch.i[k] != kBvh4Empty;
            if (used[k] && ch.i[k] < 0) first_leaf = std::min(first_leaf, (~ch.i[k]) >> 3);
        }
        q.base = first_leaf == INT32_MAX ? 0u : static_cast<uint32_t>(first_leaf);
        for (int k = 0; k < 4; ++k) {
            if (!used[k]) { q.child[k] = kQ4Empty; continue; }
            const int32_t c = ch.i[k];
            if (c >= 0) { q.child[k] = static_cast<uint16_t>(c); continue; }
            const int32_t off = ((~c) >> 3) - first_leaf, cnt = ((~c) & 7) + 1;
            if (off > 4094) return {};
            q.child[k] = static_cast<uint16_t>(kQ4Leaf | (off << 3) | (cnt - 1));
        }
        for (int a = 0; a < 3; ++a) {
            const DevBvh4Plane& P0 = b4.planes[static_cast<size_t>(2 * a) * N + i];
            const DevBvh4Plane& P1 = b4.planes[static_cast<size_t>(2 * a + 1) * N + i];
            double L = HUGE_VAL, H = -HUGE_VAL;
            for (int k = 0; k < 4; ++k) {
                if (!used[k]) continue;
                if (!std::isfinite(P0.f[k]) || !std::isfinite(P1.f[k]) || !(P0.f[k] <= P1.f[k])) return {};
                L = std::min(L, static_cast<double>(P0.f[k]));
                H = std::max(H, static_cast<double>(P1.f[k]));
            }
            if (!(L <= H)) { L = 0.0; H = 0.0; }       // no child (cannot happen for a collapsed node)
            int e = -100;
            if (H > L) e = std::max(e, static_cast<int>(std::ceil(std::log2((H - L) / 255.0))) - 1);
            double m = 0.0, s = 0.0;
            for (;; ++e) {
                if (e > 104) return {};
                s = std::ldexp(1.0, e);
                m = std::floor(L / s);
                if (m < -8388608.0 || m > 8388607.0) continue;
                if (std::ceil(H / s) - m <= 255.0) break;
            }
            uint32_t lo = 0, hi = 0;
            for (int k = 0; k < 4; ++k) {
                if (!used[k]) continue;
                const double ql = std::floor(P0.f[k] / s) - m, qh = std::ceil(P1.f[k] / s) - m;
                if (!(ql >= 0.0 && qh <= 255.0 && ql <= qh)) return {};
                lo |= static_cast<uint32_t>(ql) << (8 * k);
                hi |= static_cast<uint32_t>(qh) << (8 * k);
            }
            q.frame[a] = static_cast<int32_t>((static_cast<uint32_t>(static_cast<int32_t>(m)) & 0xFFFFFFu) |
                                              (static_cast<uint32_t>(e + 127) << 24));
            q.lo[a] = lo;
            q.hi[a] = hi;
        }
    }
    return out;
}

int bvh4_stack_need(const Bvh4Result& b4) {
    if (b4.root < 0 || b4.n_nodes == 0) return 1;
    const int N = b4.n_nodes;
    int worst = 0;
    std::vector<std::pair<int32_t, int>> todo{{b4.root, 0}};      // (node, pending siblings above it)
    while (!todo.empty()) {
        const auto [node, pend] = todo.back();
        todo.pop_back();
        const DevBvh4Plane& ch = b4.planes[static_cast<size_t>(6) * N + node];
        int kids = 0;
        for (int k = 0; k < 4; ++k) kids += ch.i[k] != kBvh4Empty ? 1 : 0;
        const int here = pend + std::max(0, kids - 1);
        worst = std::max(worst, here);
        for (int k = 0; k < 4; ++k)
            if (ch.i[k] != kBvh4Empty && ch.i[k] >= 0) todo.push_back({ch.i[k], here});
    }
    return worst + 1;
}

float half_to_float(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    const float sign = (h & 0x8000) ? -1.0f : 1.0f;
    if (e == 31) return m ? std::numeric_limits<float>::quiet_NaN() : sign * std::numeric_limits<float>::infinity();
    // both forms are exact in f32 (11 significant bits)
    return sign * (e == 0 ? std::ldexp(static_cast<float>(m), -24) : std::ldexp(static_cast<float>(1024 + m), e - 25));
}

namespace {
// Finite halves in value order: key k in [-0x7BFF, 0x7BFF] <-> bits (k >= 0 ? k : 0x8000 | -k).
uint16_t half_of_key(int k) { return static_cast<uint16_t>(k >= 0 ? k : (0x8000 | -k)); }
constexpr int kHalfMaxKey = 0x7BFF;   // 65504
}  // namespace

bool half_round_down(float v, uint16_t& out) {
    if (!(std::fabs(v) <= 65504.0f)) return false;          // NaN, inf or outside the finite range
    int lo = -kHalfMaxKey, hi = kHalfMaxKey;                 // largest key with value <= v (value(lo) <= v)
    while (lo < hi) {
        const int mid = lo + (hi - lo + 1) / 2;
        if (half_to_float(half_of_key(mid)) <= v) lo = mid; else hi = mid - 1;
    }
    out = half_of_key(lo);
    return true;
}

bool half_round_up(float v, uint16_t& out) {
    if (!(std::fabs(v) <= 65504.0f)) return false;
    int lo = -kHalfMaxKey, hi = kHalfMaxKey;                 // smallest key with value >= v
    while (lo < hi) {
        const int mid = lo + (hi - lo) / 2;
        if (half_to_float(half_of_key(mid)) >= v) hi = mid; else lo = mid + 1;
    }
    out = half_of_key(lo);
    return true;
}

std::vector<DevBvhNodeH> half_nodes(const BvhResult& b2) {
    std::vector<DevBvhNodeH> out(b2.nodes.size());
    for (size_t k = 0; k < b2.nodes.size(); ++k) {
        const DevBvhNode& n = b2.nodes[k];
        DevBvhNodeH& h = out[k];
        for (int a = 0; a < 3; ++a) {
            if (!half_round_down(n.lo0[a], h.b[a]) || !half_round_up(n.hi0[a], h.b[3 + a]) ||
                !half_round_down(n.lo1[a], h.b[6 + a]) || !half_round_up(n.hi1[a], h.b[9 + a]))
                return {};
        }
        h.c0 = n.c0;
        h.c1 = n.c1;
    }
    return out;
}

int bvh_depth(const BvhResult& b2) {
    if (b2.root < 0 || b2.nodes.empty()) return 0;
    int worst = 0;
    std::vector<std::pair<int32_t, int>> todo{{b2.root, 1}};
    while (!todo.empty()) {
        const auto [node, d] = todo.back();
        todo.pop_back();
        worst = std::max(worst, d);
        for (int32_t c : {b2.nodes[node].c0, b2.nodes[node].c1})
            if (c >= 0) todo.push_back({c, d + 1});
    }
    return worst;
}

}  // namespace rtamd
