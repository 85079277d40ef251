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

// Image-plane rectangle of a box seen from the camera.  A camera ray is
// dir = normalize(M (px, py, 1)) (camera.rs:78), so a world point X it passes
// through has M^-1 (X - pos) = s (px, py, 1) with s > 0.  When every corner of
// the box lies strictly in front of the camera plane (third coordinate > 0),
// the box's image is the convex hull of the corner images (the perspective map
// keeps segments straight on that side), so their bounding rectangle holds
// every (px, py) whose ray meets the box.  A relative 1e-5 margin absorbs the
// rounding of the ray direction and of this projection (far below a pixel).
namespace {
void project_box(const float lo[3], const float hi[3], const double pos[3], const double inv[9], float rect[4],
                 float& tmin) {
    double r[4] = {HUGE_VAL, HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    bool front = true;
    for (int c = 0; c < 8 && front; ++c) {
        const double X[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
        const double d[3] = {X[0] - pos[0], X[1] - pos[1], X[2] - pos[2]};
        double q[3];
        for (int i = 0; i < 3; ++i) q[i] = inv[3 * i] * d[0] + inv[3 * i + 1] * d[1] + inv[3 * i + 2] * d[2];
        const double dn = std::fabs(d[0]) + std::fabs(d[1]) + std::fabs(d[2]);
        if (!(q[2] > 1e-9 * dn) || !std::isfinite(q[0]) || !std::isfinite(q[1])) { front = false; break; }
        const double px = q[0] / q[2], py = q[1] / q[2];
        r[0] = std::min(r[0], px); r[1] = std::min(r[1], py);
        r[2] = std::max(r[2], px); r[3] = std::max(r[3], py);
    }
    if (!front) {
        rect[0] = rect[1] = -HUGE_VALF;
        rect[2] = rect[3] = HUGE_VALF;
    } else {
        for (int i = 0; i < 2; ++i) rect[i] = down(r[i] - 1e-5 * (1.0 + std::fabs(r[i])));
        for (int i = 2; i < 4; ++i) rect[i] = up(r[i] + 1e-5 * (1.0 + std::fabs(r[i])));
    }
    // distance from the camera to the box: a hit inside it is at t >= this
    // (unit direction up to rounding; the 1e-6 relative cut covers that)
    double dd = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double v = pos[a] < lo[a] ? lo[a] - pos[a] : (pos[a] > hi[a] ? pos[a] - hi[a] : 0.0);
        dd += v * v;
    }
    const double dist = std::sqrt(dd) * (1.0 - 1e-6);
    tmin = std::isfinite(dist) ? down(dist) : 0.0f;
}
}  // namespace

std::vector<DevCamNode> camera_nodes(const BvhResult& b2, const double pos[3], const double m[9]) {
    std::vector<DevCamNode> out(b2.nodes.size());
    // M^-1 by the adjugate
    const double a = m[0], b = m[1], c = m[2], d = m[3], e = m[4], f = m[5], g = m[6], h = m[7], i = m[8];
    const double det = a * (e * i - f * h) - b * (d * i - f * g) + c * (d * h - e * g);
    const double inv[9] = {(e * i - f * h) / det, (c * h - b * i) / det, (b * f - c * e) / det,
                           (f * g - d * i) / det, (a * i - c * g) / det, (c * d - a * f) / det,
                           (d * h - e * g) / det, (b * g - a * h) / det, (a * e - b * d) / det};
    bool ok = std::isfinite(det) && det != 0.0;
    for (double v : inv) ok = ok && std::isfinite(v);
    for (size_t k = 0; k < b2.nodes.size(); ++k) {
        const DevBvhNode& n = b2.nodes[k];
        DevCamNode& o = out[k];
        if (ok) {
            project_box(n.lo0, n.hi0, pos, inv, o.r0, o.tmin0);
            project_box(n.lo1, n.hi1, pos, inv, o.r1, o.tmin1);
        } else {                                  // degenerate camera: every box everywhere
            for (float* r : {o.r0, o.r1}) { r[0] = r[1] = -HUGE_VALF; r[2] = r[3] = HUGE_VALF; }
            o.tmin0 = o.tmin1 = 0.0f;
        }
        o.c0 = n.c0;
        o.c1 = n.c1;
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

ClusterResult build_clusters(const BvhResult& b2, size_t n_spheres) {
    ClusterResult out;
    if (n_spheres == 0) return out;
    // (first, count) of every subtree: the builder partitions in place, so a
    // subtree's spheres are one contiguous range of the leaf order
    auto range = [&](int32_t ptr, auto&& self) -> std::pair<int32_t, int32_t> {
        if (ptr < 0) return {(~ptr) >> 3, ((~ptr) & 7) + 1};
        const auto a = self(b2.nodes[ptr].c0, self), b = self(b2.nodes[ptr].c1, self);
        return {std::min(a.first, b.first), a.second + b.second};
    };
    auto cut = [&](int32_t ptr, const float lo[3], const float hi[3], auto&& self) -> void {
        const auto r = range(ptr, range);
        if (ptr < 0 || r.second <= kClusterMax) {
            DevCluster c{};
            for (int k = 0; k < 3; ++k) { c.lo[k] = lo[k]; c.hi[k] = hi[k]; }
            c.first = r.first;
            c.count = r.second;
            out.clusters.push_back(c);
            return;
        }
        const DevBvhNode& nd = b2.nodes[ptr];
        self(nd.c0, nd.lo0, nd.hi0, self);
        self(nd.c1, nd.lo1, nd.hi1, self);
    };
    const float inf = std::numeric_limits<float>::infinity();
    const float all_lo[3] = {-inf, -inf, -inf}, all_hi[3] = {inf, inf, inf};
    if (b2.root < 0) {                                   // the whole set is one leaf: one cluster, any ray tests it
        cut(b2.root, all_lo, all_hi, cut);
    } else {
        const DevBvhNode& r = b2.nodes[b2.root];
        cut(r.c0, r.lo0, r.hi0, cut);
        cut(r.c1, r.lo1, r.hi1, cut);
    }
    const size_t n = out.clusters.size();
    if (n > static_cast<size_t>(64 * kClusterSlotsMax) || n >= kClusterNone) { out.clusters.clear(); return out; }
    out.slots = static_cast<int>((n + 63) / 64);
    const size_t ns = static_cast<size_t>(64) * out.slots;
    out.perm.assign(8 * ns, kClusterNone);
    std::vector<uint16_t> ids(n);
    for (int o = 0; o < 8; ++o) {
        // octant o: bit a set = the ray's direction component a is negative; clusters
        // sorted by centre . s (s_a = +1 / -1), so the ones a ray meets first come first
        const double sx = (o & 1) ? -1.0 : 1.0, sy = (o & 2) ? -1.0 : 1.0, sz = (o & 4) ? -1.0 : 1.0;
        auto key = [&](uint16_t i) {
            const DevCluster& c = out.clusters[i];
            const double cx = 0.5 * (static_cast<double>(c.lo[0]) + c.hi[0]);
            const double cy = 0.5 * (static_cast<double>(c.lo[1]) + c.hi[1]);
            const double cz = 0.5 * (static_cast<double>(c.lo[2]) + c.hi[2]);
            const double k = sx * cx + sy * cy + sz * cz;
            return std::isfinite(k) ? k : -HUGE_VAL;
        };
        for (size_t i = 0; i < n; ++i) ids[i] = static_cast<uint16_t>(i);
        std::stable_sort(ids.begin(), ids.end(), [&](uint16_t a, uint16_t b) { return key(a) < key(b); });
        for (size_t i = 0; i < n; ++i) out.perm[o * ns + i] = ids[i];
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
