// Light-view grids for point-light shadow queries (DESIGN.md "Light-view grids").
//
// A shadow query toward a point light (raytrace.rs:39-49) asks whether some
// sphere reports a hit with t*t < |L - p|^2 on the ray from p toward L.  Such a
// hit point h lies on the segment between p and L (or within the 1e-5 offset
// past L), inside the sphere's padded box (the BVH's pad, DESIGN.md "BVH
// exactness"), and its direction from L is the direction of p from L up to
// f64 rounding.  So the spheres whose padded boxes cover that direction, as
// seen from L, are a superset of the possible blockers: each cell of a cube
// map around L lists the spheres whose box projects onto it.  The device
// tests exactly those spheres with the exact quadratic (any-hit), which gives
// the same answer as testing all of them.  Spheres whose box comes within
// kNearLight of L (and non-finite ones) are tested for every query instead.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "bvh_build.hpp"

namespace rtamd {
namespace {

constexpr double kNearLight = 1e-3;     // >> the 1e-5 offset past L a hit may have
constexpr double kUMargin = 1e-5;       // face-coordinate margin >> the device's f32 rounding (~3e-7)

struct Range {
    double lo, hi;
    bool empty() const { return !(lo <= hi); }
};

// Face coordinate range of u = d_b / d_a' over the box points with d_a' > 0,
// where d_a' in [amin, amax] (amax > 0) and d_b in [blo, bhi].
Range face_range(double amin, double amax, double blo, double bhi) {
    const double inf = std::numeric_limits<double>::infinity();
    if (amin > 0.0) {
        return Range{std::min(blo / amin, blo / amax), std::max(bhi / amin, bhi / amax)};
    }
    // d_a' reaches 0+: u is unbounded on the side where d_b can have that sign
    return Range{blo >= 0.0 ? blo / amax : -inf, bhi <= 0.0 ? bhi / amax : inf};
}

int cell_of(double u, int R) {
    const double x = std::floor((u + 1.0) * 0.5 * R);
    if (!(x >= 0.0)) return 0;          // also -inf
    if (x > R - 1) return R - 1;
    return static_cast<int>(x);
}

}  // namespace

LightGridResult build_light_grids(const std::vector<DevSphere>& spheres, const std::vector<double>& r_leaf,
                                  const std::vector<DevLight>& lights, double pad, int r_override) {
    LightGridResult out;
    out.grids.assign(lights.size(), DevLightGrid{});
    const size_t n = spheres.size();
    for (size_t li = 0; li < lights.size(); ++li) {
        const DevLight& Lt = lights[li];
        DevLightGrid& g = out.grids[li];
        g.R = 0;
        if (Lt.kind != 0 || n == 0) continue;            // point lights only (rt_light_kind RT_LIGHT_POINT)
        const double L[3] = {Lt.v[0], Lt.v[1], Lt.v[2]};
        if (!std::isfinite(L[0]) || !std::isfinite(L[1]) || !std::isfinite(L[2])) continue;
        g.lx = L[0]; g.ly = L[1]; g.lz = L[2];
        // boxes relative to L, widened for the subtraction's rounding
        std::vector<double> lo(3 * n), hi(3 * n), nearv(n);
        std::vector<char> always(n, 0);
        std::vector<double> ang;
        for (size_t k = 0; k < n; ++k) {
            const double c[3] = {spheres[k].cx, spheres[k].cy, spheres[k].cz};
            const double r = std::fabs(r_leaf[k]) + pad;
            double d2 = 0.0;
            bool finite = std::isfinite(r);
            bool at_light = true;
            for (int i = 0; i < 3; ++i) {
                double a = c[i] - r - L[i], b = c[i] + r - L[i];
                a -= 1e-12 * (1.0 + std::fabs(a));
                b += 1e-12 * (1.0 + std::fabs(b));
                lo[3 * k + i] = a; hi[3 * k + i] = b;
                finite &= std::isfinite(a) && std::isfinite(b);
                at_light &= a - kNearLight <= 0.0 && 0.0 <= b + kNearLight;
                const double gap = std::max({0.0, a, -b});
                d2 += gap * gap;
            }
            always[k] = !finite || at_light;
            nearv[k] = finite ? std::sqrt(d2) : 0.0;
            if (!always[k]) {
                const double dc = std::sqrt((c[0] - L[0]) * (c[0] - L[0]) + (c[1] - L[1]) * (c[1] - L[1]) +
                                            (c[2] - L[2]) * (c[2] - L[2]));
                if (dc > r) ang.push_back(std::asin(std::min(1.0, r / dc)));
            }
        }
        // R: a cell about the median sphere's angular radius (u = tan, du/dtheta >= 1)
        int R = 64;
        if (!ang.empty()) {
            std::nth_element(ang.begin(), ang.begin() + ang.size() / 2, ang.end());
            const double th = ang[ang.size() / 2];
            R = static_cast<int>(std::lround(std::clamp(2.0 / std::max(th, 1e-6), 16.0, 512.0)));
        }
        if (r_override > 0) R = r_override;
        g.R = R;
        // the always list
        g.always_begin = static_cast<uint32_t>(out.ent.size());
        for (size_t k = 0; k < n; ++k)
            if (always[k]) out.ent.push_back(DevLgEntry{static_cast<int32_t>(k), 0.0f});
        g.always_end = static_cast<uint32_t>(out.ent.size());
        // per face: cell rectangles of each sphere, then the face's bounding rectangle
        for (int f = 0; f < 6; ++f) {
            const int a = f >> 1, b = (a + 1) % 3, cax = (a + 2) % 3;
            const double s = (f & 1) ? -1.0 : 1.0;
            struct Rect { int i0, i1, j0, j1; };
            std::vector<Rect> rect(n, Rect{1, 0, 1, 0});
            int fx0 = R, fx1 = -1, fy0 = R, fy1 = -1;
            for (size_t k = 0; k < n; ++k) {
                if (always[k]) continue;
                const double alo = s > 0 ? lo[3 * k + a] : -hi[3 * k + a];
                const double ahi = s > 0 ? hi[3 * k + a] : -lo[3 * k + a];
                if (!(ahi > 0.0)) continue;
                const Range u = face_range(alo, ahi, lo[3 * k + b], hi[3 * k + b]);
                const Range v = face_range(alo, ahi, lo[3 * k + cax], hi[3 * k + cax]);
                if (u.empty() || v.empty() || u.lo > 1.0 + kUMargin || u.hi < -1.0 - kUMargin ||
                    v.lo > 1.0 + kUMargin || v.hi < -1.0 - kUMargin)
                    continue;
                Rect& q = rect[k];
                q.i0 = cell_of(u.lo - kUMargin, R); q.i1 = cell_of(u.hi + kUMargin, R);
                q.j0 = cell_of(v.lo - kUMargin, R); q.j1 = cell_of(v.hi + kUMargin, R);
                fx0 = std::min(fx0, q.i0); fx1 = std::max(fx1, q.i1);
                fy0 = std::min(fy0, q.j0); fy1 = std::max(fy1, q.j1);
            }
            g.off_base[f] = static_cast<uint32_t>(out.off.size());
            if (fx1 < fx0) {                          // nothing projects onto this face
                g.fx0[f] = 0; g.fy0[f] = 0; g.fw[f] = 0; g.fh[f] = 0;
                continue;
            }
            const int w = fx1 - fx0 + 1, h = fy1 - fy0 + 1;
            g.fx0[f] = fx0; g.fy0[f] = fy0; g.fw[f] = w; g.fh[f] = h;
            std::vector<std::vector<int32_t>> cells(static_cast<size_t>(w) * h);
            for (size_t k = 0; k < n; ++k) {
                const Rect& q = rect[k];
                if (q.i1 < q.i0) continue;
                for (int j = q.j0; j <= q.j1; ++j)
                    for (int i = q.i0; i <= q.i1; ++i)
                        cells[static_cast<size_t>(j - fy0) * w + (i - fx0)].push_back(static_cast<int32_t>(k));
            }
            for (auto& cl : cells) {
                std::sort(cl.begin(), cl.end(), [&](int32_t x, int32_t y) {
                    return nearv[x] < nearv[y] || (nearv[x] == nearv[y] && x < y);
                });
                out.off.push_back(static_cast<uint32_t>(out.ent.size()));
                for (int32_t k : cl) {
                    // f32 lower bound of the box distance
                    float nf = static_cast<float>(nearv[k]);
                    if (static_cast<double>(nf) > nearv[k]) nf = std::nextafter(nf, 0.0f);
                    out.ent.push_back(DevLgEntry{k, nf});
                }
            }
            out.off.push_back(static_cast<uint32_t>(out.ent.size()));
        }
    }
    return out;
}

// View grid of the camera: the same cube map, centred on the
// camera position, for the camera rays' NEAREST-hit query.  Every camera ray
// starts at the camera, so a hit point's direction from the camera is the ray
// direction (up to f64 rounding) and it lies in the sphere's padded box: the
// ray's cell lists every sphere that can report a hit.  Lists are sorted by
// box distance from the camera (f32, rounded down), which bounds t from below,
// so the device stops at the first entry beyond its current best t.  R cells
// per face side; halved until the lists hold at most `max_entries` entries
// (built by counting per cell, then filling, so large faces stay cheap).
LightGridResult build_view_grid(const std::vector<DevSphere>& spheres, const std::vector<double>& r_leaf,
                                const double pos[3], double pad, int R, size_t max_entries) {
    LightGridResult out;
    out.grids.assign(1, DevLightGrid{});
    DevLightGrid& g = out.grids[0];
    g.R = 0;
    const size_t n = spheres.size();
    if (n == 0 || !std::isfinite(pos[0]) || !std::isfinite(pos[1]) || !std::isfinite(pos[2])) return out;
    g.lx = pos[0]; g.ly = pos[1]; g.lz = pos[2];
    std::vector<double> lo(3 * n), hi(3 * n), nearv(n);
    std::vector<char> always(n, 0);
    for (size_t k = 0; k < n; ++k) {
        const double c[3] = {spheres[k].cx, spheres[k].cy, spheres[k].cz};
        const double r = std::fabs(r_leaf[k]) + pad;
        double d2 = 0.0;
        bool finite = std::isfinite(r), at_cam = true;
        for (int i = 0; i < 3; ++i) {
            double a = c[i] - r - pos[i], b = c[i] + r - pos[i];
            a -= 1e-12 * (1.0 + std::fabs(a));
            b += 1e-12 * (1.0 + std::fabs(b));
            lo[3 * k + i] = a; hi[3 * k + i] = b;
            finite &= std::isfinite(a) && std::isfinite(b);
            at_cam &= a - kNearLight <= 0.0 && 0.0 <= b + kNearLight;
            const double gap = std::max({0.0, a, -b});
            d2 += gap * gap;
        }
        always[k] = !finite || at_cam;
        nearv[k] = finite ? std::sqrt(d2) : 0.0;
    }
    struct Rect { int i0, i1, j0, j1; };
    std::vector<Rect> rect(6 * n);
    int fx0[6], fx1[6], fy0[6], fy1[6];
    for (R = std::max(1, R);; R = std::max(1, R / 2)) {
        size_t total = 0;
        for (int f = 0; f < 6; ++f) {
            const int a = f >> 1, b = (a + 1) % 3, cax = (a + 2) % 3;
            const double s = (f & 1) ? -1.0 : 1.0;
            fx0[f] = R; fx1[f] = -1; fy0[f] = R; fy1[f] = -1;
            for (size_t k = 0; k < n; ++k) {
                Rect& q = rect[f * n + k];
                q = Rect{1, 0, 1, 0};
                if (always[k]) continue;
                const double alo = s > 0 ? lo[3 * k + a] : -hi[3 * k + a];
                const double ahi = s > 0 ? hi[3 * k + a] : -lo[3 * k + a];
                if (!(ahi > 0.0)) continue;
                const Range u = face_range(alo, ahi, lo[3 * k + b], hi[3 * k + b]);
                const Range v = face_range(alo, ahi, lo[3 * k + cax], hi[3 * k + cax]);
                if (u.empty() || v.empty() || u.lo > 1.0 + kUMargin || u.hi < -1.0 - kUMargin ||
                    v.lo > 1.0 + kUMargin || v.hi < -1.0 - kUMargin)
                    continue;
                q.i0 = cell_of(u.lo - kUMargin, R); q.i1 = cell_of(u.hi + kUMargin, R);
                q.j0 = cell_of(v.lo - kUMargin, R); q.j1 = cell_of(v.hi + kUMargin, R);
                fx0[f] = std::min(fx0[f], q.i0); fx1[f] = std::max(fx1[f], q.i1);
                fy0[f] = std::min(fy0[f], q.j0); fy1[f] = std::max(fy1[f], q.j1);
                total += static_cast<size_t>(q.i1 - q.i0 + 1) * (q.j1 - q.j0 + 1);
            }
        }
        if (total <= max_entries || R == 1) break;
    }
    g.R = R;
    g.always_begin = 0;
    for (size_t k = 0; k < n; ++k)
        if (always[k]) out.ent.push_back(DevLgEntry{static_cast<int32_t>(k), 0.0f});
    g.always_end = static_cast<uint32_t>(out.ent.size());
    for (int f = 0; f < 6; ++f) {
        g.off_base[f] = static_cast<uint32_t>(out.off.size());
        if (fx1[f] < fx0[f]) { g.fx0[f] = 0; g.fy0[f] = 0; g.fw[f] = 0; g.fh[f] = 0; continue; }
        const int w = fx1[f] - fx0[f] + 1, h = fy1[f] - fy0[f] + 1;
        g.fx0[f] = fx0[f]; g.fy0[f] = fy0[f]; g.fw[f] = w; g.fh[f] = h;
        const size_t cells = static_cast<size_t>(w) * h;
        std::vector<uint32_t> cnt(cells + 1, 0);
        for (size_t k = 0; k < n; ++k) {
            const Rect& q = rect[f * n + k];
            for (int j = q.j0; j <= q.j1; ++j)
                for (int i = q.i0; i <= q.i1; ++i) ++cnt[static_cast<size_t>(j - fy0[f]) * w + (i - fx0[f])];
        }
        const uint32_t base = static_cast<uint32_t>(out.ent.size());
        uint32_t run = base;
        const size_t ob = out.off.size();
        out.off.resize(ob + cells + 1);
        for (size_t c = 0; c < cells; ++c) { out.off[ob + c] = run; run += cnt[c]; cnt[c] = out.off[ob + c]; }
        out.off[ob + cells] = run;
        out.ent.resize(run);
        for (size_t k = 0; k < n; ++k) {        // sphere order within a cell, then sorted by distance
            const Rect& q = rect[f * n + k];
            float nf = static_cast<float>(nearv[k]);
            if (static_cast<double>(nf) > nearv[k]) nf = std::nextafter(nf, 0.0f);
            for (int j = q.j0; j <= q.j1; ++j)
                for (int i = q.i0; i <= q.i1; ++i)
                    out.ent[cnt[static_cast<size_t>(j - fy0[f]) * w + (i - fx0[f])]++] = DevLgEntry{static_cast<int32_t>(k), nf};
        }
        for (size_t c = 0; c < cells; ++c)
            std::sort(out.ent.begin() + out.off[ob + c], out.ent.begin() + out.off[ob + c + 1],
                      [](const DevLgEntry& x, const DevLgEntry& y) { return x.near < y.near || (x.near == y.near && x.sph < y.sph); });
    }
    return out;
}

// The device's candidate list for a shadow query from p toward light `li`
// (occluded_lgrid, trace_common.hpp), with the same f32 arithmetic: the always
// list, then p's cell up to the early stop.  Returns false when the device
// would test every sphere (degenerate direction) or the light has no grid.
bool light_grid_candidates(const LightGridResult& lg, int li, const double p[3], std::vector<int32_t>& out) {
    out.clear();
    if (li < 0 || li >= static_cast<int>(lg.grids.size())) return false;
    const DevLightGrid& g = lg.grids[li];
    if (g.R <= 0) return false;
    for (uint32_t e = g.always_begin; e < g.always_end; ++e) out.push_back(lg.ent[e].sph);
    const float dx = static_cast<float>(p[0] - g.lx), dy = static_cast<float>(p[1] - g.ly),
                dz = static_cast<float>(p[2] - g.lz);
    const float ax = std::fabs(dx), ay = std::fabs(dy), az = std::fabs(dz);
    const int fa = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    const float da = fa == 0 ? dx : fa == 1 ? dy : dz;
    const float db = fa == 0 ? dy : fa == 1 ? dz : dx;
    const float dc = fa == 0 ? dz : fa == 1 ? dx : dy;
    if (!(std::fabs(da) > 0.0f && std::fabs(da) < 3.0e38f)) return false;
    const int f = 2 * fa + (da < 0.0f ? 1 : 0);
    const float inv = 1.0f / std::fabs(da);
    const float R = static_cast<float>(g.R);
    const int ci = std::min(std::max(static_cast<int>(std::floor((db * inv + 1.0f) * 0.5f * R)), 0), g.R - 1);
    const int cj = std::min(std::max(static_cast<int>(std::floor((dc * inv + 1.0f) * 0.5f * R)), 0), g.R - 1);
    const int li2 = ci - g.fx0[f], lj = cj - g.fy0[f];
    if (li2 < 0 || lj < 0 || li2 >= g.fw[f] || lj >= g.fh[f]) return true;
    const uint32_t cell = g.off_base[f] + static_cast<uint32_t>(lj * g.fw[f] + li2);
    const float dist = std::sqrt(dx * dx + dy * dy + dz * dz) * 1.00001f + 1e-5f;
    for (uint32_t e = lg.off[cell]; e < lg.off[cell + 1]; ++e) {
        if (lg.ent[e].near > dist) break;
        out.push_back(lg.ent[e].sph);
    }
    return true;
}

}  // namespace rtamd
