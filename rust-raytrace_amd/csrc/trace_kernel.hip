// Per-pixel ray tracing on CDNA4 (gfx950): one work-item per pixel.
//
// One launch replaces the reference's whole pixel loop (main.rs:45-57): each
// lane maps its pixel to a camera ray (main.rs:50-53, camera.rs:76-80), runs
// the recursive ray_color / PhongMaterial::color chain (raytrace.rs:30-67,
// 261-276) as a fixed-depth loop, and writes its f32 RGB and sRGB-quantised
// BGR bytes (color.rs:593-600,628-632).
//
// Exactness: every operation is the reference's f64 operation in the
// reference's order, compiled with -ffp-contract=off (no FMA fusion; Rust never
// fuses).  f64 add/mul/div/sqrt are IEEE correctly rounded on gfx950, so the
// only possible difference from the CPU is pow() (raytrace.rs:55): OCML vs
// glibc, <= 1 ulp.  The recursion `res + ks * ray_color(child)`
// (raytrace.rs:63) is evaluated inner-first, exactly: each level's local
// colour is pushed on a per-lane stack and folded backwards at the end.
//
// Scene::intersect (scene.rs:247-249) semantics kept exactly: every object is
// tested; the winner is the smallest t with ties going to the FIRST object in
// file order, except that a NaN t (only a plane can produce one, 0/0) sorts
// below every number and wins.  Shadow queries use an any-hit early exit that
// is provably equivalent (see occluded()).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "device_layout.hpp"

namespace rtamd {

__constant__ double c_srgb_avg[255];

namespace {

constexpr double kMinSignificance = 1.0 / 256.0 / 2.0;            // raytrace.rs:17
constexpr double kEps = 0.00001;                                   // raytrace.rs:43,62
constexpr double kFrac1Pi = 0.318309886183790671537767526745028724; // f64::consts::FRAC_1_PI
constexpr int kBlock = 256;                                        // 4 waves = 16x16 pixels

struct Ray {
    double ox, oy, oz, dx, dy, dz;
};

struct Hit {
    double t;
    int32_t obj;        // object id, INT32_MAX = no hit
    int32_t prim;       // sphere index or plane index
    bool sphere;
    bool nan_t;
};

__device__ __forceinline__ double clamp_zero(double x) { return x < 0.0 ? 0.0 : x; }

// color.rs:593-600 as a binary search over the strictly increasing table.
__device__ __forceinline__ uint8_t to_srgb(double v) {
    if (!(v < c_srgb_avg[254])) return 255;      // also NaN
    int lo = 0, hi = 254;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int mid = (lo + hi) >> 1;
        bool lt = v < c_srgb_avg[mid];
        hi = lt ? mid : hi;
        lo = lt ? lo : mid + 1;
    }
    return static_cast<uint8_t>(lo);
}

// shapes.rs:60-89: the exact quadratic; returns the t the reference would
// return, or -1 when it returns None.  `a2` = 2.0*a, `a4` = 4.0*a hoisted per
// ray (the same f64 products the reference forms per test).
__device__ __forceinline__ bool sphere_t(const DevSphere& s, const Ray& r, double a2, double a4, double& t) {
    const double ocx = r.ox - s.cx, ocy = r.oy - s.cy, ocz = r.oz - s.cz;
    const double b = 2.0 * (r.dx * ocx + r.dy * ocy + r.dz * ocz);
    const double cc = (ocx * ocx + ocy * ocy + ocz * ocz) - s.rr;
    const double disc = b * b - a4 * cc;
    if (disc > 0.0) {
        const double sq = sqrt(disc);
        const double t1 = (-b - sq) / a2;
        if (t1 > 0.0) { t = t1; return true; }
        const double t2 = (-b + sq) / a2;
        if (t2 > 0.0) { t = t2; return true; }
    }
    return false;
}

// shapes.rs:100-112: t = n.(p - o) / n.d ; None iff t <= 0 (a NaN t is a hit).
__device__ __forceinline__ bool plane_t(const DevPlane& p, const Ray& r, double& t) {
    const double ex = p.px - r.ox, ey = p.py - r.oy, ez = p.pz - r.oz;
    t = (p.nx * ex + p.ny * ey + p.nz * ez) / (p.nx * r.dx + p.ny * r.dy + p.nz * r.dz);
    return !(t <= 0.0);
}

template <class SpherePtr>
__device__ __forceinline__ Hit nearest(const DevScene& sc, SpherePtr S, const Ray& r) {
    Hit h;
    h.t = __builtin_huge_val();
    h.obj = INT32_MAX;
    h.prim = -1;
    h.sphere = false;
    h.nan_t = false;
    // Planes first (few).  scene.rs:248 min_by_key(FloatNotNan): a NaN t is
    // the minimum key; the first NaN in file order wins outright.
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        const int32_t obj = sc.plane_obj[i];
        if (t != t) {
            if (!h.nan_t || obj < h.obj) { h.nan_t = true; h.t = t; h.obj = obj; h.prim = i; h.sphere = false; }
        } else if (!h.nan_t && (t < h.t || (t == h.t && obj < h.obj))) {
            h.t = t; h.obj = obj; h.prim = i; h.sphere = false;
        }
    }
    if (h.nan_t) return h;      // no sphere can produce a NaN t
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;     // direction.sqnorm()
    const double a2 = 2.0 * a, a4 = 4.0 * a;
    const int n = sc.n_spheres;
#pragma unroll 2
    for (int i = 0; i < n; ++i) {
        const DevSphere s = S[i];
        double t;
        if (sphere_t(s, r, a2, a4, t)) {
            const int32_t obj = sc.sphere_obj[i];
            if (t < h.t || (t == h.t && obj < h.obj)) { h.t = t; h.obj = obj; h.prim = i; h.sphere = true; }
        }
    }
    return h;
}

// The shadow test of raytrace.rs:41-49: `intersect(shadow ray)` is Some and
// (range is None or t*t < range).  Equivalent any-hit form:
//  * no range (directional light): shadowed iff ANY object reports a hit;
//  * with range (point light): if any plane reports a NaN t the nearest-hit
//    is that NaN hit and NaN*NaN < r2 is false -> lit; otherwise shadowed iff
//    SOME hit has t*t < r2 (t_min <= t_i and rounding is monotone, so the
//    nearest one then qualifies too).
template <class SpherePtr>
__device__ __forceinline__ bool occluded(const DevScene& sc, SpherePtr S, const Ray& r, bool has_range, double r2) {
    bool plane_block = false;
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        if (!has_range) return true;
        if (t != t) return false;
        plane_block |= t * t < r2;
    }
    if (plane_block) return true;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const double a2 = 2.0 * a, a4 = 4.0 * a;
    const int n = sc.n_spheres;
    for (int i = 0; i < n; ++i) {
        const DevSphere s = S[i];
        double t;
        if (sphere_t(s, r, a2, a4, t)) {
            if (!has_range || t * t < r2) return true;
        }
    }
    return false;
}

struct Col {
    double r, g, b;
};

// ray_color (raytrace.rs:261-267) from depth 0 with significance 1.0,
// PhongMaterial::color (raytrace.rs:30-67) flattened.  `rays`/`shadows`
// count every Scene::intersect call, exactly as the reference issues them.
template <class SpherePtr>
__device__ Col trace(const DevScene& sc, SpherePtr S, Ray ray, uint32_t max_depth, uint32_t& rays, uint32_t& shadows) {
    double st_r[kMaxLevels], st_g[kMaxLevels], st_b[kMaxLevels];
    int32_t st_obj[kMaxLevels];
    int lvl = 0;
    double sig = 1.0;
    uint32_t depth = 0;
    Col term;
    for (;;) {
        const Hit h = nearest(sc, S, ray);
        ++rays;
        if (h.obj == INT32_MAX) {                                  // background, raytrace.rs:228-232
            term = Col{sc.bg[0], sc.bg[1], sc.bg[2]};
            break;
        }
        const DevMaterial& m = sc.mats[h.obj];
        Col res{m.amb[0], m.amb[1], m.amb[2]};
        if (depth > max_depth) { term = res; break; }             // raytrace.rs:33
        // pt = ray.cast(t) (shapes.rs:22-24)
        const double ptx = ray.ox + ray.dx * h.t, pty = ray.oy + ray.dy * h.t, ptz = ray.oz + ray.dz * h.t;
        double nx, ny, nz;
        if (h.sphere) {             // normalize(ray.cast(t) - center) (shapes.rs:61)
            const DevSphere s = S[h.prim];
            const double ux = ptx - s.cx, uy = pty - s.cy, uz = ptz - s.cz;
            const double l = sqrt(ux * ux + uy * uy + uz * uz);
            nx = ux / l; ny = uy / l; nz = uz / l;
        } else {
            const DevPlane& p = sc.planes[h.prim];
            nx = p.nx; ny = p.ny; nz = p.nz;
        }
        const bool diffuse = m.kd_sig * sig > kMinSignificance;
        const bool specular = m.ks_sig * sig > kMinSignificance;
        if (nx * ray.dx + ny * ray.dy + nz * ray.dz > 0.0) { nx = -nx; ny = -ny; nz = -nz; }
        if (diffuse || specular) {
            for (int li = 0; li < sc.n_lights; ++li) {
                const DevLight& L = sc.lights[li];
                double lx, ly, lz, r2 = 0.0;
                const bool has_range = L.kind == 0;
                if (has_range) {    // PointLight, scene.rs:122-126
                    const double vx = L.v[0] - ptx, vy = L.v[1] - pty, vz = L.v[2] - ptz;
                    r2 = vx * vx + vy * vy + vz * vz;
                    const double l = sqrt(r2);
                    lx = vx / l; ly = vy / l; lz = vz / l;
                } else {            // DirectionalLight, scene.rs:135-138
                    lx = -L.v[0]; ly = -L.v[1]; lz = -L.v[2];
                }
                const Ray sray{ptx + lx * kEps, pty + ly * kEps, ptz + lz * kEps, lx, ly, lz};
                ++rays;
                ++shadows;
                if (occluded(sc, S, sray, has_range, r2)) continue;
                if (diffuse) {
                    const double s = clamp_zero(lx * nx + ly * ny + lz * nz);
                    res.r = res.r + ((m.kd[0] * L.color[0]) * s) * kFrac1Pi;
                    res.g = res.g + ((m.kd[1] * L.color[1]) * s) * kFrac1Pi;
                    res.b = res.b + ((m.kd[2] * L.color[2]) * s) * kFrac1Pi;
                }
                if (specular) {
                    const double hx = lx - ray.dx, hy = ly - ray.dy, hz = lz - ray.dz;
                    const double hl = sqrt(hx * hx + hy * hy + hz * hz);
                    const double c = clamp_zero(nx * (hx / hl) + ny * (hy / hl) + nz * (hz / hl));
                    const double p = pow(c, m.exponent);
                    res.r = res.r + (m.ks[0] * L.color[0]) * p;
                    res.g = res.g + (m.ks[1] * L.color[1]) * p;
                    res.b = res.b + (m.ks[2] * L.color[2]) * p;
                }
            }
        }
        if (!specular) { term = res; break; }
        // raytrace.rs:59-64: reflect and recurse; keep (res, object) for the fold.
        st_r[lvl] = res.r; st_g[lvl] = res.g; st_b[lvl] = res.b; st_obj[lvl] = h.obj;
        ++lvl;
        const double dn = ray.dx * nx + ray.dy * ny + ray.dz * nz;
        const double k2 = 2.0 * dn;
        const double rdx = ray.dx - nx * k2, rdy = ray.dy - ny * k2, rdz = ray.dz - nz * k2;
        ray = Ray{ptx + rdx * kEps, pty + rdy * kEps, ptz + rdz * kEps, rdx, rdy, rdz};
        sig = sig * m.ks_sig;
        ++depth;
    }
    // Fold inner-first: res_k + ks_k * color_{k+1}  (raytrace.rs:63)
    Col acc = term;
    for (int k = lvl - 1; k >= 0; --k) {
        const DevMaterial& m = sc.mats[st_obj[k]];
        acc.r = st_r[k] + m.ks[0] * acc.r;
        acc.g = st_g[k] + m.ks[1] * acc.g;
        acc.b = st_b[k] + m.ks[2] * acc.b;
    }
    return acc;
}

template <bool kLds>
__global__ __launch_bounds__(kBlock) void trace_frame_kernel(DevScene sc, FrameParams fp) {
    extern __shared__ __attribute__((aligned(16))) DevSphere lds_spheres[];
    if constexpr (kLds) {
        for (int i = threadIdx.x; i < sc.n_spheres; i += kBlock) lds_spheres[i] = sc.spheres[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // 16x16 pixel tile per workgroup, 8x8 per wave: neighbouring rays in a
    // wave take the same branches more often.
    const uint32_t lx = blockIdx.x * 16u + (wave & 1) * 8u + (lane & 7);
    const uint32_t ly = blockIdx.y * 16u + (wave >> 1) * 8u + (lane >> 3);
    uint32_t rays = 0, shadows = 0;
    if (lx < fp.tile_w && ly < fp.tile_h) {
        const uint32_t x = fp.x0 + lx;
        const uint32_t y = fp.y0 + ((ly / fp.band) * fp.band_stride + fp.band_phase) * fp.band + ly % fp.band;
        // main.rs:50-53 with the deterministic centre jitter (jx = jy = 0.5)
        const double px = ((static_cast<double>(x) + 0.5) - fp.hw) * fp.scale;
        const double py = ((static_cast<double>(y) + 0.5) - fp.hh) * fp.scale;
        // camera.rs:78: normalize(M * (px, py, 1))
        const double* M = sc.cam_m;
        const double dx = M[0] * px + M[1] * py + M[2] * 1.0;
        const double dy = M[3] * px + M[4] * py + M[5] * 1.0;
        const double dz = M[6] * px + M[7] * py + M[8] * 1.0;
        const double l = sqrt(dx * dx + dy * dy + dz * dz);
        const Ray cam{sc.cam_pos[0], sc.cam_pos[1], sc.cam_pos[2], dx / l, dy / l, dz / l};
        Col res{0.0, 0.0, 0.0};
        for (uint32_t k = 0; k < fp.spp; ++k) {
            Col c;
            if constexpr (kLds) c = trace(sc, static_cast<const DevSphere*>(lds_spheres), cam, fp.max_depth, rays, shadows);
            else c = trace(sc, sc.spheres, cam, fp.max_depth, rays, shadows);
            // raytrace.rs:271-275: (BLACK + c) / samples(=1); main.rs:54: res + that
            c = Col{(0.0 + c.r) / 1.0, (0.0 + c.g) / 1.0, (0.0 + c.b) / 1.0};
            res = Col{res.r + c.r, res.g + c.g, res.b + c.b};
        }
        const double aa = static_cast<double>(fp.spp);
        res = Col{res.r / aa, res.g / aa, res.b / aa};            // main.rs:56
        const size_t p = static_cast<size_t>(ly) * fp.tile_w + lx;
        if (fp.out_rgb) {
            fp.out_rgb[3 * p + 0] = static_cast<float>(res.r);
            fp.out_rgb[3 * p + 1] = static_cast<float>(res.g);
            fp.out_rgb[3 * p + 2] = static_cast<float>(res.b);
        }
        if (fp.out_bgr) {
            uint8_t* q = fp.out_bgr + static_cast<size_t>(ly) * fp.bgr_pitch + 3u * lx;
            q[0] = to_srgb(res.b);
            q[1] = to_srgb(res.g);
            q[2] = to_srgb(res.r);
            if (lx == fp.tile_w - 1)       // BMP row padding is zero (main.rs:42)
                for (uint32_t k = 3u * fp.tile_w; k < fp.bgr_pitch; ++k)
                    fp.out_bgr[static_cast<size_t>(ly) * fp.bgr_pitch + k] = 0;
        }
    }
    // Per-wave sums, one atomic per wave into a sharded counter.
    for (int off = 32; off > 0; off >>= 1) {
        rays += __shfl_xor(rays, off, 64);
        shadows += __shfl_xor(shadows, off, 64);
    }
    if (lane == 0) {
        const uint32_t shard = (blockIdx.y * gridDim.x + blockIdx.x) % kCounterShards;
        atomicAdd(&fp.counters[shard], static_cast<unsigned long long>(rays));
        atomicAdd(&fp.counters[kCounterShards + shard], static_cast<unsigned long long>(shadows));
    }
}

}  // namespace

// Host-side launcher.  mode: 1 = spheres staged in LDS, 2 = read from global.
hipError_t launch_trace_frame(const DevScene& sc, const FrameParams& fp, int mode, hipStream_t stream) {
    dim3 grid((fp.tile_w + 15) / 16, (fp.tile_h + 15) / 16);
    if (mode == 1) {
        size_t lds = static_cast<size_t>(sc.n_spheres) * sizeof(DevSphere);
        hipLaunchKernelGGL(trace_frame_kernel<true>, grid, dim3(kBlock), lds, stream, sc, fp);
    } else {
        hipLaunchKernelGGL(trace_frame_kernel<false>, grid, dim3(kBlock), 0, stream, sc, fp);
    }
    return hipGetLastError();
}

hipError_t upload_srgb_table(const double* avg255) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_srgb_avg), avg255, 255 * sizeof(double));
}

}  // namespace rtamd
