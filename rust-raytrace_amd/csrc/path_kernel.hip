// The general path on CDNA4 (gfx950): every material, light and camera class
// of the reference, including the stochastic and branching ones the
// wavefront chain does not carry:
//   IndirectPhongMaterial  raytrace.rs:69-121   `samples` children per hit
//   TransparentMaterial    raytrace.rs:169-226  reflection + refraction children
//   AreaLight              scene.rs:142-155     keyed light position per hit
//   DepthOfFieldCamera     camera.rs:83-123     `samples` lens samples per AA sample
//   random AA jitter       main.rs:51-52        keyed (x, y) offset per AA sample
// plus Phong / Fresnel / point / directional exactly as the wavefront path.
//
// One work-item per pixel runs main.rs:45-56 (AA samples, camera samples)
// and the whole ray_color recursion as a loop over an explicit stack: a hit
// that spawns a child stores its frame (hit point, flipped normal, incoming
// direction, significance, partial colour, material factors, path key) at
// its depth and descends; a returning colour is folded into the parent's
// partial colour in the reference's operation order (`res = res + term`,
// child by child), and the parent spawns its next child or returns.  The
// stack lives in HBM, SoA per depth, so the lanes of a wave at the same depth
// read and write consecutive words.  Queries go through the sphere BVH (exact
// f64 leaf tests, trace_common.hpp), staged in LDS when it fits.
//
// Every random draw is keyed on its place in the recursion (trace_common.hpp
// "keyed RNG"), so the image does not depend on the schedule and the oracle's
// REF_RNG_KEYED mode reproduces it draw for draw.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_layout.hpp"
#include "launch_api.hpp"
// the compiler's divisions in the normalisations here (the hoisted-reciprocal form measured
// C1 8.702 vs 8.627 ms on this kernel, while it helped the wavefront kernels)
#ifndef RT_DIVK
#define RT_DIVK 0
#endif
#include "trace_common.hpp"

namespace rtamd {

namespace {

constexpr int kPathBlock = 256;
#ifndef RT_PATH_WAVES
#define RT_PATH_WAVES 2       // min waves per SIMD: 256 VGPRs, no spills (C1 11.4 -> 8.4 ms against 4 waves)
#endif
constexpr double kPi = 3.14159265358979323846264338327950288;      // f64::consts::PI
constexpr int32_t kFlDiffuse = 1, kFlSpecular = 2, kFlRefract = 4;
constexpr int32_t kFlMore = 8;          // the frame has children left after the one in flight (extension stored)

__device__ __forceinline__ double clamp_one(double x) { return x > 1.0 ? 1.0 : x; }   // raytrace.rs:26-28

// One level of the recursion: what PhongMaterial / IndirectPhongMaterial /
// FresnelMaterial / TransparentMaterial::color holds across its child calls.
struct Frame {
    Col res;                    // colour so far
    double g, g2;               // fold factors of the child in flight (see fold_child)
    double ptx, pty, ptz;       // pt = ray.cast(t)
    double nx, ny, nz;          // normal flipped toward the viewer
    double dx, dy, dz;          // incoming ray direction
    double sig;                 // significance the hit was reached with
    double f;                   // Fresnel / Transparent: Schlick factor; Phong / IndirectPhong: 1
    double ax, ay, az;          // Transparent: unnormalised refraction vector; IndirectPhong: sample direction
    uint64_t key;               // path key of the hit
    int32_t obj, next, flags;   // object id, index of the child in flight, kFl* bits
};

// Compact part: colour, fold factors, object, child, flags.
__device__ __forceinline__ void store_compact(const PathStack& st, int L, uint32_t t, const Frame& F) {
    st.f(L, 0)[t] = F.res.r; st.f(L, 1)[t] = F.res.g; st.f(L, 2)[t] = F.res.b;
    st.f(L, 3)[t] = F.g; st.f(L, 4)[t] = F.g2;
    st.i(L, 0)[t] = F.obj;
    st.i(L, 1)[t] = F.next;
    st.i(L, 2)[t] = F.flags;
}

__device__ __forceinline__ void store_extension(const PathStack& st, int L, uint32_t t, const Frame& F) {
    const double v[kPathF - kPathCompact] = {F.ptx, F.pty, F.ptz, F.nx, F.ny, F.nz, F.dx, F.dy, F.dz,
                                             F.sig, F.f, F.ax, F.ay, F.az};
#pragma unroll
    for (int k = 0; k < kPathF - kPathCompact; ++k) st.f(L, kPathCompact + k)[t] = v[k];
    st.key(L)[t] = F.key;
}

__device__ __forceinline__ void load_compact(const PathStack& st, int L, uint32_t t, Frame& F) {
    F.res = Col{st.f(L, 0)[t], st.f(L, 1)[t], st.f(L, 2)[t]};
    F.g = st.f(L, 3)[t]; F.g2 = st.f(L, 4)[t];
    F.obj = st.i(L, 0)[t];
    F.next = st.i(L, 1)[t];
    F.flags = st.i(L, 2)[t];
}

__device__ __forceinline__ void load_extension(const PathStack& st, int L, uint32_t t, Frame& F) {
    double v[kPathF - kPathCompact];
#pragma unroll
    for (int k = 0; k < kPathF - kPathCompact; ++k) v[k] = st.f(L, kPathCompact + k)[t];
    F.ptx = v[0]; F.pty = v[1]; F.ptz = v[2];
    F.nx = v[3]; F.ny = v[4]; F.nz = v[5];
    F.dx = v[6]; F.dy = v[7]; F.dz = v[8];
    F.sig = v[9];
    F.f = v[10];
    F.ax = v[11]; F.ay = v[12]; F.az = v[13];
    F.key = st.key(L)[t];
}

// Texture::sample (texture.rs:46-58) of skybox face k: bilinear over
// Color::from_srgb texels (color.rs:611-613), coordinates clamped to [0, 1].
__device__ __forceinline__ double clamp01(double x) { return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x); }   // texture.rs:28-31

__device__ __forceinline__ Col texel(const DevScene& sc, const DevTexFace& f, uint32_t x, uint32_t y) {
    const uint8_t* p = sc.tex + f.off + 3ull * (x + static_cast<uint64_t>(y) * f.w);
    return Col{sc.srgb_values[p[0]], sc.srgb_values[p[1]], sc.srgb_values[p[2]]};
}

__device__ __forceinline__ Col tex_sample(const DevScene& sc, int k, double u, double v) {
    const DevTexFace f = sc.faces[k];
    const double x = clamp01(u) * static_cast<double>(f.w - 1);
    const double y = clamp01(v) * static_cast<double>(f.h - 1);
    const uint32_t x0 = x >= 0.0 ? static_cast<uint32_t>(x) : 0u;   // `as u32`: NaN -> 0
    const uint32_t y0 = y >= 0.0 ? static_cast<uint32_t>(y) : 0u;
    const uint32_t x1 = x0 >= f.w - 1 ? f.w - 1 : x0 + 1;
    const uint32_t y1 = y0 >= f.h - 1 ? f.h - 1 : y0 + 1;
    const double xx = x - static_cast<double>(x0), yy = y - static_cast<double>(y0);
    const Col a = texel(sc, f, x0, y0), b = texel(sc, f, x0, y1), c = texel(sc, f, x1, y0), d = texel(sc, f, x1, y1);
    const Col cx0{a.r * (1.0 - yy) + b.r * yy, a.g * (1.0 - yy) + b.g * yy, a.b * (1.0 - yy) + b.b * yy};
    const Col cx1{c.r * (1.0 - yy) + d.r * yy, c.g * (1.0 - yy) + d.g * yy, c.b * (1.0 - yy) + d.b * yy};
    return Col{cx0.r * (1.0 - xx) + cx1.r * xx, cx0.g * (1.0 - xx) + cx1.g * xx, cx0.b * (1.0 - xx) + cx1.b * xx};
}

// Background::color (raytrace.rs:228-256): the solid colour, or the skybox
// face the direction's dominant axis points at (x, then y, then z; no strict
// winner: BLACK).
__device__ __forceinline__ Col background(const DevScene& sc, const Ray& r) {
    if (!sc.skybox) return Col{sc.bg[0], sc.bg[1], sc.bg[2]};
    const double dx = r.dx, dy = r.dy, dz = r.dz;
    const double ax = fabs(dx), ay = fabs(dy), az = fabs(dz);
    if (ax > az && ax > ay) {
        const double px = -dz / dx, py = -dy / ax;
        return tex_sample(sc, dx > 0.0 ? 0 : 1, px * 0.5 + 0.5, py * 0.5 + 0.5);
    }
    if (ay > ax && ay > az) {
        const double px = dx / ay, py = dz / dy;
        return tex_sample(sc, dy > 0.0 ? 2 : 3, px * 0.5 + 0.5, py * 0.5 + 0.5);
    }
    if (az > ax && az > ay) {
        const double px = dx / dz, py = -dy / az;
        return tex_sample(sc, dz > 0.0 ? 4 : 5, px * 0.5 + 0.5, py * 0.5 + 0.5);
    }
    return Col{0.0, 0.0, 0.0};
}

// camera.rs:76-80 (simple) and camera.rs:109-122 (depth of field; theta and
// r2 keyed on the camera sample).
__device__ __forceinline__ Ray camera_project(const DevScene& sc, double px, double py, uint64_t kc) {
    const double* M = sc.cam_m;
    const double dx = M[0] * px + M[1] * py + M[2] * 1.0;
    const double dy = M[3] * px + M[4] * py + M[5] * 1.0;
    const double dz = M[6] * px + M[7] * py + M[8] * 1.0;
    if (!sc.cam_dof) {
        const double l = sqrt(dx * dx + dy * dy + dz * dz);
        return Ray{sc.cam_pos[0], sc.cam_pos[1], sc.cam_pos[2], dx / l, dy / l, dz / l};
    }
    const double ipx = sc.cam_pos[0] + dx, ipy = sc.cam_pos[1] + dy, ipz = sc.cam_pos[2] + dz;     // image plane
    const double s = sc.cam_focus / sc.cam_im_dist;
    const double fpx = sc.cam_pos[0] + dx * s, fpy = sc.cam_pos[1] + dy * s, fpz = sc.cam_pos[2] + dz * s;   // focal point
    const double theta = key_f64(kc, 0) * (2.0 * kPi);
    const double r2 = key_closed01(kc, 1);
    const double rad = sqrt(r2) * sc.cam_aperture;
    const double vx = cos(theta) * rad, vy = sin(theta) * rad, vz = 0.0;
    const double ox = ipx + ((M[0] * vx + M[1] * vy) + M[2] * vz);
    const double oy = ipy + ((M[3] * vx + M[4] * vy) + M[5] * vz);
    const double oz = ipz + ((M[6] * vx + M[7] * vy) + M[8] * vz);
    const double ex = fpx - ox, ey = fpy - oy, ez = fpz - oz;
    const double l = sqrt(ex * ex + ey * ey + ez * ez);
    return Ray{ox, oy, oz, ex / l, ey / l, ez / l};
}

// The part of Material::color before any child call: flags, the Schlick
// factor, Transparent's refraction vector, and the direct lighting with its
// shadow queries (raytrace.rs:31-56, 69-97, 125-157, 171-211).
template <int kNodes>
__device__ void shade_hit(const DevScene& sc, const BvhView& v, const DevMaterial& m, const Ray& r, const Hit& h,
                          double sig, uint64_t key, Frame& F, uint64_t& rays, uint64_t& shadows) {
    F.ptx = r.ox + r.dx * h.t; F.pty = r.oy + r.dy * h.t; F.ptz = r.oz + r.dz * h.t;   // ray.cast(t)
    double rnx, rny, rnz;
    hit_normal(sc, v.sph, h.prim, F.ptx, F.pty, F.ptz, rnx, rny, rnz);
    const double nd = rnx * r.dx + rny * r.dy + rnz * r.dz;
    const bool flip = nd > 0.0;
    F.nx = flip ? -rnx : rnx; F.ny = flip ? -rny : rny; F.nz = flip ? -rnz : rnz;
    F.dx = r.dx; F.dy = r.dy; F.dz = r.dz;
    F.sig = sig;
    F.key = key;
    F.obj = h.obj;
    F.next = -1;
    F.ax = F.ay = F.az = 0.0;
    F.g = F.g2 = 0.0;
    bool diffuse, specular;
    if (m.kind == kMatTransparent) {                                   // raytrace.rs:171-195
        F.res = Col{0.0, 0.0, 0.0};
        const double n = flip ? m.ior : 1.0 / m.ior;
        const double sin2 = (n * n) * (1.0 - nd * nd);
        const bool refr = sin2 < 1.0;
        if (refr) {
            const double cs = sqrt(1.0 - sin2);
            const double k = n * fabs(nd) + cs;
            F.ax = r.dx * n - F.nx * k; F.ay = r.dy * n - F.ny * k; F.az = r.dz * n - F.nz * k;
        }
        double r0 = (m.ior - 1.0) / (m.ior + 1.0);
        r0 = r0 * r0;
        const double omcos = flip ? (refr ? 1.0 - (F.nx * F.ax + F.ny * F.ay + F.nz * F.az) : 0.0) : 1.0 - fabs(nd);
        const double omcos2 = omcos * omcos;
        F.f = refr ? clamp_one(r0 + (((1.0 - r0) * omcos2) * omcos2) * omcos) : 1.0;
        diffuse = false;
        specular = (m.ks_sig * F.f) * sig > kMinSignificance;
        F.flags = (specular ? kFlSpecular : 0) | (refr ? kFlRefract : 0);
    } else {
        F.res = Col{m.amb[0], m.amb[1], m.amb[2]};
        const Shading s = shading_flags<true>(m, sig, nd);             // f = 1 unless Fresnel
        F.f = s.f;
        diffuse = s.diffuse;
        specular = s.specular;
        F.flags = (diffuse ? kFlDiffuse : 0) | (specular ? kFlSpecular : 0);
    }
    if (!(diffuse || specular)) return;
    const int32_t hint = h.prim >= 0 ? h.prim : -1;                    // the sphere the point lies on
    for (int l = 0; l < sc.n_lights; ++l) {
        const DevLight& Lt = sc.lights[l];
        double lx, ly, lz, r2;
        const bool has_range = light_dir_keyed(Lt, l, key, F.ptx, F.pty, F.ptz, lx, ly, lz, r2);
        const Ray sray{F.ptx + lx * kEps, F.pty + ly * kEps, F.ptz + lz * kEps, lx, ly, lz};
        ++rays;
        ++shadows;
        if (occluded_bvh<false, kNodes, 0>(sc, v, sray, has_range, r2, hint)) continue;
        add_light(F.res, m, Lt, diffuse, specular, F.f, lx, ly, lz, F.nx, F.ny, F.nz, F.dx, F.dy, F.dz);
    }
}

// The first child ray of frame F with index >= i, or -1: its ray and
// significance (raytrace.rs:58-64, 98-106, 159-164, 212-224), the fold factors
// F.g / F.g2 its colour will be folded with, and kFlMore when F has children
// left after it.
__device__ __forceinline__ int next_child(Frame& F, const DevMaterial& m, int i, Ray& cr, double& csig) {
    const bool specular = (F.flags & kFlSpecular) != 0;
    F.flags &= ~kFlMore;
    if (m.kind == kMatIndirect) {
        if (i >= static_cast<int>(m.samples) || !(F.flags & (kFlDiffuse | kFlSpecular))) return -1;
        const double r1 = key_f64(F.key, 128u + 2u * static_cast<uint32_t>(i)) * 2.0 - 1.0;
        const double r2 = key_f64(F.key, 129u + 2u * static_cast<uint32_t>(i)) * (2.0 * kPi);
        const double sin_theta = 1.0 - r1 * r1;                        // sic: no sqrt (raytrace.rs:103)
        const double x = sin_theta * cos(r2), z = sin_theta * sin(r2);
        const bool keep = (x * F.nx + r1 * F.ny + z * F.nz) >= 0.0;
        F.ax = keep ? x : -x; F.ay = keep ? r1 : -r1; F.az = keep ? z : -z;
        cr = Ray{F.ptx + F.ax * kEps, F.pty + F.ay * kEps, F.ptz + F.az * kEps, F.ax, F.ay, F.az};
        csig = F.sig;                                                 // significance passed unchanged
        F.g = F.nx * F.ax + F.ny * F.ay + F.nz * F.az;                // dot(normal, dir)
        if (specular) {   // sic: (dir - ray.direction) with ray the NEW ray: 0/0 (raytrace.rs:108,115)
            const double hx = F.ax - F.ax, hy = F.ay - F.ay, hz = F.az - F.az;
            const double hl = sqrt(hx * hx + hy * hy + hz * hz);
            F.g2 = pow(clamp_zero(F.nx * (hx / hl) + F.ny * (hy / hl) + F.nz * (hz / hl)), m.exponent);
        }
        if (i + 1 < static_cast<int>(m.samples)) F.flags |= kFlMore;
        return i;
    }
    const bool refract = m.kind == kMatTransparent && F.f < 1.0 && (F.flags & kFlRefract);   // raytrace.rs:216-224
    if (i == 0 && specular) {                                          // mirror reflection
        cr = reflect_ray(Ray{0.0, 0.0, 0.0, F.dx, F.dy, F.dz}, F.ptx, F.pty, F.ptz, F.nx, F.ny, F.nz);
        csig = (F.f * F.sig) * m.ks_sig;                               // Phong: (1 * sig) * ks_sig == sig * ks_sig
        F.g = F.f;
        if (refract) F.flags |= kFlMore;
        return 0;
    }
    if (i <= 1 && refract) {
        const double omf = clamp_one(1.0 - F.f);
        const double l = sqrt(F.ax * F.ax + F.ay * F.ay + F.az * F.az);
        const double rx = F.ax / l, ry = F.ay / l, rz = F.az / l;
        cr = Ray{F.ptx + rx * kEps, F.pty + ry * kEps, F.ptz + rz * kEps, rx, ry, rz};
        csig = omf * F.sig;
        F.g = omf;
        return 1;
    }
    return -1;
}

// Fold the colour c of child F.next into F.res (the `res = res + ...` lines)
// with the factors next_child recorded.
__device__ __forceinline__ void fold_child(Frame& F, const DevMaterial& m, const Col& c) {
    if (m.kind == kMatIndirect) {                                      // raytrace.rs:107-118
        const double fac = static_cast<double>(m.samples) * 0.5;
        if (F.flags & kFlDiffuse) {                                    // ((kd * c) * dot(n, dir)) / fac
            F.res.r = F.res.r + ((m.kd[0] * c.r) * F.g) / fac;
            F.res.g = F.res.g + ((m.kd[1] * c.g) * F.g) / fac;
            F.res.b = F.res.b + ((m.kd[2] * c.b) * F.g) / fac;
        }
        if (F.flags & kFlSpecular) {                                   // ((ks * c) * pow) / fac
            F.res.r = F.res.r + ((m.ks[0] * c.r) * F.g2) / fac;
            F.res.g = F.res.g + ((m.ks[1] * c.g) * F.g2) / fac;
            F.res.b = F.res.b + ((m.ks[2] * c.b) * F.g2) / fac;
        }
        return;
    }
    if (F.next == 0) {                      // reflection: res + (ks * child) * f  (raytrace.rs:63 / 163 / 214)
        F.res.r = F.res.r + (m.ks[0] * c.r) * F.g;
        F.res.g = F.res.g + (m.ks[1] * c.g) * F.g;
        F.res.b = F.res.b + (m.ks[2] * c.b) * F.g;
    } else {                                // refraction: res + child * omf  (raytrace.rs:222)
        F.res.r = F.res.r + c.r * F.g;
        F.res.g = F.res.g + c.g * F.g;
        F.res.b = F.res.b + c.b * F.g;
    }
}

// ray_color(camera ray, 1.0, 0, key) -- raytrace.rs:261-267 -- with the
// recursion unrolled over the HBM stack (levels 0 .. max_depth hold frames).
template <int kNodes>
__device__ Col trace_path(const DevScene& sc, const BvhView& v, const FrameParams& fp, const PathStack& st, uint32_t t,
                          Ray ray, uint64_t key, uint64_t& rays, uint64_t& shadows) {
    double sig = 1.0;
    int L = 0;
    for (;;) {
        Col c;
        const Hit h = nearest_bvh<false, kNodes, 0>(sc, v, ray);
        ++rays;
        Frame F;
        Ray cr;
        double csig = 0.0;
        int child = -1;
        if (h.obj == INT32_MAX) {
            c = background(sc, ray);                                    // raytrace.rs:228-256
        } else {
            const DevMaterial& m = sc.mats[h.obj];
            if (static_cast<uint32_t>(L) > fp.max_depth) {             // raytrace.rs:33 / 72 / 126 / 172
                c = m.kind == kMatTransparent ? Col{0.0, 0.0, 0.0} : Col{m.amb[0], m.amb[1], m.amb[2]};
            } else {
                shade_hit<kNodes>(sc, v, m, ray, h, sig, key, F, rays, shadows);
                child = next_child(F, m, 0, cr, csig);
                c = F.res;
            }
        }
        if (child >= 0) {                                              // descend
            F.next = child;
            store_compact(st, L, t, F);
            if (F.flags & kFlMore) store_extension(st, L, t, F);
            ray = cr;
            sig = csig;
            key = key_child(F.key, static_cast<uint64_t>(child));
            ++L;
            continue;
        }
        bool resumed = false;                                          // return c to the parents
        while (L > 0) {
            --L;
            Frame P;
            load_compact(st, L, t, P);
            const DevMaterial& m = sc.mats[P.obj];
            fold_child(P, m, c);
            if (P.flags & kFlMore) {                                   // spawn the next child
                load_extension(st, L, t, P);
                const int nx = next_child(P, m, P.next + 1, cr, csig);
                P.next = nx;
                store_compact(st, L, t, P);                            // the extension is unchanged
                ray = cr;
                sig = csig;
                key = key_child(P.key, static_cast<uint64_t>(nx));
                ++L;
                resumed = true;
                break;
            }
            c = P.res;
        }
        if (!resumed) return c;
    }
}

// kNodes: 2 = binary BVH, spheres and object ids staged in LDS; 0 = read through the caches.
template <int kNodes>
__global__ __launch_bounds__(kPathBlock, RT_PATH_WAVES) void path_kernel(DevScene sc, FrameParams fp, PathStack st) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double* s_srgb = reinterpret_cast<double*>(lds);
    for (int i = threadIdx.x; i < 255; i += kPathBlock) s_srgb[i] = fp.srgb[i];
    BvhView v = global_view(sc);
    if constexpr (kNodes == 2) {
        v.lnodes = stage_node_planes<kPathBlock>(sc.bvh, sc.n_bvh, lds + 2048);
        DevSphere* ls = reinterpret_cast<DevSphere*>(lds + 2048 + node_planes_bytes(sc.n_bvh));
        int32_t* lo = reinterpret_cast<int32_t*>(ls + sc.n_spheres);
        for (int i = threadIdx.x; i < sc.n_spheres; i += kPathBlock) { ls[i] = sc.spheres[i]; lo[i] = sc.sphere_obj[i]; }
        v.nl = sc.n_bvh;
        v.sph = ls;
        v.obj = lo;
    }
    __syncthreads();
    const uint32_t t = blockIdx.x * kPathBlock + threadIdx.x;
    const uint64_t npix = static_cast<uint64_t>(fp.tile_w) * fp.rows;
    uint64_t rays = 0, shadows = 0;
    const double ns = static_cast<double>(sc.cam_samples), aa = static_cast<double>(fp.spp);
    // G = fp.path_group lanes of one wave share a pixel: lane j of the group traces
    // AA samples j, j + G, ..., and the group adds the sample colours in sample
    // order through cross-lane reads, so the sum is main.rs:47-55's
    // `res = res + raytrace(..)` sequence exactly.  G > 1 when the frame has too
    // few pixels to fill the chip one pixel per lane (C1: 64 k pixels x 1024 samples).
    const uint32_t G = fp.path_group;
    const uint32_t lane = threadIdx.x & 63u, gl = lane & (G - 1u), gbase = lane - gl;
    for (uint64_t p = t / G; p < npix; p += st.T / G) {               // main.rs:45-56
        const uint32_t lx = static_cast<uint32_t>(p % fp.tile_w);
        const uint32_t lr = fp.row0 + static_cast<uint32_t>(p / fp.tile_w);
        const uint32_t x = fp.x0 + lx;
        const uint32_t y = fp.y0 + ((lr / fp.band) * fp.band_stride + fp.band_phase) * fp.band + lr % fp.band;
        const uint64_t kp = key_pixel(fp.seed, x, y);
        Col res{0.0, 0.0, 0.0};
        for (uint32_t a0 = 0; a0 < fp.spp; a0 += G) {
            const uint32_t a = a0 + gl;
            Col r{0.0, 0.0, 0.0};                                      // raytrace.rs:270-276
            if (a < fp.spp) {
                const uint64_t ka = key_child(kp, a);
                const double jx = fp.jitter ? key_f64(ka, 0) : 0.5;   // x drawn before y (main.rs:51-52)
                const double jy = fp.jitter ? key_f64(ka, 1) : 0.5;
                const double px = ((static_cast<double>(x) + jx) - fp.hw) * fp.scale;
                const double py = ((static_cast<double>(y) + jy) - fp.hh) * fp.scale;
                for (uint32_t cs = 0; cs < sc.cam_samples; ++cs) {
                    const uint64_t kc = key_child(ka, cs);
                    const Col c = trace_path<kNodes>(sc, v, fp, st, t, camera_project(sc, px, py, kc), kc, rays, shadows);
                    r = Col{r.r + c.r, r.g + c.g, r.b + c.b};
                }
                r = Col{r.r / ns, r.g / ns, r.b / ns};
            }
            if (G == 1) {
                res = Col{res.r + r.r, res.g + r.g, res.b + r.b};
            } else {
                const uint32_t m = min(G, fp.spp - a0);
                for (uint32_t j = 0; j < m; ++j) {                     // sample order
                    const int src = static_cast<int>(gbase + j);
                    res = Col{res.r + __shfl(r.r, src, 64), res.g + __shfl(r.g, src, 64), res.b + __shfl(r.b, src, 64)};
                }
            }
        }
        res = Col{res.r / aa, res.g / aa, res.b / aa};
        if (gl == 0) write_pixel(fp, lx, lr, res, s_srgb);
    }
    for (int off = 32; off > 0; off >>= 1) {
        rays += __shfl_xor(rays, off, 64);
        shadows += __shfl_xor(shadows, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        const uint32_t shard = (t >> 6) % kCounterShards;
        atomicAdd(&fp.counters[shard], static_cast<unsigned long long>(rays));
        atomicAdd(&fp.counters[kCounterShards + shard], static_cast<unsigned long long>(shadows));
    }
}

}  // namespace

int path_waves_per_simd() { return RT_PATH_WAVES; }

size_t path_lds_bytes(const DevScene& sc, bool staged) {
    size_t b = 2048;
    if (staged) b += node_planes_bytes(sc.n_bvh) + static_cast<size_t>(sc.n_spheres) * (sizeof(DevSphere) + 4);
    return b;
}

hipError_t launch_path(const DevScene& sc, const FrameParams& fp, const PathStack& st, bool staged, hipStream_t stream) {
    const uint64_t npix = static_cast<uint64_t>(fp.tile_w) * fp.rows;
    const uint64_t want = (npix * fp.path_group + kPathBlock - 1) / kPathBlock;   // path_group lanes per pixel
    const dim3 grid(static_cast<uint32_t>(want < st.T / kPathBlock ? want : st.T / kPathBlock));
    if (grid.x == 0) return hipSuccess;
    if (staged) hipLaunchKernelGGL(path_kernel<2>, grid, dim3(kPathBlock), path_lds_bytes(sc, true), stream, sc, fp, st);
    else hipLaunchKernelGGL(path_kernel<0>, grid, dim3(kPathBlock), path_lds_bytes(sc, false), stream, sc, fp, st);
    return hipGetLastError();
}

// rt_ctx_reserve: the first launch of any kernel of this file loads its code object.
__global__ void path_warm(uint32_t* sink) {
    if (sink && threadIdx.x == 0) sink[blockIdx.x] = 0u;
}

hipError_t launch_path_warmup(hipStream_t s) {
    hipLaunchKernelGGL(path_warm, dim3(1), dim3(64), 0, s, nullptr);
    return hipGetLastError();
}

}  // namespace rtamd
