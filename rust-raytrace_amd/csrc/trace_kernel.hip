// Per-pixel ray tracing on CDNA4 (gfx950).
//
// Two schedules of the same exact math (trace_common.hpp):
//
//  * trace_frame_kernel ("megakernel"): one work-item per pixel runs the whole
//    recursive ray_color / PhongMaterial::color chain (raytrace.rs:30-67,
//    261-276) as a loop.  Simple, but a wave lives as long as its deepest
//    pixel and holds all shading state across every intersection loop.
//
//  * wavefront (wf_*): one generation per recursion depth k.  Queue Q_k in HBM
//    holds exactly the rays ray_color is called with at depth k; per
//    generation:
//        wf_nearest    Scene::intersect for every ray of Q_k (scene.rs:247-249)
//                      and compaction of the hits that need light evaluation
//        wf_occlusion  the shadow queries of those hits (raytrace.rs:41-49)
//        wf_shade      the Phong sum (raytrace.rs:31-56), push of the level's
//                      local colour, compaction of the reflection rays into
//                      Q_{k+1} (raytrace.rs:58-64)
//    then wf_fold evaluates `res + ks * ray_color(child)` inner-first from the
//    per-pixel level stack (bit-exact, raytrace.rs:63) and writes f32 RGB +
//    sRGB BGR.  Every lane of every launch holds a live ray: no divergence over
//    path length, small kernels, high occupancy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "device_layout.hpp"
#include "trace_common.hpp"

namespace rtamd {

__constant__ double c_srgb_avg[255];

namespace {

constexpr int kBlock = 256;                 // 4 waves

// ---------------------------------------------------------------- megakernel

template <class SpherePtr>
__device__ Col trace_chain(const DevScene& sc, SpherePtr S, Ray ray, uint32_t max_depth, uint32_t& rays,
                           uint32_t& shadows) {
    double st_r[kMaxLevels], st_g[kMaxLevels], st_b[kMaxLevels];
    int32_t st_obj[kMaxLevels];
    int lvl = 0;
    double sig = 1.0;
    uint32_t depth = 0;
    Col term;
    for (;;) {
        const Hit h = nearest_brute(sc, S, ray);
        ++rays;
        if (h.obj == INT32_MAX) { term = Col{sc.bg[0], sc.bg[1], sc.bg[2]}; break; }   // raytrace.rs:228-232
        const DevMaterial& m = sc.mats[h.obj];
        Col res{m.amb[0], m.amb[1], m.amb[2]};
        if (depth > max_depth) { term = res; break; }             // raytrace.rs:33
        const double ptx = ray.ox + ray.dx * h.t, pty = ray.oy + ray.dy * h.t, ptz = ray.oz + ray.dz * h.t;
        double nx, ny, nz;
        hit_normal(sc, sc.spheres, h.prim, ptx, pty, ptz, nx, ny, nz);
        const bool diffuse = m.kd_sig * sig > kMinSignificance;
        const bool specular = m.ks_sig * sig > kMinSignificance;
        if (nx * ray.dx + ny * ray.dy + nz * ray.dz > 0.0) { nx = -nx; ny = -ny; nz = -nz; }
        if (diffuse || specular) {
            for (int li = 0; li < sc.n_lights; ++li) {
                const DevLight& L = sc.lights[li];
                double lx, ly, lz, r2;
                const bool has_range = light_dir(L, ptx, pty, ptz, lx, ly, lz, r2);
                const Ray sray{ptx + lx * kEps, pty + ly * kEps, ptz + lz * kEps, lx, ly, lz};
                ++rays;
                ++shadows;
                if (occluded_brute(sc, S, sray, has_range, r2)) continue;
                add_light(res, m, L, diffuse, specular, lx, ly, lz, nx, ny, nz, ray.dx, ray.dy, ray.dz);
            }
        }
        if (!specular) { term = res; break; }
        st_r[lvl] = res.r; st_g[lvl] = res.g; st_b[lvl] = res.b; st_obj[lvl] = h.obj;
        ++lvl;
        ray = reflect_ray(ray, ptx, pty, ptz, nx, ny, nz);
        sig = sig * m.ks_sig;
        ++depth;
    }
    Col acc = term;                                                // fold inner-first (raytrace.rs:63)
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
    // 16x16 pixel tile per workgroup, 8x8 per wave
    const uint32_t lx = blockIdx.x * 16u + (wave & 1) * 8u + (lane & 7);
    const uint32_t ly = blockIdx.y * 16u + (wave >> 1) * 8u + (lane >> 3);
    uint32_t rays = 0, shadows = 0;
    if (lx < fp.tile_w && ly < fp.rows) {
        const Ray cam = camera_ray(sc, fp, lx, fp.row0 + ly);
        Col c;
        if constexpr (kLds) c = trace_chain(sc, static_cast<const DevSphere*>(lds_spheres), cam, fp.max_depth, rays, shadows);
        else c = trace_chain(sc, sc.spheres, cam, fp.max_depth, rays, shadows);
        write_pixel(fp, lx, fp.row0 + ly, average_samples(c, fp.spp));
        rays *= fp.spp;          // identical centre-jitter samples: traced once, counted as the reference issues them
        shadows *= fp.spp;
    }
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

// ---------------------------------------------------------------- wavefront

// Wave-aggregated append: one atomic per wave, lanes get consecutive slots in
// lane order (keeps neighbouring rays neighbours).  All 64 lanes must call it.
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool want) {
    const unsigned long long mask = __ballot(want);
    if (mask == 0) return 0xFFFFFFFFu;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll(static_cast<long long>(mask)) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, static_cast<uint32_t>(__popcll(mask)));
    base = __shfl(base, leader, 64);
    const uint32_t below = static_cast<uint32_t>(__popcll(mask & ((1ull << lane) - 1ull)));
    return want ? base + below : 0xFFFFFFFFu;
}

// Generation-0 slot i -> pixel of the chunk, in 8x8 tiles (one tile per wave).
__device__ __forceinline__ bool slot_pixel(const WfBufs& b, const FrameParams& fp, uint32_t i, uint32_t& lx,
                                           uint32_t& ly) {
    const uint32_t tile = i >> 6, w = i & 63u;
    lx = (tile % b.tiles_x) * 8u + (w & 7u);
    ly = (tile / b.tiles_x) * 8u + (w >> 3);
    return lx < fp.tile_w && ly < fp.rows;
}

__device__ __forceinline__ Ray load_ray(const WfBufs& b, int q, uint32_t i) {
    return Ray{b.qo[q][0][i], b.qo[q][1][i], b.qo[q][2][i], b.qd[q][0][i], b.qd[q][1][i], b.qd[q][2][i]};
}

// Ray of queue entry i of generation k (generation 0 is computed, not stored).
template <bool kCam>
__device__ __forceinline__ bool entry_ray(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int k, uint32_t i,
                                          Ray& r, double& sig, uint32_t& p) {
    if constexpr (kCam) {
        uint32_t lx, ly;
        if (!slot_pixel(b, fp, i, lx, ly)) return false;
        r = camera_ray(sc, fp, lx, fp.row0 + ly);
        sig = 1.0;                                    // raytrace.rs:273 via main.rs:54
        p = ly * fp.tile_w + lx;
    } else {
        const int q = k & 1;
        r = load_ray(b, q, i);
        sig = b.qsig[q][i];
        p = b.qpix[q][i];
    }
    return true;
}

// Sphere sources of the wavefront intersection kernels.
constexpr int kSrcGlobal = 0;       // brute force, sphere list through the caches
constexpr int kSrcLds = 1;          // brute force, sphere list staged in LDS per workgroup
constexpr int kSrcBvhG = 2;         // BVH from HBM/L2, scratch stack
constexpr int kSrcBvhGS = 3;        // BVH from HBM/L2, register short stack
constexpr int kSrcBvhL = 4;         // BVH + spheres in LDS, scratch stack
constexpr int kSrcBvhLS = 5;        // BVH + spheres in LDS, register short stack
constexpr int kSrcBvhP = 6;         // top of the BVH in LDS, spheres from HBM/L2, register short stack

template <int kSrc>
struct Src {
    static constexpr bool bvh = kSrc >= kSrcBvhG;
    static constexpr bool sph_lds = kSrc == kSrcLds || kSrc == kSrcBvhL || kSrc == kSrcBvhLS;
    static constexpr int nodes = (kSrc == kSrcBvhL || kSrc == kSrcBvhLS) ? 2 : (kSrc == kSrcBvhP ? 1 : 0);
    static constexpr bool short_stack = kSrc == kSrcBvhGS || kSrc == kSrcBvhLS || kSrc == kSrcBvhP;
    // all-LDS staging is ~60 KB per workgroup: 1024-thread groups share one copy between 16 waves
    static constexpr int threads = nodes == 2 ? 1024 : 256;
};

template <int kSrc>
constexpr int threads_of() { return Src<kSrc>::threads; }

// Stage what the source keeps in LDS; returns the view the queries use.
template <int kSrc>
__device__ __forceinline__ BvhView stage_lds(const DevScene& sc, const WfBufs& b, unsigned char* lds) {
    constexpr int T = threads_of<kSrc>();
    BvhView v{nullptr, 0, sc.bvh, sc.spheres, sc.sphere_obj};
    if constexpr (kSrc == kSrcLds) {
        DevSphere* ls = reinterpret_cast<DevSphere*>(lds);
        for (int i = threadIdx.x; i < sc.n_spheres; i += T) ls[i] = sc.spheres[i];
        v.sph = ls;
        __syncthreads();
    } else if constexpr (Src<kSrc>::nodes > 0) {
        DevBvhNode* ln = reinterpret_cast<DevBvhNode*>(lds);
        for (int i = threadIdx.x; i < b.lds_nodes; i += T) ln[i] = sc.bvh[i];
        v.lnodes = ln;
        v.nl = b.lds_nodes;
        if constexpr (Src<kSrc>::sph_lds) {
            DevSphere* ls = reinterpret_cast<DevSphere*>(lds + static_cast<size_t>(b.lds_nodes) * sizeof(DevBvhNode));
            int32_t* lo = reinterpret_cast<int32_t*>(ls + sc.n_spheres);
            for (int i = threadIdx.x; i < sc.n_spheres; i += T) { ls[i] = sc.spheres[i]; lo[i] = sc.sphere_obj[i]; }
            v.sph = ls;
            v.obj = lo;
        }
        __syncthreads();
    }
    return v;
}

template <int kSrc, bool kCount>
__device__ __forceinline__ Hit nearest_any(const DevScene& sc, const BvhView& v, const Ray& r, Work* w) {
    if constexpr (Src<kSrc>::bvh) return nearest_bvh<kCount, Src<kSrc>::nodes, Src<kSrc>::short_stack>(sc, v, r, w);
    else return nearest_brute<kCount>(sc, v.sph, r, w);
}

template <int kSrc, bool kCount>
__device__ __forceinline__ bool occluded_any(const DevScene& sc, const BvhView& v, const Ray& r, bool has_range,
                                             double r2, Work* w) {
    if constexpr (Src<kSrc>::bvh)
        return occluded_bvh<kCount, Src<kSrc>::nodes, Src<kSrc>::short_stack>(sc, v, r, has_range, r2, w);
    else return occluded_brute<kCount>(sc, v.sph, r, has_range, r2, w);
}

// One atomic per wave into totals[at], totals[at + 1].
template <bool kCount>
__device__ __forceinline__ void flush_work(const WfBufs& b, int at, Work w) {
    if constexpr (kCount) {
        unsigned long long bx = w.boxes, sp = w.spheres;
        for (int off = 32; off > 0; off >>= 1) {
            bx += __shfl_xor(bx, off, 64);
            sp += __shfl_xor(sp, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&b.totals[at], bx);
            atomicAdd(&b.totals[at + 1], sp);
        }
    }
}

__device__ __forceinline__ void set_terminal(const WfBufs& b, uint32_t p, Col c, int k) {
    b.term[0][p] = c.r; b.term[1][p] = c.g; b.term[2][p] = c.b;
    b.nlev[p] = static_cast<uint8_t>(k);
}

// Scene::intersect for every ray of Q_k (generation 0: the camera rays of the
// chunk, computed here).  Outcomes that end the chain without lighting are
// resolved on the spot (miss -> background; depth cut-off or insignificant
// surface -> ambient, raytrace.rs:32-35); the rest become dense shade records.
template <int kSrc, bool kCam, bool kCount>
__global__ __launch_bounds__(threads_of<kSrc>()) void wf_nearest(DevScene sc, FrameParams fp, WfBufs b, int k) {
    constexpr int T = threads_of<kSrc>();
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const BvhView v = stage_lds<kSrc>(sc, b, lds);
    Work w;
    const uint32_t n = kCam ? b.slots : b.cnt[kCntQ + k];
    for (uint32_t base = blockIdx.x * T; base < n; base += gridDim.x * T) {
        const uint32_t i = base + threadIdx.x;
        bool shade = false;
        Ray r{};
        double sig = 0.0, ptx = 0.0, pty = 0.0, ptz = 0.0;
        uint32_t p = 0;
        Hit h{};
        if (i < n && entry_ray<kCam>(sc, fp, b, k, i, r, sig, p)) {
            h = nearest_any<kSrc, kCount>(sc, v, r, &w);
            if (h.obj == INT32_MAX) {
                set_terminal(b, p, Col{sc.bg[0], sc.bg[1], sc.bg[2]}, k);          // raytrace.rs:265, 228-232
            } else {
                const DevMaterial& m = sc.mats[h.obj];
                const bool lit = static_cast<uint32_t>(k) <= fp.max_depth &&       // raytrace.rs:33
                                 (m.kd_sig * sig > kMinSignificance || m.ks_sig * sig > kMinSignificance);
                if (!lit) {
                    set_terminal(b, p, Col{m.amb[0], m.amb[1], m.amb[2]}, k);
                } else {
                    shade = true;
                    ptx = r.ox + r.dx * h.t; pty = r.oy + r.dy * h.t; ptz = r.oz + r.dz * h.t;   // ray.cast(t)
                }
            }
        }
        const uint32_t slot = wave_append(&b.cnt[kCntS + k], shade);
        if (shade) {
            b.sr_pt[0][slot] = ptx; b.sr_pt[1][slot] = pty; b.sr_pt[2][slot] = ptz;
            b.sr_d[0][slot] = r.dx; b.sr_d[1][slot] = r.dy; b.sr_d[2][slot] = r.dz;
            b.sr_sig[slot] = sig;
            b.sr_obj[slot] = h.obj;
            b.sr_prim[slot] = h.prim;
            b.sr_pix[slot] = p;
            b.occ[slot] = 0u;
        }
    }
    flush_work<kCount>(b, 2, w);
}

// The shadow queries of every shade record (raytrace.rs:39-49): one work-item
// per (record, light) pair -- the lights of one hit are independent queries --
// setting bit l of the record's occlusion mask.
template <int kSrc, bool kCount>
__global__ __launch_bounds__(threads_of<kSrc>()) void wf_occlusion(DevScene sc, FrameParams fp, WfBufs b, int k) {
    constexpr int T = threads_of<kSrc>();
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const BvhView v = stage_lds<kSrc>(sc, b, lds);
    Work w;
    const uint32_t L = static_cast<uint32_t>(sc.n_lights);
    const uint32_t n = b.cnt[kCntS + k] * L;
    for (uint32_t q = blockIdx.x * T + threadIdx.x; q < n; q += gridDim.x * T) {
        const uint32_t j = q / L, l = q - j * L;
        const double ptx = b.sr_pt[0][j], pty = b.sr_pt[1][j], ptz = b.sr_pt[2][j];
        double lx, ly, lz, r2;
        const bool has_range = light_dir(sc.lights[l], ptx, pty, ptz, lx, ly, lz, r2);
        const Ray sray{ptx + lx * kEps, pty + ly * kEps, ptz + lz * kEps, lx, ly, lz};
        if (occluded_any<kSrc, kCount>(sc, v, sray, has_range, r2, &w)) atomicOr(&b.occ[j], 1u << l);
    }
    flush_work<kCount>(b, 4, w);
}

// The Phong sum of every shade record (raytrace.rs:31-56), then either the
// level push + reflection ray into Q_{k+1} (raytrace.rs:58-64) or the end of
// the chain.
__global__ __launch_bounds__(kBlock) void wf_shade(DevScene sc, FrameParams fp, WfBufs b, int k) {
    const uint32_t n = b.cnt[kCntS + k];
    const int qn = (k + 1) & 1;
    for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
        const uint32_t j = base + threadIdx.x;
        bool refl = false;
        Ray rr{};
        double nsig = 0.0;
        uint32_t p = 0;
        if (j < n) {
            const double ptx = b.sr_pt[0][j], pty = b.sr_pt[1][j], ptz = b.sr_pt[2][j];
            const double dx = b.sr_d[0][j], dy = b.sr_d[1][j], dz = b.sr_d[2][j];
            const double sig = b.sr_sig[j];
            const int32_t obj = b.sr_obj[j];
            p = b.sr_pix[j];
            const DevMaterial& m = sc.mats[obj];
            Col res{m.amb[0], m.amb[1], m.amb[2]};                               // raytrace.rs:32
            const bool diffuse = m.kd_sig * sig > kMinSignificance;
            const bool specular = m.ks_sig * sig > kMinSignificance;
            double nx, ny, nz;
            hit_normal(sc, sc.spheres, b.sr_prim[j], ptx, pty, ptz, nx, ny, nz);
            if (nx * dx + ny * dy + nz * dz > 0.0) { nx = -nx; ny = -ny; nz = -nz; }
            if (sc.n_lights > 0) {
                const uint32_t mask = b.occ[j];
                for (int l = 0; l < sc.n_lights; ++l) {
                    if ((mask >> l) & 1u) continue;                              // shadowed (raytrace.rs:42-49)
                    const DevLight& L = sc.lights[l];
                    double lx, ly, lz, r2;
                    light_dir(L, ptx, pty, ptz, lx, ly, lz, r2);
                    add_light(res, m, L, diffuse, specular, lx, ly, lz, nx, ny, nz, dx, dy, dz);
                }
            }
            if (specular) {
                const size_t at = static_cast<size_t>(k) * b.cap + p;
                b.st[0][at] = res.r; b.st[1][at] = res.g; b.st[2][at] = res.b;
                b.st_obj[at] = obj;
                rr = reflect_ray(Ray{0, 0, 0, dx, dy, dz}, ptx, pty, ptz, nx, ny, nz);
                nsig = sig * m.ks_sig;
                refl = true;
            } else {
                set_terminal(b, p, res, k);
            }
        }
        const uint32_t slot = wave_append(&b.cnt[kCntQ + k + 1], refl);
        if (refl) {
            b.qo[qn][0][slot] = rr.ox; b.qo[qn][1][slot] = rr.oy; b.qo[qn][2][slot] = rr.oz;
            b.qd[qn][0][slot] = rr.dx; b.qd[qn][1][slot] = rr.dy; b.qd[qn][2][slot] = rr.dz;
            b.qsig[qn][slot] = nsig;
            b.qpix[qn][slot] = p;
        }
    }
}

// The fold factor of a level is the specular colour of its object
// (raytrace.rs:63).
__device__ __forceinline__ Col fold_pixel(const DevScene& sc, const WfBufs& b, const double* ks_lds, uint32_t p) {
    Col acc{b.term[0][p], b.term[1][p], b.term[2][p]};
    for (int k = static_cast<int>(b.nlev[p]) - 1; k >= 0; --k) {       // res_k + ks_k * acc
        const size_t at = static_cast<size_t>(k) * b.cap + p;
        const int32_t obj = b.st_obj[at];
        double k0, k1, k2;
        if (ks_lds) {
            k0 = ks_lds[3 * obj]; k1 = ks_lds[3 * obj + 1]; k2 = ks_lds[3 * obj + 2];
        } else {
            const DevMaterial& m = sc.mats[obj];
            k0 = m.ks[0]; k1 = m.ks[1]; k2 = m.ks[2];
        }
        acc.r = b.st[0][at] + k0 * acc.r;
        acc.g = b.st[1][at] + k1 * acc.g;
        acc.b = b.st[2][at] + k2 * acc.b;
    }
    return acc;
}

// kStaged: every group of 256 pixels lies in one output row (tile_w % 256 == 0,
// BGR rows unpadded and dword aligned): the block assembles its 3 KiB of RGB
// and 768 B of BGR in LDS and stores them as whole dwords.
template <bool kStaged>
__global__ __launch_bounds__(kBlock) void wf_fold(DevScene sc, FrameParams fp, WfBufs b, int n_objects) {
    __shared__ float s_rgb[3 * kBlock];
    __shared__ uint32_t s_bgr[3 * kBlock / 4];
    // (an LDS table of the fold factors was measured slower: 52 KB per block
    // cut occupancy more than the gathers it saved)
    const double* ks_lds = nullptr;
    (void)n_objects;
    const uint32_t npix = fp.tile_w * fp.rows;
    for (uint32_t base = blockIdx.x * kBlock; base < npix; base += gridDim.x * kBlock) {
        const uint32_t p = base + threadIdx.x;
        if constexpr (!kStaged) {
            if (p < npix) {
                const Col res = average_samples(fold_pixel(sc, b, ks_lds, p), fp.spp);
                write_pixel(fp, p % fp.tile_w, fp.row0 + p / fp.tile_w, res);
            }
        } else {
            const Col res = average_samples(fold_pixel(sc, b, ks_lds, p), fp.spp);   // npix % 256 == 0 here
            s_rgb[3 * threadIdx.x + 0] = static_cast<float>(res.r);
            s_rgb[3 * threadIdx.x + 1] = static_cast<float>(res.g);
            s_rgb[3 * threadIdx.x + 2] = static_cast<float>(res.b);
            uint8_t* sb = reinterpret_cast<uint8_t*>(s_bgr);
            sb[3 * threadIdx.x + 0] = to_srgb(res.b);
            sb[3 * threadIdx.x + 1] = to_srgb(res.g);
            sb[3 * threadIdx.x + 2] = to_srgb(res.r);
            __syncthreads();
            const uint32_t row = fp.row0 + base / fp.tile_w, lx0 = base % fp.tile_w;
            if (fp.out_rgb) {
                float* dst = fp.out_rgb + (static_cast<size_t>(row) * fp.tile_w + lx0) * 3;
                for (int q = threadIdx.x; q < 3 * kBlock; q += kBlock) dst[q] = s_rgb[q];
            }
            if (fp.out_bgr && threadIdx.x < 3 * kBlock / 4) {
                uint32_t* dst = reinterpret_cast<uint32_t*>(fp.out_bgr + static_cast<size_t>(row) * fp.bgr_pitch + 3 * lx0);
                dst[threadIdx.x] = s_bgr[threadIdx.x];
            }
            __syncthreads();
        }
    }
}

// Scene::intersect calls of this chunk: every pixel's camera ray, every later
// queue entry, and one shadow query per light per shaded hit.
// (atomics: chunks on different streams finish concurrently)
__global__ void wf_tally(FrameParams fp, WfBufs b, int n_lights, int generations) {
    const int t = threadIdx.x;                                  // kCntWords threads
    atomicAdd(&b.gen_totals[t], static_cast<unsigned long long>(b.cnt[t]));
    if (t == 0) {
        unsigned long long nearest = static_cast<unsigned long long>(fp.tile_w) * fp.rows, shadow = 0;
        for (int k = 1; k < generations; ++k) nearest += b.cnt[kCntQ + k];
        for (int k = 0; k < generations; ++k) shadow += static_cast<unsigned long long>(b.cnt[kCntS + k]) * n_lights;
        atomicAdd(&b.totals[0], nearest * fp.spp);
        atomicAdd(&b.totals[1], shadow * fp.spp);
    }
}

inline int blocks_for(uint64_t items, int cap_blocks) {
    uint64_t b = (items + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    return static_cast<int>(b < static_cast<uint64_t>(cap_blocks) ? b : cap_blocks);
}

}  // namespace

// Host-side launchers -------------------------------------------------------

// mode: 1 = spheres staged in LDS, 2 = read from global.
hipError_t launch_trace_frame(const DevScene& sc, const FrameParams& fp, int mode, hipStream_t stream) {
    dim3 grid((fp.tile_w + 15) / 16, (fp.rows + 15) / 16);
    if (mode == 1) {
        size_t lds = static_cast<size_t>(sc.n_spheres) * sizeof(DevSphere);
        hipLaunchKernelGGL(trace_frame_kernel<true>, grid, dim3(kBlock), lds, stream, sc, fp);
    } else {
        hipLaunchKernelGGL(trace_frame_kernel<false>, grid, dim3(kBlock), 0, stream, sc, fp);
    }
    return hipGetLastError();
}

// One chunk (fp.row0, fp.rows) through every generation.  Counters in b.cnt
// must be zero on entry (the caller memsets them).
template <int kSrc>
size_t lds_bytes_of(const DevScene& sc, const WfBufs& b) {
    size_t bytes = 0;
    if constexpr (kSrc == kSrcLds) bytes = static_cast<size_t>(sc.n_spheres) * sizeof(DevSphere);
    if constexpr (Src<kSrc>::nodes > 0) bytes = static_cast<size_t>(b.lds_nodes) * sizeof(DevBvhNode);
    if constexpr (Src<kSrc>::bvh && Src<kSrc>::sph_lds)
        bytes += static_cast<size_t>(sc.n_spheres) * (sizeof(DevSphere) + sizeof(int32_t));
    return bytes;
}

template <int kSrc, bool kCount>
void launch_generation(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int k, hipStream_t s) {
    constexpr int T = threads_of<kSrc>();
    const size_t lds = lds_bytes_of<kSrc>(sc, b);
    // Workgroups that stage LDS are kept resident-sized (the copy is per block);
    // the others fill every SIMD.
    const uint64_t cap = kSrc == kSrcLds ? 1024 : Src<kSrc>::nodes == 2 ? 512 : 16384;
    const int gq = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>((b.slots + T - 1) / T, cap)));
    const int gs = blocks_for(b.slots, 8192);
    if (k == 0) hipLaunchKernelGGL((wf_nearest<kSrc, true, kCount>), dim3(gq), dim3(T), lds, s, sc, fp, b, k);
    else hipLaunchKernelGGL((wf_nearest<kSrc, false, kCount>), dim3(gq), dim3(T), lds, s, sc, fp, b, k);
    if (sc.n_lights > 0) {
        const uint64_t items = static_cast<uint64_t>(b.slots) * sc.n_lights;
        const int go = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>((items + T - 1) / T, cap)));
        hipLaunchKernelGGL((wf_occlusion<kSrc, kCount>), dim3(go), dim3(T), lds, s, sc, fp, b, k);
    }
    hipLaunchKernelGGL(wf_shade, dim3(gs), dim3(kBlock), 0, s, sc, fp, b, k);
}

// One chunk (fp.row0, fp.rows) through every generation.  Counters in b.cnt
// must be zero on entry (the caller memsets them).  src: 0 brute/global,
// 1 brute/LDS, 2 BVH.
hipError_t launch_wavefront(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int src, bool count,
                            hipStream_t s, hipEvent_t mark, int mark_gen) {
    const int gens = static_cast<int>(fp.max_depth) + 2;          // depths 0 .. max_depth+1
    for (int k = 0; k < gens; ++k) {
#define RT_GEN(S) (count ? launch_generation<S, true>(sc, fp, b, k, s) : launch_generation<S, false>(sc, fp, b, k, s))
        switch (src) {
        case kSrcGlobal: RT_GEN(kSrcGlobal); break;
        case kSrcLds: RT_GEN(kSrcLds); break;
        case kSrcBvhG: RT_GEN(kSrcBvhG); break;
        case kSrcBvhGS: RT_GEN(kSrcBvhGS); break;
        case kSrcBvhL: RT_GEN(kSrcBvhL); break;
        case kSrcBvhLS: RT_GEN(kSrcBvhLS); break;
        default: RT_GEN(kSrcBvhP); break;
        }
#undef RT_GEN
        if (mark && k == mark_gen) {
            const hipError_t e = hipEventRecord(mark, s);
            if (e != hipSuccess) return e;
        }
    }
    const bool staged = fp.tile_w % kBlock == 0 && fp.bgr_pitch == 3 * fp.tile_w &&
                        (reinterpret_cast<uintptr_t>(fp.out_bgr) & 3) == 0;
    const dim3 gf(blocks_for(static_cast<uint64_t>(fp.tile_w) * fp.rows, 2048));
    const int n_objects = sc.n_spheres + sc.n_planes;
    if (staged) hipLaunchKernelGGL(wf_fold<true>, gf, dim3(kBlock), 0, s, sc, fp, b, n_objects);
    else hipLaunchKernelGGL(wf_fold<false>, gf, dim3(kBlock), 0, s, sc, fp, b, n_objects);
    hipLaunchKernelGGL(wf_tally, dim3(1), dim3(kCntWords), 0, s, fp, b, sc.n_lights, gens);
    return hipGetLastError();
}

hipError_t upload_srgb_table(const double* avg255) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_srgb_avg), avg255, 255 * sizeof(double));
}

}  // namespace rtamd
