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
#include "launch_api.hpp"
#include "trace_common.hpp"

namespace rtamd {

__constant__ double c_srgb_avg[255];

// RT_STAMP=1 (diagnostic builds only, tools/stamp_probe.py): per generation,
// wf_nearest's wave-cycles by phase from s_memtime stamps taken after a full
// wait, [k][0] setup (region scan + LDS staging), [1] ray load + region entry,
// [2] traversal, [3] finish (records, rays, terminals), [4] chunks, [5] waves;
// the counting kernels add [6] the slowest lane's and [7] all lanes' node
// visits per chunk (divergence); [8..10] the traversal's descend / leaf / pop
// loops (wave-cycles), [12] the slowest wave's traversal cycles, [13..15] the
// waves' iterations of those three loops.  Read with rt_debug_stamps (this
// build only).
#ifndef RT_STAMP
#define RT_STAMP 0
#endif
#if RT_STAMP
// (fields 12.. in a second array: a [kMaxGenerations][16] array hits a gfx950
// backend error, "Operand has incorrect register class")
__device__ unsigned long long g_stamp[kMaxGenerations][12];
__device__ unsigned long long g_stamp2[kMaxGenerations][4];
#define RT_STAMP_AT(v)                                                            \
    do {                                                                          \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");              \
        v = __builtin_amdgcn_s_memtime();                                         \
    } while (0)
#else
#define RT_STAMP_AT(v) ((void)0)
#endif

namespace {

constexpr int kBlock = 256;                 // 4 waves

// ---------------------------------------------------------------- megakernel

template <class SpherePtr>
__device__ Col trace_chain(const DevScene& sc, SpherePtr S, Ray ray, uint32_t max_depth, uint32_t& rays,
                           uint32_t& shadows) {
    double st_r[kMaxLevels], st_g[kMaxLevels], st_b[kMaxLevels], st_f[kMaxLevels];
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
        const double nd = nx * ray.dx + ny * ray.dy + nz * ray.dz;
        const Shading sh = shading_flags(m, sig, nd);
        const bool diffuse = sh.diffuse, specular = sh.specular;
        if (nd > 0.0) { nx = -nx; ny = -ny; nz = -nz; }
        if (diffuse || specular) {
            for (int li = 0; li < sc.n_lights; ++li) {
                const DevLight& L = sc.lights[li];
                double lx, ly, lz, r2;
                const bool has_range = light_dir(L, ptx, pty, ptz, lx, ly, lz, r2);
                const Ray sray{ptx + lx * kEps, pty + ly * kEps, ptz + lz * kEps, lx, ly, lz};
                ++rays;
                ++shadows;
                if (occluded_brute(sc, S, sray, has_range, r2)) continue;
                add_light(res, m, L, diffuse, specular, sh.f, lx, ly, lz, nx, ny, nz, ray.dx, ray.dy, ray.dz);
            }
        }
        if (!specular) { term = res; break; }
        st_r[lvl] = res.r; st_g[lvl] = res.g; st_b[lvl] = res.b; st_obj[lvl] = h.obj; st_f[lvl] = sh.f;
        ++lvl;
        ray = reflect_ray(ray, ptx, pty, ptz, nx, ny, nz);
        sig = (sh.f * sig) * m.ks_sig;                             // raytrace.rs:63 / 163
        ++depth;
    }
    Col acc = term;                                                // fold inner-first (raytrace.rs:63 / 163)
    for (int k = lvl - 1; k >= 0; --k) {
        const DevMaterial& m = sc.mats[st_obj[k]];
        acc.r = st_r[k] + (m.ks[0] * acc.r) * st_f[k];
        acc.g = st_g[k] + (m.ks[1] * acc.g) * st_f[k];
        acc.b = st_b[k] + (m.ks[2] * acc.b) * st_f[k];
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
//
// Queues are BLOCK-PARTITIONED: a queue of generation k is G regions of R
// entries, region r written only by workgroup r of the producing kernel
// (appending through an LDS counter) and its size published in rq/rs[k*G+r].
// No global atomic sits on the data path: a single global queue counter
// serialises at ~88 atomics/us (MI355X_MICROARCH.md, "dequeue") and was the
// measured bottleneck of the first version.  Consumers read the queue DENSELY:
// each workgroup scans the G region sizes into LDS and maps item i to
// (region, offset) by binary search, so small tail queues still fill whole
// waves.  Every queue kernel runs exactly G workgroups of kWfThreads and
// grid-strides over its items, so workgroup b produces at most R outputs.

// Wave-aggregated append to an LDS counter: one LDS atomic per wave, lanes
// get consecutive slots in lane order.  All 64 lanes must call it.
__device__ __forceinline__ uint32_t lds_append(uint32_t* counter, bool want) {
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

// Work dealing: a queue is consumed in 64-item chunks; chunk c goes to wave
// slot c mod W (W = G * 16 waves).  Slots are numbered workgroup-first
// (b.wg_major = 0: a small tail queue spreads over every workgroup) or
// workgroup-major (b.wg_major = 1: consecutive chunks fill one workgroup's
// waves, so the workgroups past the queue's end exit at once and free their
// CU for the kernels of the other stream).  Either way a workgroup takes at
// most 16 chunks per round of W, i.e. at most R items.  Loop condition and
// chunk are wave-uniform.
// A queue smaller than b.spread_below items is always dealt workgroup-first
// (its few chunks then occupy every CU instead of a few whole workgroups).
__device__ __forceinline__ bool deal_major(const WfBufs& b, uint32_t n) { return b.wg_major && n >= b.spread_below; }

__device__ __forceinline__ uint32_t wave_slot(const WfBufs& b, uint32_t n) {
    const uint32_t wave = threadIdx.x >> 6;
    return deal_major(b, n) ? blockIdx.x * (kWfThreads / 64) + wave : wave * b.G + blockIdx.x;
}

// Whether this workgroup's first chunk is below n (workgroup-uniform).
__device__ __forceinline__ bool wg_has_work(const WfBufs& b, uint32_t n, uint32_t width = 64) {
    const uint64_t first = deal_major(b, n) ? static_cast<uint64_t>(blockIdx.x) * (kWfThreads / 64) : blockIdx.x;
    return first * width < n;
}

#define RT_FOR_CHUNKS(b, n, j)                                                              \
    for (uint32_t rt_c = wave_slot(b, n), rt_w = (b).G * (kWfThreads / 64);                  \
         static_cast<uint64_t>(rt_c) * 64u < static_cast<uint64_t>(n); rt_c += rt_w)        \
        if (const uint32_t j = rt_c * 64u + (threadIdx.x & 63u); true)

// Exclusive scan of the G region sizes `counts` into s_scan[0..G]
// (s_scan[G] = queue size; G <= kMaxScan: the regions of up to kMaxScan / G
// consecutive generations, laid out one after the other).  s_wave: 16 words.
// Ends with a barrier.
template <int kT = kWfThreads>
__device__ void region_scan(const uint32_t* counts, uint32_t G, uint32_t* s_scan, uint32_t* s_wave) {
    const uint32_t per = (G + kT - 1) / kT;                         // 1 .. 4 (1024 threads), .. 16 (256)
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    constexpr int kPer = (kMaxScan + kT - 1) / kT;
    uint32_t v[kPer] = {}, sum = 0;
    for (uint32_t e = 0; e < per; ++e) {
        const uint32_t i = t * per + e;
        v[e] = i < G ? counts[i] : 0u;
        sum += v[e];
    }
    uint32_t inc = sum;                                              // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off, 64);
        if (lane >= static_cast<uint32_t>(off)) inc += o;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < kT / 64; ++w) { const uint32_t x = s_wave[w]; s_wave[w] = acc; acc += x; }
    }
    __syncthreads();
    uint32_t run = s_wave[wave] + inc - sum;
    for (uint32_t e = 0; e < per; ++e) {
        const uint32_t i = t * per + e;
        if (i < G) s_scan[i] = run;
        run += v[e];
    }
    if (t == kT - 1) s_scan[G] = run;
    __syncthreads();
}

// Dense item i (< s_scan[G]) -> its entry index region * R + offset.
__device__ __forceinline__ size_t region_entry(const uint32_t* s_scan, uint32_t G, uint32_t R, uint32_t i) {
    uint32_t lo = 0, hi = G - 1;                  // largest r with s_scan[r] <= i
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_scan[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return static_cast<size_t>(lo) * R + (i - s_scan[lo]);
}

// Generation-0 slot j of the chunk (8x8 tiles, row-major) -> local pixel.
__device__ __forceinline__ bool slot_pixel(const WfBufs& b, const FrameParams& fp, uint32_t j, uint32_t& lx, uint32_t& ly) {
    const uint32_t tile = j >> 6, w = j & 63u;
    lx = (tile % b.tiles_x) * 8u + (w & 7u);
    ly = (tile / b.tiles_x) * 8u + (w >> 3);
    return lx < fp.tile_w && ly < fp.rows;
}

// Streaming accesses (queues, shade records, levels): each word is written once
// and read once by a later launch, so they bypass L2 allocation (nontemporal)
// and leave it to the BVH / sphere lines the traversals re-read.
#ifndef RT_NT
#define RT_NT 1
#endif
template <class T>
__device__ __forceinline__ T ldn(const T* p) {
#if RT_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <class T, class U>
__device__ __forceinline__ void stn(T* p, U v) {
#if RT_NT
    __builtin_nontemporal_store(static_cast<T>(v), p);
#else
    *p = static_cast<T>(v);
#endif
}

// RT_NT >= 2: also the shadow-list entries and the shade records' last read;
// RT_NT >= 3: also the shadow kernels' record reads.
template <int kLevel, class T>
__device__ __forceinline__ T ldn_if(const T* p) {
#if RT_NT
    if constexpr (RT_NT >= kLevel) return __builtin_nontemporal_load(p);
#endif
    return *p;
}
template <int kLevel, class T, class U>
__device__ __forceinline__ void stn_if(T* p, U v) {
#if RT_NT
    if constexpr (RT_NT >= kLevel) { __builtin_nontemporal_store(static_cast<T>(v), p); return; }
#endif
    *p = static_cast<T>(v);
}

// the fold's loads (RT_NT_FOLD=1: nontemporal; measured 346 -> 413 us per fold at C3, so plain)
#ifndef RT_NT_FOLD
#define RT_NT_FOLD 0
#endif
constexpr int kNtFold = RT_NT_FOLD ? 1 : 99;
// the queue loads of the nearest-hit kernel (RT_NT_QLOAD=0: plain loads)
#ifndef RT_NT_QLOAD
#define RT_NT_QLOAD 1
#endif
constexpr int kNtQ = RT_NT_QLOAD ? 1 : 99;

__device__ __forceinline__ Ray load_ray(const WfBufs& b, int q, size_t i) {
    return Ray{ldn_if<kNtQ>(&b.qf(q, 0)[i]), ldn_if<kNtQ>(&b.qf(q, 1)[i]), ldn_if<kNtQ>(&b.qf(q, 2)[i]),
               ldn_if<kNtQ>(&b.qf(q, 3)[i]), ldn_if<kNtQ>(&b.qf(q, 4)[i]), ldn_if<kNtQ>(&b.qf(q, 5)[i])};
}

// Occupancy / unrolling of the fold and shading kernels (A/B builds: EXTRA=-D...)
#ifndef RT_FOLD_UNROLL
#define RT_FOLD_UNROLL 4        // levels whose loads are issued together
#endif
#ifndef RT_FOLD_WAVES
#define RT_FOLD_WAVES 1         // wf_fold's launch bounds: min waves per SIMD (1: the compiler's choice, 96 VGPRs)
#endif
#ifndef RT_FOLD_THREADS
#define RT_FOLD_THREADS 256     // wf_fold's workgroup size
#endif
#ifndef RT_SHADE_WAVES
#define RT_SHADE_WAVES 1
#endif

// Sphere sources of the wavefront intersection kernels.
constexpr int kSrcGlobal = 0;       // brute force, sphere list through the caches
constexpr int kSrcLds = 1;          // brute force, sphere list staged in LDS per workgroup
constexpr int kSrcBvhG = 2;         // binary BVH from HBM/L2 (trees too deep for the 4-wide stack)
constexpr int kSrcBvhL8 = 7;        // binary BVH + spheres in LDS, 64 VGPRs: two 1024-thread workgroups per CU
constexpr int kSrcBvhL8C = 9;       // kSrcBvhL8 with compact 32-bit stack entries (small trees, depth <= kShortStack)
constexpr int kSrcBvh4L = 10;       // 4-wide BVH + spheres in LDS, 64 VGPRs (shadow queries without a light grid)
constexpr int kSrcBvh4G = 11;       // 4-wide BVH + spheres from HBM/L2, 64 VGPRs (idem)
// Trees too large for LDS: the breadth-first top of the binary tree (DevScene::pfx2
// nodes, chosen by the host) in LDS, the rest and the spheres from HBM/L2 (64 VGPRs).
constexpr int kSrcBvhP = 8;         // binary BVH, LDS prefix
constexpr int kSrcBvhPH = 5;        // binary BVH with binary16 bounds (DevBvhNodeH), LDS prefix of twice the nodes
constexpr int kSrcBvhPHC = 6;       // kSrcBvhPH with compact 32-bit stack entries (18-bit codes: <= 16383 spheres)
// Shadow kernel when every light is a point light with a light-view grid: no
// tree walk at all (so no traversal stack in scratch and no register spills),
// spheres from LDS or HBM/L2.
constexpr int kSrcGridL = 14;
constexpr int kSrcGridG = 15;
// Generation 0 only: camera rays through the camera's view grid (nearest_cgrid),
// spheres staged in LDS (22) or read through L2 (23).
constexpr int kSrcCamGridL = 22;
constexpr int kSrcCamGridG = 23;
// The quantised 4-wide tree (DevQNode4, nearest_q4), spheres from HBM/L2 (64 VGPRs): every
// node in LDS (25, trees of <= ~1500 nodes such as C4's) or the breadth-first top
// DevScene::pfxq nodes in LDS and the rest through L2 (26, C5); tuning qtree, off by default
constexpr int kSrcQ4 = 25;
constexpr int kSrcQ4P = 26;

template <int kSrc>
struct Src {
    static constexpr bool grid = kSrc == kSrcGridL || kSrc == kSrcGridG;
    static constexpr bool cgrid = kSrc == kSrcCamGridL || kSrc == kSrcCamGridG;
    static constexpr bool q4 = kSrc == kSrcQ4 || kSrc == kSrcQ4P;
    static constexpr bool bvh = kSrc >= kSrcBvhG && !grid && !cgrid && !q4;
    static constexpr bool wide = kSrc == kSrcBvh4L || kSrc == kSrcBvh4G;
    static constexpr bool half = kSrc == kSrcBvhPH || kSrc == kSrcBvhPHC;
    static constexpr int compact_bits = kSrc == kSrcBvhL8C ? 16 : kSrc == kSrcBvhPHC ? 18 : 0;
    static constexpr bool prefix = kSrc == kSrcBvhP || half;
    static constexpr bool all_lds = kSrc == kSrcBvhL8 || kSrc == kSrcBvhL8C || kSrc == kSrcBvh4L;
    static constexpr bool sph_lds = kSrc == kSrcLds || all_lds || kSrc == kSrcGridL || kSrc == kSrcCamGridL;
    static constexpr int nodes = all_lds ? 2 : half ? 3 : prefix ? 1 : 0;
    static constexpr int waves = kSrc >= kSrcBvhL8 || half ? 8 : 4;   // min waves per SIMD
};

// Nodes of the LDS prefix of a prefix source.
template <int kSrc>
__host__ __device__ inline int32_t prefix_nodes(const DevScene& sc) {
    if (kSrc == kSrcBvhP) return min(sc.n_bvh, sc.pfx2);
    if (Src<kSrc>::half) return min(sc.n_bvh, 2 * sc.pfx2);     // same LDS bytes, 32-B nodes
    if (kSrc == kSrcQ4P) return min(sc.n_q4, sc.pfxq);
    if (kSrc == kSrcQ4) return sc.n_q4;
    return 0;
}

// LDS layout of the intersection kernels: [staged data][region scan, G + 1][wave sums, 16][counter].
template <int kSrc>
__host__ __device__ inline size_t staged_bytes(const DevScene& sc) {
    size_t bytes = 0;
    if (Src<kSrc>::q4) bytes = static_cast<size_t>(prefix_nodes<kSrc>(sc)) * sizeof(DevQNode4);
    if (kSrc == kSrcLds || kSrc == kSrcGridL) bytes = static_cast<size_t>(sc.n_spheres) * sizeof(DevSphere);
    if (kSrc == kSrcCamGridL) bytes = static_cast<size_t>(sc.n_spheres) * (sizeof(DevSphere) + sizeof(int32_t));
    if (kSrc == kSrcBvhP) bytes = static_cast<size_t>(prefix_nodes<kSrc>(sc)) * sizeof(DevBvhNode);
    if (Src<kSrc>::half) bytes = static_cast<size_t>(prefix_nodes<kSrc>(sc)) * sizeof(DevBvhNodeH);
    if (Src<kSrc>::nodes == 2)
        bytes = Src<kSrc>::wide ? static_cast<size_t>(sc.n_bvh4) * kBvh4Planes * sizeof(DevBvh4Plane) : node_planes_bytes(sc.n_bvh);
    if (Src<kSrc>::bvh && Src<kSrc>::sph_lds) bytes += static_cast<size_t>(sc.n_spheres) * (sizeof(DevSphere) + sizeof(int32_t));
    return (bytes + 15) / 16 * 16;
}

// Stage what the source keeps in LDS (the whole tree and the spheres, or the
// top of the tree); returns the view the queries use.
// kNearest: the nearest-hit walk's byte-offset node encoding (stage_node_planes).
template <int kSrc, bool kNearest = false>
__device__ __forceinline__ BvhView stage_lds(const DevScene& sc, unsigned char* lds) {
    constexpr int T = kWfThreads;
    BvhView v = global_view(sc);
    size_t off = 0;
    if constexpr (Src<kSrc>::q4) {
        const int32_t nl = prefix_nodes<kSrc>(sc);
        uint4* ln = reinterpret_cast<uint4*>(lds);
        const uint4* gn = reinterpret_cast<const uint4*>(sc.q4);
        for (int i = threadIdx.x; i < 3 * nl; i += T) ln[i] = gn[i];
        v.q4l = reinterpret_cast<const DevQNode4*>(lds);
        v.nq = nl;
        return v;
    } else if constexpr (kSrc == kSrcBvhP) {
        DevBvhNode* ln = reinterpret_cast<DevBvhNode*>(lds);
        const int32_t nl = prefix_nodes<kSrc>(sc);
        for (int i = threadIdx.x; i < nl; i += T) ln[i] = sc.bvh[i];
        v.pnodes = ln;
        v.nl = nl;
        return v;
    } else if constexpr (Src<kSrc>::half) {
        DevBvhNodeH* ln = reinterpret_cast<DevBvhNodeH*>(lds);
        const int32_t nl = prefix_nodes<kSrc>(sc);
        for (int i = threadIdx.x; i < nl; i += T) ln[i] = sc.bvh_h[i];
        v.hpnodes = ln;
        v.hgnodes = sc.bvh_h;
        v.nl = nl;
        return v;
    } else if constexpr (kSrc == kSrcLds || kSrc == kSrcGridL) {
        DevSphere* ls = reinterpret_cast<DevSphere*>(lds);
        for (int i = threadIdx.x; i < sc.n_spheres; i += T) ls[i] = sc.spheres[i];
        v.sph = ls;
        return v;
    } else if constexpr (kSrc == kSrcCamGridL) {
        DevSphere* ls = reinterpret_cast<DevSphere*>(lds);
        int32_t* lo = reinterpret_cast<int32_t*>(ls + sc.n_spheres);
        for (int i = threadIdx.x; i < sc.n_spheres; i += T) { ls[i] = sc.spheres[i]; lo[i] = sc.sphere_obj[i]; }
        v.sph = ls;
        v.obj = lo;
        return v;
    } else if constexpr (Src<kSrc>::nodes == 2 && Src<kSrc>::wide) {
        DevBvh4Plane* lp = reinterpret_cast<DevBvh4Plane*>(lds);
        const int n = kBvh4Planes * sc.n_bvh4;
        for (int i = threadIdx.x; i < n; i += T) lp[i] = sc.bvh4[i];
        v.p4 = lp;
        off = static_cast<size_t>(n) * sizeof(DevBvh4Plane);
    } else if constexpr (Src<kSrc>::nodes == 2) {
        v.lnodes = stage_node_planes<T, kNearest>(sc.bvh, sc.n_bvh, lds);
        v.nl = sc.n_bvh;
        off = node_planes_bytes(sc.n_bvh);
    }
    if constexpr (Src<kSrc>::bvh && Src<kSrc>::sph_lds) {
        DevSphere* ls = reinterpret_cast<DevSphere*>(lds + off);
        int32_t* lo = reinterpret_cast<int32_t*>(ls + sc.n_spheres);
        for (int i = threadIdx.x; i < sc.n_spheres; i += T) { ls[i] = sc.spheres[i]; lo[i] = sc.sphere_obj[i]; }
        v.sph = ls;
        v.obj = lo;
    }
    return v;
}

// register entries on top of the binary16 prefix walk's stack (src 5, 6): three (C4 49.80-49.86
// vs 50.07-50.09 ms with two, 50.41 with one, 50.36 with four; C5 equal within 0.5%)
#ifndef RT_HALF_REG
#define RT_HALF_REG 3
#endif
// register entries on top of the compact stack (the whole tree in LDS, src 9): one (C3 3.054 vs
// 3.116 ms, 8-way share 0.756 vs 0.765 ms on one box; two 3.168 vs 3.144 ms); A/B builds:
// EXTRA=-DRT_COMPACT_REG=n
#ifndef RT_COMPACT_REG
#define RT_COMPACT_REG 1
#endif
// Scene::intersect of one ray through the source's structure (scene.rs:247-249).
template <int kSrc, bool kCount>
__device__ __forceinline__ Hit nearest_any(const DevScene& sc, const BvhView& v, const Ray& r, Work* w) {
    if constexpr (Src<kSrc>::cgrid) return nearest_cgrid<kCount>(sc, v, r, w);
    else if constexpr (Src<kSrc>::q4) return nearest_q4<kCount, kSrc == kSrcQ4>(sc, v, r, w);
    // two stack entries in registers when the tree is read through L2 below its LDS prefix
    // (C4 74.0 -> 71.4 ms); RT_COMPACT_REG on the compact stack with the whole tree in LDS (the
    // 64-bit stack: 3.66 -> 3.80 ms with 1-4 in round 2)
    else if constexpr (Src<kSrc>::bvh && Src<kSrc>::nodes == 2)
        return nearest_bvh_bl<kCount, 2, Src<kSrc>::compact_bits ? RT_COMPACT_REG : 0, Src<kSrc>::compact_bits>(sc, v, r, w);
    else if constexpr (Src<kSrc>::bvh && Src<kSrc>::half) return nearest_bvh_bl<kCount, 3, RT_HALF_REG, Src<kSrc>::compact_bits>(sc, v, r, w);
    else if constexpr (Src<kSrc>::bvh && Src<kSrc>::prefix) return nearest_bvh_bl<kCount, 1, 2>(sc, v, r, w);
    else if constexpr (Src<kSrc>::bvh) return nearest_bvh_bl<kCount, 0, 0>(sc, v, r, w);
    else return nearest_brute<kCount>(sc, v.sph, r, w);
}

template <int kSrc, bool kCount>
__device__ __forceinline__ bool occluded_any(const DevScene& sc, const BvhView& v, const Ray& r, bool has_range,
                                             double r2, int32_t hint, Work* w) {
    if constexpr (Src<kSrc>::wide) return occluded_bvh4<kCount>(sc, v, r, has_range, r2, hint, w);
    else if constexpr (Src<kSrc>::bvh) return occluded_bvh<kCount, Src<kSrc>::nodes, 0>(sc, v, r, has_range, r2, hint, w);
    else return occluded_brute<kCount>(sc, v.sph, r, has_range, r2, w);
}

// One global atomic per workgroup into totals[at], totals[at + 1]
// (instrumented kernels only; every thread of the workgroup must call it).
template <bool kCount>
__device__ __forceinline__ void flush_work(const WfBufs& b, int at, Work w) {
    if constexpr (kCount) {
        __shared__ unsigned long long s_w[2];
        if (threadIdx.x == 0) { s_w[0] = 0; s_w[1] = 0; }
        __syncthreads();
        unsigned long long bx = w.boxes, sp = w.spheres;
        for (int off = 32; off > 0; off >>= 1) {
            bx += __shfl_xor(bx, off, 64);
            sp += __shfl_xor(sp, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&s_w[0], bx);
            atomicAdd(&s_w[1], sp);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicAdd(&b.totals[at], s_w[0]);
            atomicAdd(&b.totals[at + 1], s_w[1]);
        }
    }
}

// A camera ray that misses everything: the pixel is the background averaged
// over samples, precomputed on the host (FrameParams::bg_*), written here (it
// starts no chain, so wf_fold never sees it).
__device__ __forceinline__ void write_background_pixel(const FrameParams& fp, const WfBufs& b, uint32_t p) {
    const uint32_t lx = p % fp.tile_w, row = fp.row0 + p / fp.tile_w;
    if (fp.out_rgb) {
        float* q = fp.out_rgb + (static_cast<size_t>(row) * fp.tile_w + lx) * 3;
        q[0] = fp.bg_rgb[0]; q[1] = fp.bg_rgb[1]; q[2] = fp.bg_rgb[2];
    }
    if (fp.out_bgr) {
        uint8_t* q = fp.out_bgr + static_cast<size_t>(row) * fp.bgr_pitch + 3u * lx;
        q[0] = fp.bg_bgr[0]; q[1] = fp.bg_bgr[1]; q[2] = fp.bg_bgr[2];
        if (lx == fp.tile_w - 1)       // BMP row padding is zero (main.rs:42)
            for (uint32_t k = 3u * fp.tile_w; k < fp.bgr_pitch; ++k) fp.out_bgr[static_cast<size_t>(row) * fp.bgr_pitch + k] = 0;
    }
}

// The colour that ends a chain without lighting: the background (obj INT32_MAX,
// a miss) or the object's ambient colour (cut-off, insignificant surface).
__device__ __forceinline__ Col end_colour(const DevScene& sc, int32_t obj) {
    if (obj == INT32_MAX) return Col{sc.bg[0], sc.bg[1], sc.bg[2]};
    const DevMaterial& m = sc.mats[obj];
    return Col{m.amb[0], m.amb[1], m.amb[2]};
}

typedef uint32_t U32x4 __attribute__((ext_vector_type(4)));

// The final colour of chain c (pixel p of the chunk): into ccol[c] for wf_compose
// (chain order: coalesced), or straight into the frame.
__device__ __forceinline__ void emit_chain(const FrameParams& fp, const WfBufs& b, uint32_t c, uint32_t p, Col res,
                                           const double* srgb) {
    if (b.compose) {
        const uint32_t q = static_cast<uint32_t>(to_srgb(res.b, srgb)) | (static_cast<uint32_t>(to_srgb(res.g, srgb)) << 8) |
                           (static_cast<uint32_t>(to_srgb(res.r, srgb)) << 16);
        const U32x4 v = {__float_as_uint(static_cast<float>(res.r)), __float_as_uint(static_cast<float>(res.g)),
                         __float_as_uint(static_cast<float>(res.b)), q};
        stn(reinterpret_cast<U32x4*>(b.ccol()) + c, v);
    } else {
        write_pixel(fp, p % fp.tile_w, fp.row0 + p / fp.tile_w, res, srgb);
    }
}

// Chain c ends in generation k with colour col (wf_fold folds its k levels onto it).
__device__ __forceinline__ void set_terminal(const WfBufs& b, uint32_t c, Col col, int k) {
    stn(&b.term(0)[c], col.r); stn(&b.term(1)[c], col.g); stn(&b.term(2)[c], col.b);
    b.nlev()[c] = static_cast<uint8_t>(k);
}

// LDS of a queue kernel after its staged data.
constexpr int kQueueCounters = 2;           // this workgroup's shade records and reflection rays

struct QueueLds {
    uint32_t* scan;     // G + 1
    uint32_t* wave;     // 16
    uint32_t* count;    // shade records, reflection rays appended by this workgroup
};

__device__ __forceinline__ QueueLds queue_lds(unsigned char* at, uint32_t G) {
    uint32_t* p = reinterpret_cast<uint32_t*>(at);
    return QueueLds{p, p + G + 1, p + G + 1 + kWfThreads / 64};
}

__host__ __device__ inline size_t queue_lds_bytes(uint32_t G) { return (G + 1 + kWfThreads / 64 + kQueueCounters) * 4u; }

// What follows a nearest hit (all 64 lanes call it; `live` lanes carry a
// query): a miss or a cut-off ends the chain at once (terminal colour; a
// camera ray that ends writes its final pixel); a lit hit becomes a shade
// record of generation k, and a specular one also queues its reflection ray in
// Q_{k+1}.  counts[0..1]: this workgroup's LDS append counters (records, rays).
// Chains: a lit camera hit starts chain c = its record's entry (generation 0,
// pixel cpix[c]); its records, reflection rays, levels and terminal carry c
// (`p` is the pixel for kCam, the chain otherwise), so the levels and
// terminals of a generation are written in about the order of its records.
template <bool kCam, bool kFresnel>
__device__ __forceinline__ void finish_nearest(const DevScene& sc, const FrameParams& fp, const WfBufs& b,
                                               const DevSphere* sph, int k, bool live, const Ray& r, double sig,
                                               uint32_t p, const Hit& h, uint32_t* counts, size_t obase, size_t rbase) {
    bool shade = false, refl = false;
    double ptx = 0.0, pty = 0.0, ptz = 0.0, nsig = 0.0;
    Ray rr{};
    // a chain that ends here without lighting: background (end_obj INT32_MAX) or the
    // object's ambient colour
    bool ends = false;
    int32_t end_obj = INT32_MAX;
    if (live) {
        if (h.obj == INT32_MAX) {                                           // raytrace.rs:265, 228-232
            if constexpr (kCam) {                                           // no levels: final now
                if (b.compose) stn(&b.pmap()[p], kPixBackground);
                else write_background_pixel(fp, b, p);
            } else {
                ends = true;
            }
        } else {
            const DevMaterial& m = sc.mats[h.obj];
            if (static_cast<uint32_t>(k) > fp.max_depth) {                  // raytrace.rs:33 / 126
                ends = true;
                end_obj = h.obj;
            } else {
                ptx = r.ox + r.dx * h.t; pty = r.oy + r.dy * h.t; ptz = r.oz + r.dz * h.t;   // ray.cast(t)
                double nx, ny, nz;
                hit_normal(sc, sph, h.prim, ptx, pty, ptz, nx, ny, nz);
                const double nd = nx * r.dx + ny * r.dy + nz * r.dz;
                const Shading sh = shading_flags<kFresnel>(m, sig, nd);
                if (!sh.diffuse && !sh.specular) {
                    ends = true;
                    end_obj = h.obj;
                } else {
                    shade = true;
                    if (sh.specular) {                                      // raytrace.rs:58-64 / 159-164
                        if (nd > 0.0) { nx = -nx; ny = -ny; nz = -nz; }
                        rr = reflect_ray(r, ptx, pty, ptz, nx, ny, nz);
                        nsig = (sh.f * sig) * m.ks_sig;
                        refl = true;
                    }
                }
            }
        }
    }
    if (ends) {
        if constexpr (kCam) {                              // no levels: the final pixel now
            if (b.compose) stn(&b.pmap()[p], kPixAmbient | static_cast<uint32_t>(end_obj));
            else write_pixel(fp, p % fp.tile_w, fp.row0 + p / fp.tile_w, average_samples(end_colour(sc, end_obj), fp.spp));
        } else {
            set_terminal(b, p, end_colour(sc, end_obj), k);
        }
    }
    if constexpr (kCam) {
        if (b.mark && live) stn(&b.cmark()[p], static_cast<uint8_t>(shade ? 1 : 0));
    }
    const uint32_t slot = lds_append(&counts[0], shade);
    const uint32_t chain = kCam ? static_cast<uint32_t>(obase) + slot : p;   // (slot valid when shade)
    if (kCam && shade && b.compose) stn(&b.pmap()[p], chain);
    if (shade) {
        const size_t at = rbase + slot;
        stn(&b.rf(0)[at], ptx); stn(&b.rf(1)[at], pty); stn(&b.rf(2)[at], ptz);
        stn(&b.rf(3)[at], r.dx); stn(&b.rf(4)[at], r.dy); stn(&b.rf(5)[at], r.dz);
        stn(&b.rf(6)[at], sig);
        stn(&b.ru(0)[at], static_cast<uint32_t>(h.obj));
        stn(&b.ru(1)[at], static_cast<uint32_t>(h.prim));
        stn(&b.ru(2)[at], chain);
        stn(&b.ru(3)[at], 0u);
        if constexpr (kCam) {
            stn(&b.cpix()[chain], p);
            b.nlev()[chain] = kNlevRunning;                   // set_terminal gives the level count
        }
    }
    const uint32_t rslot = lds_append(&counts[1], refl);
    if (refl) {
        const int qn = (k + 1) & 1;
        const size_t at = obase + rslot;
        stn(&b.qf(qn, 0)[at], rr.ox); stn(&b.qf(qn, 1)[at], rr.oy); stn(&b.qf(qn, 2)[at], rr.oz);
        stn(&b.qf(qn, 3)[at], rr.dx); stn(&b.qf(qn, 4)[at], rr.dy); stn(&b.qf(qn, 5)[at], rr.dz);
        stn(&b.qf(qn, 6)[at], nsig);
        stn(&b.qpix(qn)[at], chain);
    }
}

// Scene::intersect for every ray of Q_k (generation 0: the camera rays of the
// chunk, computed here).  Outcomes that end the chain without lighting are
// resolved on the spot (miss -> background; depth cut-off or insignificant
// surface -> ambient, raytrace.rs:32-35); the rest become shade records of
// generation k in this workgroup's region, and a specular hit also appends
// its reflection ray (raytrace.rs:58-64) to Q_{k+1} right here: the next
// generation depends only on the hit, never on the shadow rays or the Phong
// sum, so those run on the other stream, off the critical path.
template <int kSrc, bool kCam, bool kCount, bool kFresnel>
__global__ __launch_bounds__(kWfThreads, Src<kSrc>::waves) void wf_nearest(DevScene sc, FrameParams fp, WfBufs b, int k) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
#ifndef RT_NEAR_PRIO
#define RT_NEAR_PRIO 2
#endif
    // the nearest-hit chain is the frame's critical path: its waves win issue
    // arbitration over the shadow / shading waves sharing a SIMD
    if (RT_NEAR_PRIO) __builtin_amdgcn_s_setprio(RT_NEAR_PRIO);
    [[maybe_unused]] unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0, acc[6] = {0, 0, 0, 0, 0, 0};
    RT_STAMP_AT(st0);
    const QueueLds ql = queue_lds(lds + staged_bytes<kSrc>(sc), b.G);
    if (threadIdx.x < kQueueCounters) ql.count[threadIdx.x] = 0;
    uint32_t n;
    if constexpr (kCam) {
        n = b.slots;
    } else {
        region_scan(b.rq() + k * b.G, b.G, ql.scan, ql.wave);
        n = ql.scan[b.G];
    }
    if (!wg_has_work(b, n)) {                  // nothing dealt here: publish empty regions, free the CU
        if (threadIdx.x == 0) {
            b.rs()[k * b.G + blockIdx.x] = 0;
            b.rq()[(k + 1) * b.G + blockIdx.x] = 0;
        }
        return;
    }
    const BvhView v = stage_lds<kSrc, true>(sc, lds);
    __syncthreads();                                       // publishes the LDS staging and counters
    RT_STAMP_AT(st1);
    acc[0] = st1 - st0;
    Work w;
    const size_t obase = static_cast<size_t>(blockIdx.x) * b.R;
    const size_t rbase = static_cast<size_t>(k) * b.qcap + obase;
    RT_FOR_CHUNKS(b, n, j) {
        RT_STAMP_AT(st0);
        [[maybe_unused]] const uint32_t visits0 = w.boxes;
        Ray r{};
        double sig = 0.0;
        uint32_t p = 0;
        Hit h{};
        bool live = false;
        if (j < n) {
            if constexpr (kCam) {
                uint32_t lx, ly;
                if (slot_pixel(b, fp, j, lx, ly)) {
                    r = camera_ray(sc, fp, lx, fp.row0 + ly);
                    sig = 1.0;                              // raytrace.rs:273 via main.rs:54
                    p = ly * fp.tile_w + lx;
                    live = true;
                }
            } else {
                const size_t at = region_entry(ql.scan, b.G, b.R, j);
                r = load_ray(b, k & 1, at);
                sig = ldn_if<kNtQ>(&b.qf(k & 1, 6)[at]);
                p = ldn_if<kNtQ>(&b.qpix(k & 1)[at]);
                live = true;
            }
        }
        RT_STAMP_AT(st1);
        if (live) h = nearest_any<kSrc, kCount>(sc, v, r, &w);
        RT_STAMP_AT(st2);
        finish_nearest<kCam, kFresnel>(sc, fp, b, v.sph, k, live, r, sig, p, h, ql.count, obase, rbase);
        RT_STAMP_AT(st3);
#if RT_STAMP
        acc[1] += st1 - st0; acc[2] += st2 - st1; acc[3] += st3 - st2; acc[4] += 1;
        if constexpr (kCount) {
            unsigned long long mx = (w.boxes - visits0) / 2, sm = mx;
            for (int off = 32; off > 0; off >>= 1) {
                mx = max(mx, static_cast<unsigned long long>(__shfl_xor(mx, off, 64)));
                sm += __shfl_xor(sm, off, 64);
            }
            if ((threadIdx.x & 63) == 0) { atomicAdd(&g_stamp[k][6], mx); atomicAdd(&g_stamp[k][7], sm); }
        }
#endif
    }
#if RT_STAMP
    for (int q = 0; q < 3; ++q)               // the wave's time in each loop = its longest-running lane's
        for (int off = 32; off > 0; off >>= 1)
            w.cyc[q] = max(w.cyc[q], static_cast<unsigned long long>(__shfl_xor(w.cyc[q], off, 64)));
    if ((threadIdx.x & 63) == 0) {
        for (int q = 0; q < 5; ++q) atomicAdd(&g_stamp[k][q], acc[q]);
        atomicAdd(&g_stamp[k][5], 1ull);
        for (int q = 0; q < 3; ++q) atomicAdd(&g_stamp[k][8 + q], w.cyc[q]);
        atomicMax(&g_stamp2[k][0], acc[2]);
    }
    for (int q = 0; q < 3; ++q) {
        unsigned long long ws = w.wsteps[q];
        for (int off = 32; off > 0; off >>= 1) ws += __shfl_xor(ws, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_stamp2[k][1 + q], ws);
    }
#endif
    __syncthreads();
    if (threadIdx.x == 0) {
        b.rs()[k * b.G + blockIdx.x] = ql.count[0];
        b.rq()[(k + 1) * b.G + blockIdx.x] = ql.count[1];
    }
    flush_work<kCount>(b, 2, w);
}

// A shade record's fields (loaded ahead of its shading by wf_shade).
struct ShadeIn {
    double ptx, pty, ptz, dx, dy, dz, sig;
    int32_t obj, prim;
    uint32_t c, mask;
};

__device__ __forceinline__ ShadeIn shade_load(const WfBufs& b, size_t at, bool mask) {
    ShadeIn in;
    in.ptx = ldn_if<2>(&b.rf(0)[at]); in.pty = ldn_if<2>(&b.rf(1)[at]); in.ptz = ldn_if<2>(&b.rf(2)[at]);
    in.dx = ldn_if<2>(&b.rf(3)[at]); in.dy = ldn_if<2>(&b.rf(4)[at]); in.dz = ldn_if<2>(&b.rf(5)[at]);
    in.sig = ldn_if<2>(&b.rf(6)[at]);
    in.obj = static_cast<int32_t>(ldn_if<2>(&b.ru(0)[at]));
    in.prim = static_cast<int32_t>(ldn_if<2>(&b.ru(1)[at]));
    in.c = ldn_if<2>(&b.ru(2)[at]);                         // the record's chain
    in.mask = mask ? b.ru(3)[at] : 0u;
    return in;
}

// What a shading leaves for the fused tail: the local colour, whether the hit
// reflects, its Schlick factor and the normal turned toward the ray.
struct ShadeOut {
    Col res;
    bool specular;
    double f, nx, ny, nz;
};

// The Phong sum of one shade record of generation k (raytrace.rs:31-56) with
// the shadow mask of its lights (bit l set: light l shadowed): a specular hit
// pushes the level's local colour (its reflection ray was already queued by
// wf_nearest); any other hit ends the chain with it.  kTerm = false (the fused
// tail): a non-specular hit's colour is returned for the caller's in-register
// fold instead of being written as the chain's terminal.
template <bool kFresnel, bool kTerm = true>
__device__ __forceinline__ ShadeOut shade_compute(const DevScene& sc, const WfBufs& b, int k, const ShadeIn& in) {
    const double ptx = in.ptx, pty = in.pty, ptz = in.ptz, dx = in.dx, dy = in.dy, dz = in.dz, sig = in.sig;
    const int32_t obj = in.obj;
    const uint32_t c = in.c, mask = in.mask;
    const DevMaterial& m = sc.mats[obj];
    Col res{m.amb[0], m.amb[1], m.amb[2]};                               // raytrace.rs:32
    double nx, ny, nz;
    hit_normal(sc, sc.spheres, in.prim, ptx, pty, ptz, nx, ny, nz);
    const double nd = nx * dx + ny * dy + nz * dz;
    const Shading sh = shading_flags<kFresnel>(m, sig, nd);
    const bool diffuse = sh.diffuse, specular = sh.specular;
    if (nd > 0.0) { nx = -nx; ny = -ny; nz = -nz; }
    for (int l = 0; l < sc.n_lights; ++l) {
        if ((mask >> l) & 1u) continue;                                  // shadowed (raytrace.rs:42-49)
        const DevLight& L = sc.lights[l];
        double lx, ly, lz, r2;
        light_dir(L, ptx, pty, ptz, lx, ly, lz, r2);
        add_light(res, m, L, diffuse, specular, sh.f, lx, ly, lz, nx, ny, nz, dx, dy, dz);
    }
    if (specular) {
        const size_t st = static_cast<size_t>(k) * b.capa + c;
        stn(&b.lf(0)[st], res.r); stn(&b.lf(1)[st], res.g); stn(&b.lf(2)[st], res.b);
        stn(&b.lobj()[st], obj);
        if (kFresnel && m.kind == kMatFresnel) stn(&b.lf(3)[st], sh.f);
    } else if (kTerm) {
        set_terminal(b, c, res, k);
    }
    return ShadeOut{res, specular, sh.f, nx, ny, nz};
}

// The shadow queries of every shade record of generation k (raytrace.rs:39-49):
// one work-item per (record, light) pair -- the lights of one hit are
// independent queries -- setting bit l of the record's occlusion mask.
template <int kSrc, bool kCount>
__global__ __launch_bounds__(kWfThreads, Src<kSrc>::waves) void wf_occlusion(DevScene sc, FrameParams fp, WfBufs b, int k) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const QueueLds ql = queue_lds(lds + staged_bytes<kSrc>(sc), b.G);
    region_scan(b.rs() + k * b.G, b.G, ql.scan, ql.wave);
    const uint32_t L = static_cast<uint32_t>(sc.n_lights);
    const uint32_t nrec = ql.scan[b.G], n = nrec * L;
    if (!wg_has_work(b, n)) return;
    const BvhView v = stage_lds<kSrc>(sc, lds);
    __syncthreads();
    Work w;
    const size_t rk = static_cast<size_t>(k) * b.qcap;
    // light-major: a wave traces 64 consecutive records toward ONE light (coherent).
    // Software pipelined: the next chunk's shade points are loaded (HBM) before this
    // chunk's queries run, so their latency hides behind the list walks.
    const uint32_t W = b.G * (kWfThreads / 64), lane = threadIdx.x & 63u;
    auto item_at = [&](uint32_t qi, uint32_t& l) {
        l = qi / nrec;
        return rk + region_entry(ql.scan, b.G, b.R, qi - l * nrec);
    };
    uint32_t rc = wave_slot(b, n), lc = 0;
    size_t atc = 0;
    double pc[3] = {0.0, 0.0, 0.0};
    int32_t hc = -1;
    if (static_cast<uint64_t>(rc) * 64u + lane < n) {
        atc = item_at(rc * 64u + lane, lc);
        pc[0] = ldn_if<3>(&b.rf(0)[atc]); pc[1] = ldn_if<3>(&b.rf(1)[atc]); pc[2] = ldn_if<3>(&b.rf(2)[atc]);
        hc = static_cast<int32_t>(b.ru(1)[atc]);
    }
    for (; static_cast<uint64_t>(rc) * 64u < n; rc += W) {
        const uint64_t qn = static_cast<uint64_t>(rc + W) * 64u + lane;
        uint32_t ln = 0;
        size_t atn = 0;
        double pn[3] = {0.0, 0.0, 0.0};
        int32_t hn = -1;
        if (qn < n) {
            atn = item_at(static_cast<uint32_t>(qn), ln);
            pn[0] = ldn_if<3>(&b.rf(0)[atn]); pn[1] = ldn_if<3>(&b.rf(1)[atn]); pn[2] = ldn_if<3>(&b.rf(2)[atn]);
            hn = static_cast<int32_t>(b.ru(1)[atn]);
        }
        const uint32_t qi = rc * 64u + lane;
        const uint32_t l = lc;
        const size_t at = atc;
        const double ptx = pc[0], pty = pc[1], ptz = pc[2];
        const int32_t hint = hc;
        lc = ln; atc = atn; pc[0] = pn[0]; pc[1] = pn[1]; pc[2] = pn[2]; hc = hn;
        if (qi >= n) continue;
        double lx, ly, lz, r2;
        const bool has_range = light_dir(sc.lights[l], ptx, pty, ptz, lx, ly, lz, r2);
        const Ray sray{ptx + lx * kEps, pty + ly * kEps, ptz + lz * kEps, lx, ly, lz};
        // the sphere the point lies on is tested first (it shadows every light behind its surface)
        bool occluded;
        if constexpr (Src<kSrc>::grid)          // the host checked: every light has a grid
            occluded = occluded_lgrid<kCount>(sc, v, sc.lgrid[l], sray, r2, ptx, pty, ptz, hint, &w);
        else
            occluded = has_range && sc.lgrid && sc.lgrid[l].R > 0
                           ? occluded_lgrid<kCount>(sc, v, sc.lgrid[l], sray, r2, ptx, pty, ptz, hint, &w)
                           : occluded_any<kSrc, kCount>(sc, v, sray, has_range, r2, hint, &w);
        if (occluded) atomicOr(&b.ru(3)[at], 1u << l);
    }
    flush_work<kCount>(b, 4, w);
}

// The Phong sum of every shade record of generation k.
template <bool kFresnel>
__global__ __launch_bounds__(kWfThreads, RT_SHADE_WAVES) void wf_shade(DevScene sc, FrameParams fp, WfBufs b, int k) {
    __shared__ uint32_t s_scan[kMaxRegions + 1];
    __shared__ uint32_t s_wave[kWfThreads / 64];
    region_scan(b.rs() + k * b.G, b.G, s_scan, s_wave);
    const uint32_t n = s_scan[b.G];
    const size_t rk = static_cast<size_t>(k) * b.qcap;
    // software pipelined: the next chunk's records are loaded (HBM) before this chunk is
    // shaded, so at the kernel's 4 waves per SIMD their latency hides behind the f64 math
    const uint32_t W = gridDim.x * (kWfThreads / 64), lane = threadIdx.x & 63u;
    const bool lit = sc.n_lights > 0;
    uint32_t rc = wave_slot(b, n);
    ShadeIn cur{};
    bool have = false;
    if (static_cast<uint64_t>(rc) * 64u + lane < n) {
        cur = shade_load(b, rk + region_entry(s_scan, b.G, b.R, rc * 64u + lane), lit);
        have = true;
    }
    for (; static_cast<uint64_t>(rc) * 64u < n; rc += W) {
        const uint64_t jn = static_cast<uint64_t>(rc + W) * 64u + lane;
        ShadeIn nxt{};
        const bool have_n = jn < n;
        if (have_n) nxt = shade_load(b, rk + region_entry(s_scan, b.G, b.R, static_cast<uint32_t>(jn)), lit);
        if (have) shade_compute<kFresnel>(sc, b, k, cur);
        cur = nxt;
        have = have_n;
    }
}

// The shadow mask of a lit hit at (ptx, pty, ptz) on sphere `prim` through the
// light-view grids (raytrace.rs:39-49; the host checked every light has one):
// the operations of wf_occlusion's grid source.
template <bool kCount>
__device__ __forceinline__ uint32_t grid_shadow_mask(const DevScene& sc, const BvhView& v, double ptx, double pty,
                                                     double ptz, int32_t prim, Work& wsh) {
    uint32_t mask = 0;
    for (int l = 0; l < sc.n_lights; ++l) {
        double lx, ly, lz, r2;
        (void)light_dir(sc.lights[l], ptx, pty, ptz, lx, ly, lz, r2);
        const Ray sray{ptx + lx * kEps, pty + ly * kEps, ptz + lz * kEps, lx, ly, lz};
        if (occluded_lgrid<kCount>(sc, v, sc.lgrid[l], sray, r2, ptx, pty, ptz, prim, &wsh)) mask |= 1u << l;
    }
    return mask;
}

// One chain of the fused tail from its shade record of generation T-1 on: the
// record's shadows and shading (wf_occlusion + wf_shade), then generation by
// generation what wf_nearest (finish_nearest), wf_occlusion and wf_shade do to
// it, in registers -- the same operations on the same operands, so the levels
// it writes are the per-generation kernels' bits.  Returns the chain's
// terminal colour and sets nlev (the generation it ended in) instead of writing
// them: the caller folds the chain right away.  cnt[0][k] / cnt[1][k]: this
// workgroup's shade records of generation k / rays queued for generation k.
template <bool kFresnel, bool kCount>
__device__ __forceinline__ Col tail_chain(const DevScene& sc, const FrameParams& fp, const WfBufs& b, const BvhView& v,
                                          int k, ShadeIn in, int& nlev, uint32_t (*cnt)[kMaxGenerations], Work& wn,
                                          Work& wsh) {
    const int k0 = k;
    for (;;) {
        in.mask = grid_shadow_mask<kCount>(sc, v, in.ptx, in.pty, in.ptz, in.prim, wsh);
        const ShadeOut so = shade_compute<kFresnel, false>(sc, b, k, in);        // level k if specular
        if (!so.specular) { nlev = k; return so.res; }
        const Ray r = reflect_ray(Ray{in.ptx, in.pty, in.ptz, in.dx, in.dy, in.dz}, in.ptx, in.pty, in.ptz, so.nx, so.ny,
                                  so.nz);                                   // raytrace.rs:58-64
        const double sig = (so.f * in.sig) * sc.mats[in.obj].ks_sig;
        ++k;
        if (k > k0 + 1) atomicAdd(&cnt[1][k], 1u);                         // (Q_T was counted by wf_nearest)
        const Hit h = nearest_any<kSrcBvhL8C, kCount>(sc, v, r, &wn);
        nlev = k;
        if (h.obj == INT32_MAX) return end_colour(sc, INT32_MAX);          // raytrace.rs:265, 228-232
        const DevMaterial& m = sc.mats[h.obj];
        if (static_cast<uint32_t>(k) > fp.max_depth) return end_colour(sc, h.obj);    // raytrace.rs:33
        in.ptx = r.ox + r.dx * h.t; in.pty = r.oy + r.dy * h.t; in.ptz = r.oz + r.dz * h.t;   // ray.cast(t)
        double nx, ny, nz;
        hit_normal(sc, v.sph, h.prim, in.ptx, in.pty, in.ptz, nx, ny, nz);
        const Shading sh = shading_flags<kFresnel>(m, sig, nx * r.dx + ny * r.dy + nz * r.dz);
        if (!sh.diffuse && !sh.specular) return end_colour(sc, h.obj);
        atomicAdd(&cnt[0][k], 1u);
        in.dx = r.dx; in.dy = r.dy; in.dz = r.dz;
        in.sig = sig;
        in.obj = h.obj;
        in.prim = h.prim;
    }
}
// The fold factor of a level is the specular colour of its object times, for
// FresnelMaterial, the level's Schlick factor (raytrace.rs:63 / 163).  The chain is folded inner-first exactly as the
// recursion returns (acc = res_k + ks_k * acc); the loads of four levels are
// issued together so a pixel costs about two memory round trips per four
// levels instead of two per level.
template <bool kFresnel>
__device__ __forceinline__ Col fold_levels(const DevScene& sc, const WfBufs& b, uint32_t p, int nlev, Col acc) {
    constexpr int U = RT_FOLD_UNROLL;
    for (int k = nlev - 1; k >= 0; k -= U) {
        double sr[U], sg[U], sb[U];
        int32_t ob[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k - u >= 0) {
                const size_t at = static_cast<size_t>(k - u) * b.capa + p;
                ob[u] = ldn_if<kNtFold>(&b.lobj()[at]);
                sr[u] = ldn_if<kNtFold>(&b.lf(0)[at]); sg[u] = ldn_if<kNtFold>(&b.lf(1)[at]); sb[u] = ldn_if<kNtFold>(&b.lf(2)[at]);
            }
        }
        double kr[U], kg[U], kb[U], kf[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k - u >= 0) {
                const DevMaterial& m = sc.mats[ob[u]];
                kr[u] = m.ks[0]; kg[u] = m.ks[1]; kb[u] = m.ks[2];
                kf[u] = kFresnel && m.kind == kMatFresnel ? ldn_if<kNtFold>(&b.lf(3)[static_cast<size_t>(k - u) * b.capa + p]) : 1.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k - u >= 0) {                  // res + (ks * child) * f, f = 1 for Phong (raytrace.rs:63 / 163)
                acc.r = sr[u] + (kr[u] * acc.r) * kf[u];
                acc.g = sg[u] + (kg[u] * acc.g) * kf[u];
                acc.b = sb[u] + (kb[u] * acc.b) * kf[u];
            }
        }
    }
    return acc;
}

template <bool kFresnel>
__device__ __forceinline__ Col fold_pixel(const DevScene& sc, const WfBufs& b, uint32_t p, uint8_t nlev) {   // p: the chain
    const Col acc{ldn_if<kNtFold>(&b.term(0)[p]), ldn_if<kNtFold>(&b.term(1)[p]), ldn_if<kNtFold>(&b.term(2)[p])};
    return fold_levels<kFresnel>(sc, b, p, nlev, acc);
}

// The fused tail (WfStreams::tail_fuse = T): for a small chunk (one rank's
// share of a frame), whose late generations are a chain of latency-bound
// launches, one launch takes every chain still running at generation T-1 from
// its shade record of T-1 through all its remaining bounces (tail_chain), one
// chain per work-item, and folds it onto its levels (fold_levels, as wf_fold)
// and writes its pixel: instead of a nearest-hit launch per generation >= T
// with its shadow and shading launches, and the frame-end fold.  The launch
// waits for the B streams (the levels of generations <= T-2 are written); the
// chains that ended by generation T-1 are folded meanwhile on a B stream
// (wf_fold over nlev <= T-1; the tail's chains keep nlev = kNlevRunning).  It
// lasts about as long as the slowest chain's remaining bounces, not the sum
// over generations of each generation's slowest walk plus a launch each.
// Needs the src-9 tree (whole tree + spheres in LDS) and a light-view grid for
// every light.  Chains in contiguous runs of cw per wave (tuning tail_width;
// auto: spread over about half of the waves; 48 per wave beat 16 / 24 / 32 /
// 64 on one rank's share of an 8-way C3 frame: the slowest chain of a wave
// against the lanes its finished chains leave idle), contiguous so that the
// record loads and level stores stay coalesced.  gridDim.x workgroups, all
// resident; workgroup w publishes its counts in region w and zeros in the
// other regions r = w (mod gridDim.x) of every generation >= T.
template <bool kFresnel, bool kCount>
__global__ __launch_bounds__(kWfThreads, 4) void wf_tail(DevScene sc, FrameParams fp, WfBufs b, int T, int W) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint32_t s_cnt[2][kMaxGenerations];
    __shared__ double s_srgb[255];
    const QueueLds ql = queue_lds(lds + staged_bytes<kSrcBvhL8C>(sc), b.G);
    for (int i = threadIdx.x; i < 2 * kMaxGenerations; i += kWfThreads) (&s_cnt[0][0])[i] = 0u;
    for (int i = threadIdx.x; i < 255; i += kWfThreads) s_srgb[i] = c_srgb_avg[i];
    region_scan(b.rs() + (T - 1) * b.G, b.G, ql.scan, ql.wave);   // generation T-1's records; ends with a barrier
    const uint32_t n = ql.scan[b.G];
    const int gens = static_cast<int>(fp.max_depth) + 2;
    const uint32_t nw = gridDim.x * (kWfThreads / 64);
    const uint32_t lane = threadIdx.x & 63u, slot = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const uint32_t cw = W > 0 ? static_cast<uint32_t>(W) : max(1u, min(64u, (2u * n + nw - 1) / nw));
    Work wn, wsh;
    const BvhView v = stage_lds<kSrcBvhL8C, true>(sc, lds);
    __syncthreads();
    const size_t rk = static_cast<size_t>(T - 1) * b.qcap;
    for (uint64_t base = static_cast<uint64_t>(slot) * cw; base < n; base += static_cast<uint64_t>(nw) * cw) {
        const uint64_t j = base + lane;
        if (lane >= cw || j >= n) continue;
        const size_t at = rk + region_entry(ql.scan, b.G, b.R, static_cast<uint32_t>(j));
        const ShadeIn in = shade_load(b, at, false);
        int nlev = 0;
        const Col term = tail_chain<kFresnel, kCount>(sc, fp, b, v, T - 1, in, nlev, s_cnt, wn, wsh);
        const Col res = average_samples(fold_levels<kFresnel>(sc, b, in.c, nlev, term), fp.spp);
        emit_chain(fp, b, in.c, b.compose ? 0u : b.cpix()[in.c], res, s_srgb);
    }
    __syncthreads();
    for (uint32_t rg = blockIdx.x; rg < b.G; rg += gridDim.x) {
        const bool own = rg == blockIdx.x;
        for (int k = T + static_cast<int>(threadIdx.x); k < gens; k += kWfThreads) {
            b.rs()[k * b.G + rg] = own ? s_cnt[0][k] : 0u;
            b.rq()[(k + 1) * b.G + rg] = own ? s_cnt[1][k + 1] : 0u;
        }
    }
    flush_work<kCount>(b, 2, wn);
    flush_work<kCount>(b, 4, wsh);
}

// One chain per work-item: the chains of the chunk are generation 0's shade
// records (chain c = record entry c), dealt densely over G workgroups through
// the region scan of generation 0's record counts, 64 consecutive chains to a
// wave (so levels and terminals are read in chain order, coalesced).  The
// launch is G workgroups whatever the queue capacity: one workgroup per 256
// entries of capacity (the first design) dispatched tens of thousands of
// mostly empty workgroups, ~80 us of dispatch for one rank's share of an
// 8-way C3 frame.  Chain c folds its levels onto its terminal and writes
// pixel cpix[c].  The quantisation table is staged in LDS: the binary search
// indexes it with a different entry per lane, which from __constant__ memory
// costs nine dependent vector loads per channel.
// Only chains of lo <= nlev <= hi: with the fused tail, the chains that ended
// by generation T-1 fold on a B stream while the tail runs (every level and
// terminal they need is written by then); the tail folds its own.
// RT_FOLD_THREADS-thread workgroups (256: at the fold's ~96 VGPRs five of them,
// 20 waves, fit a CU where one 1024-thread workgroup leaves 4 wave slots idle),
// dealt block-major over (kWfThreads / RT_FOLD_THREADS) x G workgroups.
template <bool kFresnel>
__global__ __launch_bounds__(RT_FOLD_THREADS, RT_FOLD_WAVES) void wf_fold(DevScene sc, FrameParams fp, WfBufs b, uint32_t lo,
                                                                          uint32_t hi) {
    constexpr int kT = RT_FOLD_THREADS;
    __shared__ double s_srgb[255];
    __shared__ uint32_t s_scan[kMaxRegions + 1];
    __shared__ uint32_t s_wave[kT / 64];
    for (int i = threadIdx.x; i < 255; i += kT) s_srgb[i] = c_srgb_avg[i];
    region_scan<kT>(b.rs(), b.G, s_scan, s_wave);         // generation 0's records = the chains (also publishes s_srgb)
    const uint32_t n = s_scan[b.G];
    // software pipelined: the next chunk's chain header (level count, pixel, terminal) is
    // loaded before this chain's levels are folded, one dependent round trip less per chain
    const uint32_t W = gridDim.x * (kT / 64), lane = threadIdx.x & 63u;
    struct Head {
        uint32_t c, nlev, p;
        Col term;
    };
    auto head = [&](uint64_t j) {
        Head hd{0u, kNlevRunning, 0u, Col{0.0, 0.0, 0.0}};
        if (j < n) {
            hd.c = static_cast<uint32_t>(region_entry(s_scan, b.G, b.R, static_cast<uint32_t>(j)));
            hd.nlev = b.nlev()[hd.c];
            hd.p = b.compose ? 0u : b.cpix()[hd.c];
            hd.term = Col{ldn_if<kNtFold>(&b.term(0)[hd.c]), ldn_if<kNtFold>(&b.term(1)[hd.c]),
                          ldn_if<kNtFold>(&b.term(2)[hd.c])};
        }
        return hd;
    };
    uint32_t rc = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
    Head cur = head(static_cast<uint64_t>(rc) * 64u + lane);
    for (; static_cast<uint64_t>(rc) * 64u < n; rc += W) {
        const Head nxt = head(static_cast<uint64_t>(rc + W) * 64u + lane);
        if (cur.nlev >= lo && cur.nlev <= hi) {             // (kNlevRunning: not ended yet, or no chain)
            const Col res = average_samples(fold_levels<kFresnel>(sc, b, cur.c, static_cast<int>(cur.nlev), cur.term), fp.spp);
            emit_chain(fp, b, cur.c, cur.p, res, s_srgb);
        }
        cur = nxt;
    }
}

hipError_t launch_fold(const DevScene& sc, const FrameParams& fp, const WfBufs& b, hipStream_t s, LaunchMarks* m,
                       uint32_t lo, uint32_t hi) {
    hipError_t e;
    if (m && (e = m->begin(s)) != hipSuccess) return e;
    const dim3 grid(b.G * (kWfThreads / RT_FOLD_THREADS)), block(RT_FOLD_THREADS);
    if (sc.has_fresnel) hipLaunchKernelGGL((wf_fold<true>), grid, block, 0, s, sc, fp, b, lo, hi);
    else hipLaunchKernelGGL((wf_fold<false>), grid, block, 0, s, sc, fp, b, lo, hi);
    return m ? m->mark(s, kKfFold) : hipGetLastError();
}

// The frame of the chunk, row by row (WfBufs::compose): each wave writes 64
// consecutive pixels of one row -- their f32 RGB as 192 consecutive dwords and
// their sRGB BGR as 48 consecutive dwords (or bytes when the row pitch is not a
// multiple of 4), staged through LDS so every store instruction covers
// consecutive addresses -- from the pixel map (chain, background or ambient
// object) and the chains' colours in ccol.  The colours are the fold's /
// write_pixel's values: f32 of the averaged f64 colour and to_srgb of it.
constexpr int kComposeWaves = kWfThreads / 64;
__global__ __launch_bounds__(kWfThreads) void wf_compose(DevScene sc, FrameParams fp, WfBufs b) {
    __shared__ float s_rgb[kComposeWaves][192];
    __shared__ uint32_t s_bgr[kComposeWaves][48];
    __shared__ double s_srgb[255];
    for (int i = threadIdx.x; i < 255; i += kWfThreads) s_srgb[i] = c_srgb_avg[i];
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t segs = (fp.tile_w + 63u) / 64u;                    // 64-pixel segments per row
    const uint64_t total = static_cast<uint64_t>(segs) * fp.rows;
    const bool dw = ((fp.bgr_pitch | reinterpret_cast<uintptr_t>(fp.out_bgr)) & 3u) == 0;   // dword-aligned BGR rows
    for (uint64_t sg = static_cast<uint64_t>(blockIdx.x) * kComposeWaves + wave; sg < total;
         sg += static_cast<uint64_t>(gridDim.x) * kComposeWaves) {     // wave-uniform
        const uint32_t lrow = static_cast<uint32_t>(sg / segs), x0 = static_cast<uint32_t>(sg % segs) * 64u;
        const uint32_t nv = min(64u, fp.tile_w - x0);                 // pixels in this segment
        const uint32_t x = x0 + lane;
        float r = 0.0f, g = 0.0f, bl = 0.0f;
        uint32_t q = 0;
        if (lane < nv) {
            const uint32_t code = ldn(&b.pmap()[static_cast<size_t>(lrow) * fp.tile_w + x]);
            if (code == kPixBackground) {
                r = fp.bg_rgb[0]; g = fp.bg_rgb[1]; bl = fp.bg_rgb[2];
                q = fp.bg_bgr[0] | (static_cast<uint32_t>(fp.bg_bgr[1]) << 8) | (static_cast<uint32_t>(fp.bg_bgr[2]) << 16);
            } else if (code & kPixAmbient) {                           // (rare) the ambient colour of a camera hit
                const Col res = average_samples(end_colour(sc, static_cast<int32_t>(code & ~kPixAmbient)), fp.spp);
                r = static_cast<float>(res.r); g = static_cast<float>(res.g); bl = static_cast<float>(res.b);
                q = static_cast<uint32_t>(to_srgb(res.b, s_srgb)) | (static_cast<uint32_t>(to_srgb(res.g, s_srgb)) << 8) |
                    (static_cast<uint32_t>(to_srgb(res.r, s_srgb)) << 16);
            } else {
                const U32x4 cc = ldn(reinterpret_cast<const U32x4*>(b.ccol()) + code);
                r = __uint_as_float(cc[0]); g = __uint_as_float(cc[1]); bl = __uint_as_float(cc[2]);
                q = cc[3];
            }
        }
        const uint32_t orow = fp.row0 + lrow;
        if (fp.out_rgb) {
            s_rgb[wave][3 * lane] = r; s_rgb[wave][3 * lane + 1] = g; s_rgb[wave][3 * lane + 2] = bl;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            float* dst = fp.out_rgb + (static_cast<size_t>(orow) * fp.tile_w + x0) * 3;
#pragma unroll
            for (uint32_t j = 0; j < 3; ++j) {
                const uint32_t i = lane + 64u * j;
                if (i < 3 * nv) dst[i] = s_rgb[wave][i];
            }
        }
        if (fp.out_bgr) {
            uint8_t* row = fp.out_bgr + static_cast<size_t>(orow) * fp.bgr_pitch;
            if (dw) {
                uint8_t* sb = reinterpret_cast<uint8_t*>(s_bgr[wave]);
                sb[3 * lane] = static_cast<uint8_t>(q); sb[3 * lane + 1] = static_cast<uint8_t>(q >> 8);
                sb[3 * lane + 2] = static_cast<uint8_t>(q >> 16);
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                // dwords [0, ceil(3 nv / 4)) of the segment; bytes past 3 nv are row padding (zero)
                const uint32_t nd = (3 * nv + 3) / 4;
                if (lane < nd) {
                    uint32_t v = s_bgr[wave][lane];
                    const uint32_t valid = 3 * nv - 4 * lane;                // bytes of this dword that are pixels
                    if (valid < 4) v &= (1u << (8 * valid)) - 1u;
                    reinterpret_cast<uint32_t*>(row + 3 * x0)[lane] = v;
                }
                __builtin_amdgcn_wave_barrier();
            } else if (lane < nv) {
                row[3 * x] = static_cast<uint8_t>(q); row[3 * x + 1] = static_cast<uint8_t>(q >> 8);
                row[3 * x + 2] = static_cast<uint8_t>(q >> 16);
            }
            if (x0 + nv == fp.tile_w)                                  // BMP row padding is zero (main.rs:42)
                for (uint32_t k = (dw ? (3 * fp.tile_w + 3) & ~3u : 3 * fp.tile_w) + lane; k < fp.bgr_pitch; k += 64)
                    row[k] = 0;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Scene::intersect calls of this chunk: every pixel's camera ray, every later
// queue entry, and one shadow query per light per shade record; plus the
// per-generation queue sizes.  One workgroup; atomics because chunks on
// different streams may finish together.
// Sparse host copies (rt_render, tuning sparse_out): after the
// camera pass every pixel that starts no chain is final, so the host copies the
// frame then, while the generations run; after the fold only the 16-pixel row
// segments that hold a chain pixel are packed, in row order, and copied.
// wf_chain_segs: one wave per chunk row: segbits (bit s of the row's words:
// segment s holds a chain pixel) and the row's segment count.
__global__ __launch_bounds__(256) void wf_chain_segs(FrameParams fp, WfBufs b, uint32_t* segbits, uint32_t* rowcnt) {
    const uint32_t row = (blockIdx.x * 256u + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
    if (row >= fp.rows) return;
    const uint32_t nseg = (fp.tile_w + kSegPx - 1) / kSegPx, words = (nseg + 31) / 32;
    const uint8_t* m = b.cmark() + static_cast<size_t>(row) * fp.tile_w;
    uint32_t cnt = 0;
    for (uint32_t s0 = 0; s0 < nseg; s0 += 64) {
        const uint32_t s = s0 + lane;
        bool any = false;
        if (s < nseg) {
            const uint32_t x1 = min(s * kSegPx + kSegPx, fp.tile_w);
            for (uint32_t x = s * kSegPx; x < x1; ++x) any |= m[x] != 0;
        }
        const unsigned long long bal = __ballot(any);
        cnt += static_cast<uint32_t>(__popcll(bal));
        if (lane == 0) segbits[static_cast<size_t>(row) * words + s0 / 32] = static_cast<uint32_t>(bal);
        if (lane == 32 && s0 / 32 + 1 < words) segbits[static_cast<size_t>(row) * words + s0 / 32 + 1] = static_cast<uint32_t>(bal >> 32);
    }
    if (lane == 0) rowcnt[row] = cnt;
}

// rowoff[r] = segments of rows < r (exclusive scan, rowoff[rows] = total); one workgroup.
__global__ __launch_bounds__(1024) void wf_row_scan(const uint32_t* rowcnt, uint32_t rows, uint32_t* rowoff) {
    __shared__ uint32_t s_wave[16];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t per = (rows + 1023u) / 1024u, a = t * per, e = min(a + per, rows);
    uint32_t sum = 0;
    for (uint32_t i = a; i < e; ++i) sum += rowcnt[i];
    uint32_t inc = sum;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off, 64);
        if (lane >= static_cast<uint32_t>(off)) inc += o;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t w = 0; w < wave; ++w) run += s_wave[w];
    for (uint32_t i = a; i < e; ++i) { rowoff[i] = run; run += rowcnt[i]; }
    if (t == 1023) rowoff[rows] = run;
}

// After the fold: the flagged segments' BGR (48 B) and f32 RGB (192 B) in row
// order, segment i of the frame at pk_bgr + 48 i / pk_rgb + 48 i; one wave per row.
__global__ __launch_bounds__(256) void wf_chain_pack(FrameParams fp, const uint32_t* segbits, const uint32_t* rowoff,
                                                     uint8_t* pk_bgr, float* pk_rgb) {
    const uint32_t row = (blockIdx.x * 256u + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
    if (row >= fp.rows) return;
    const uint32_t nseg = (fp.tile_w + kSegPx - 1) / kSegPx, words = (nseg + 31) / 32;
    const size_t frow = fp.row0 + row;
    uint32_t base = rowoff[row];
    for (uint32_t s0 = 0; s0 < nseg; s0 += 64) {
        const uint32_t s = s0 + lane;
        const uint32_t wd = s < nseg ? segbits[static_cast<size_t>(row) * words + s / 32] : 0u;
        const bool flag = (wd >> (s % 32)) & 1u;
        const unsigned long long bal = __ballot(flag);
        const uint32_t rank = base + static_cast<uint32_t>(__popcll(bal & ((1ull << lane) - 1ull)));
        base += static_cast<uint32_t>(__popcll(bal));
        if (!flag) continue;
        const uint32_t x0 = s * kSegPx, n = min(kSegPx, fp.tile_w - x0);
        if (fp.out_bgr) {
            const uint8_t* src = fp.out_bgr + frow * fp.bgr_pitch + 3u * x0;
            uint8_t* dst = pk_bgr + static_cast<size_t>(rank) * (3 * kSegPx);
            if (n == kSegPx && fp.bgr_pitch % 4u == 0) {
                static_assert(kSegPx % 4 == 0, "segments of whole dwords");
                for (uint32_t k = 0; k < 3 * kSegPx / 4; ++k)
                    reinterpret_cast<uint32_t*>(dst)[k] = reinterpret_cast<const uint32_t*>(src)[k];
            } else {
                for (uint32_t k = 0; k < 3 * n; ++k) dst[k] = src[k];
            }
        }
        if (fp.out_rgb) {
            const float* src = fp.out_rgb + (frow * fp.tile_w + x0) * 3;
            float* dst = pk_rgb + static_cast<size_t>(rank) * (3 * kSegPx);
            for (uint32_t k = 0; k < 3 * n; ++k) dst[k] = src[k];
        }
    }
}

__global__ __launch_bounds__(kWfThreads) void wf_tally(FrameParams fp, WfBufs b, int n_lights, int generations) {
    __shared__ unsigned long long s_sum[2 * kMaxGenerations];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // one wave per (generation, queue|records) pair, lanes striding the regions
    for (int item = wave; item < 2 * generations; item += kWfThreads / 64) {
        const int g = item >> 1;
        const uint32_t* src = (item & 1) ? b.rs() : b.rq();
        unsigned long long v = 0;
        if ((item & 1) || g > 0)
            for (uint32_t r = lane; r < b.G; r += 64) v += src[g * b.G + r];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) s_sum[(item & 1) ? kMaxGenerations + g : g] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long nearest = static_cast<unsigned long long>(fp.tile_w) * fp.rows, shadow = 0;
        for (int g = 0; g < generations; ++g) {
            nearest += s_sum[g];
            shadow += s_sum[kMaxGenerations + g] * n_lights;
        }
        atomicAdd(&b.totals[0], nearest * fp.spp);
        atomicAdd(&b.totals[1], shadow * fp.spp);
    }
    for (int g = threadIdx.x; g < generations; g += kWfThreads) {
        atomicAdd(&b.gen_totals[kCntQ + g], s_sum[g]);
        atomicAdd(&b.gen_totals[kCntS + g], s_sum[kMaxGenerations + g]);
    }
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

// The shadow queries and the shading of generation k on b stream sb (after its
// nearest-hit launch).
// Stream a waits for the work issued so far on the b streams of mask (those that are
// not stream a itself): through events, or on the device (ws.dj_flags: launch_signal on
// each, one launch_join on a).
hipError_t join_b(const WfStreams& ws, uint32_t mask) {
    hipError_t e;
    uint32_t m = 0;
    for (int i = 0; i < ws.nb; ++i)
        if (((mask >> i) & 1u) && ws.b[i] != ws.a) m |= 1u << i;
    if (!m) return hipSuccess;
    if (ws.dj_flags) {
        const uint64_t n = ++*ws.dj_next;
        for (int i = 0; i < ws.nb; ++i)
            if (((m >> i) & 1u) && (e = launch_signal(ws.dj_flags + i, n, ws.b[i])) != hipSuccess) return e;
        return launch_join(ws.dj_flags, m, n, ws.dj_err, ws.a);
    }
    for (int i = 0; i < ws.nb; ++i) {
        if (!((m >> i) & 1u)) continue;
        if ((e = hipEventRecord(ws.b_done[i], ws.b[i])) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(ws.a, ws.b_done[i], 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int kSrcO, bool kCount>
hipError_t launch_shading(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int k, const WfStreams& ws,
                          hipStream_t sb, LaunchMarks* mb) {
    const dim3 grid(b.G), block(kWfThreads);
    hipError_t e;
    if (sc.n_lights > 0) {
        if (mb && (e = mb->begin(sb)) != hipSuccess) return e;
#define RT_OCC(S) hipLaunchKernelGGL((wf_occlusion<S, kCount>), grid, block, staged_bytes<S>(sc) + queue_lds_bytes(b.G), \
                                     sb, sc, fp, b, k)
        if (ws.grid_occ == 1) RT_OCC(kSrcGridL);
        else if (ws.grid_occ == 2) RT_OCC(kSrcGridG);
        else RT_OCC(kSrcO);
#undef RT_OCC
        if (mb && (e = mb->mark(sb, kKfOcclusion)) != hipSuccess) return e;
    }
    if (mb && (e = mb->begin(sb)) != hipSuccess) return e;
    if (sc.has_fresnel) hipLaunchKernelGGL(wf_shade<true>, grid, block, 0, sb, sc, fp, b, k);
    else hipLaunchKernelGGL(wf_shade<false>, grid, block, 0, sb, sc, fp, b, k);
    return mb ? mb->mark(sb, kKfShade) : hipSuccess;
}

template <int kSrcN, int kSrcO, bool kCount>
hipError_t launch_generation(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int k, const WfStreams& ws) {
    const dim3 grid(b.G), block(kWfThreads);
    hipError_t e;
    if (ws.tail_fuse > 0 && k >= ws.tail_fuse) {      // the fused tail: every generation >= T in one launch
        if (k > ws.tail_fuse) return hipSuccess;
        // the tail folds its chains: the levels of generations <= T-2 (the B streams) must be written
        if ((e = join_b(ws, (1u << ws.nb) - 1u)) != hipSuccess) return e;
        // the chains that ended by generation T-1, folded on a B stream while the tail runs
        if (ws.b[0] != ws.a) {
            if ((e = hipEventRecord(ws.near_done[k], ws.a)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(ws.b[0], ws.near_done[k], 0)) != hipSuccess) return e;
        }
        if ((e = launch_fold(sc, fp, b, ws.b[0], ws.b[0] != ws.a ? ws.mb[0] : ws.ma, 0u, static_cast<uint32_t>(k - 1))) !=
            hipSuccess)
            return e;
        if (ws.ma && (e = ws.ma->begin(ws.a)) != hipSuccess) return e;
        const size_t lds_t = staged_bytes<kSrcBvhL8C>(sc) + queue_lds_bytes(b.G);
        if (sc.has_fresnel) hipLaunchKernelGGL((wf_tail<true, kCount>), dim3(ws.tail_wgs), block, lds_t, ws.a, sc, fp, b, k, ws.tail_width);
        else hipLaunchKernelGGL((wf_tail<false, kCount>), dim3(ws.tail_wgs), block, lds_t, ws.a, sc, fp, b, k, ws.tail_width);
        return ws.ma ? ws.ma->mark(ws.a, kKfTail) : hipGetLastError();
    }
    e = ws.ma ? ws.ma->begin(ws.a) : hipSuccess;
    if (e != hipSuccess) return e;
#define RT_NEAR(S, CAM, FR) hipLaunchKernelGGL((wf_nearest<S, CAM, kCount, FR>), grid, block, \
                                               staged_bytes<S>(sc) + queue_lds_bytes(b.G), ws.a, sc, fp, b, k)
    if (k == 0 && ws.cam == 3) {                 // the camera's view grid, spheres in LDS
        if (sc.has_fresnel) RT_NEAR(kSrcCamGridL, true, true); else RT_NEAR(kSrcCamGridL, true, false);
    } else if (k == 0 && ws.cam == 4) {          // ... spheres through L2
        if (sc.has_fresnel) RT_NEAR(kSrcCamGridG, true, true); else RT_NEAR(kSrcCamGridG, true, false);
    } else if (k == 0) {
        if (sc.has_fresnel) RT_NEAR(kSrcN, true, true); else RT_NEAR(kSrcN, true, false);
    } else {
        if (sc.has_fresnel) RT_NEAR(kSrcN, false, true); else RT_NEAR(kSrcN, false, false);
    }
#undef RT_NEAR
    e = ws.ma ? ws.ma->mark(ws.a, k == 0 ? kKfCamera : kKfNearest) : hipSuccess;
    if (e != hipSuccess) return e;
    if (static_cast<uint32_t>(k) > fp.max_depth) return hipSuccess;    // no shade records past the cut-off
    // the fused tail shades the records of generation T-1 itself
    if (ws.tail_fuse > 0 && k >= ws.tail_fuse - 1) return hipSuccess;
    // shadows and shading of generation k: on a b stream once nearest_k is done
    // (generations alternate over the b streams, so consecutive ones overlap too)
    const int bi = k % ws.nb;
    const hipStream_t sb = ws.b[bi];
    if (sb != ws.a) {
        if ((e = hipEventRecord(ws.near_done[k], ws.a)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(sb, ws.near_done[k], 0)) != hipSuccess) return e;
    }
    return launch_shading<kSrcO, kCount>(sc, fp, b, k, ws, sb, ws.mb[bi]);
}

// One chunk (fp.row0, fp.rows) through every generation.  src: the sphere
// source of the nearest-hit kernel (kSrc*), src_occ: of the shadow kernel;
// count: instrumented kernels; mark is recorded on stream a after generation
// mark_gen has been launched (chunk pipelining across lanes).  The nearest-hit
// chain runs on ws.a, the shadow + shading kernels of each generation on ws.b
// streams (each waiting for its generation's nearest-hit kernel); the fold
// waits for all of them.  Supported (src, src_occ) pairs: (0, 0), (1, 1),
// (2, 2), (7, 7), (7, 10), (9, 10), (2, 11), (5, 11), (6, 11), (8, 11), (25, 11),
// (26, 11); any other pair runs as (2, 11).
hipError_t launch_wavefront(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int src, int src_occ,
                            bool count, const WfStreams& ws, hipEvent_t mark, int mark_gen) {
    const int gens = static_cast<int>(fp.max_depth) + 2;          // depths 0 .. max_depth+1
    for (int k = 0; k < gens; ++k) {
        hipError_t e;
#define RT_GEN(N, O) e = (count ? launch_generation<N, O, true>(sc, fp, b, k, ws) \
                                : launch_generation<N, O, false>(sc, fp, b, k, ws))
        switch (src * 100 + src_occ) {
        case kSrcGlobal * 101: RT_GEN(kSrcGlobal, kSrcGlobal); break;
        case kSrcLds * 101: RT_GEN(kSrcLds, kSrcLds); break;
        case kSrcBvhG * 101: RT_GEN(kSrcBvhG, kSrcBvhG); break;
        case kSrcBvhL8 * 101: RT_GEN(kSrcBvhL8, kSrcBvhL8); break;
        case kSrcBvhL8 * 100 + kSrcBvh4L: RT_GEN(kSrcBvhL8, kSrcBvh4L); break;
        case kSrcBvhL8C * 100 + kSrcBvh4L: RT_GEN(kSrcBvhL8C, kSrcBvh4L); break;
        case kSrcBvhPH * 100 + kSrcBvh4G: RT_GEN(kSrcBvhPH, kSrcBvh4G); break;
        case kSrcBvhPHC * 100 + kSrcBvh4G: RT_GEN(kSrcBvhPHC, kSrcBvh4G); break;
        case kSrcBvhP * 100 + kSrcBvh4G: RT_GEN(kSrcBvhP, kSrcBvh4G); break;
        case kSrcQ4 * 100 + kSrcBvh4G: RT_GEN(kSrcQ4, kSrcBvh4G); break;
        case kSrcQ4P * 100 + kSrcBvh4G: RT_GEN(kSrcQ4P, kSrcBvh4G); break;
        default: RT_GEN(kSrcBvhG, kSrcBvh4G); break;
        }
#undef RT_GEN
        if (e != hipSuccess) return e;
        if (k == 0 && ws.sp_s) {               // every pixel without a chain is final now
            if ((e = hipEventRecord(ws.sp_cam, ws.a)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(ws.sp_s, ws.sp_cam, 0)) != hipSuccess) return e;
            if ((e = launch_chain_segs(fp, b, ws.sp_bits, ws.sp_cnt, ws.sp_off, ws.sp_s)) != hipSuccess) return e;
            if ((e = hipEventRecord(ws.sp_ready, ws.sp_s)) != hipSuccess) return e;
        }
        if (mark && k == mark_gen) {
            e = hipEventRecord(mark, ws.a);
            if (e != hipSuccess) return e;
        }
    }
    hipError_t e;
    // the tally reads only the queue sizes: on stream a while the b streams finish the last shading
    // (or later, when statistics are asked for: ws.lazy_tally)
    if (!ws.lazy_tally) {
        if (ws.ma && (e = ws.ma->begin(ws.a)) != hipSuccess) return e;
        hipLaunchKernelGGL(wf_tally, dim3(1), dim3(kWfThreads), 0, ws.a, fp, b, sc.n_lights, gens);
        if (ws.ma && (e = ws.ma->mark(ws.a, kKfTally)) != hipSuccess) return e;
    }
    // the b streams' work joins stream a (with the fused tail only b[0]'s early fold is left: the
    // tail's launch already waited for every b stream, and none has had work since)
    if ((e = join_b(ws, ws.tail_fuse > 0 ? 1u : (1u << ws.nb) - 1u)) != hipSuccess) return e;
    // the chains not folded yet (all of them without the fused tail, which folded every chain:
    // its own as it ended them, the others on a B stream)
    if (ws.tail_fuse == 0 && (e = launch_fold(sc, fp, b, ws.a, ws.ma, 0u, kNlevRunning - 1u)) != hipSuccess) return e;
    if (b.compose) {                         // the frame, row by row, once every chain has its colour
        if (ws.ma && (e = ws.ma->begin(ws.a)) != hipSuccess) return e;
        const uint64_t segs = static_cast<uint64_t>((fp.tile_w + 63u) / 64u) * fp.rows;
        const uint32_t wgs = static_cast<uint32_t>(std::min<uint64_t>(4u * b.G, (segs + kComposeWaves - 1) / kComposeWaves));
        hipLaunchKernelGGL(wf_compose, dim3(std::max(1u, wgs)), dim3(kWfThreads), 0, ws.a, sc, fp, b);
        if (ws.ma && (e = ws.ma->mark(ws.a, kKfCompose)) != hipSuccess) return e;
    }
    if (ws.sp_s) {                           // the chain pixels' segments, packed in row order
        if ((e = hipStreamWaitEvent(ws.a, ws.sp_ready, 0)) != hipSuccess) return e;
        if ((e = launch_chain_pack(fp, ws.sp_bits, ws.sp_off, ws.sp_bgr, ws.sp_rgb, ws.a)) != hipSuccess) return e;
    }
    // every row of the chunk is final now (the fold runs in chain order, not by rows)
    if (ws.fold_ev && (e = hipEventRecord(*ws.fold_ev, ws.a)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_tally(const FrameParams& fp, const WfBufs& b, int n_lights, int generations, hipStream_t s) {
    hipLaunchKernelGGL(wf_tally, dim3(1), dim3(kWfThreads), 0, s, fp, b, n_lights, generations);
    return hipGetLastError();
}

// Device-side join of b streams into stream a (WfStreams::dj_flags): a b stream
// ends its share with wf_signal (one work-item stores the join's number into
// the stream's flag word once the kernels before it on that stream are done:
// in-order stream), and stream a runs wf_join, one wave whose lane i polls
// flag i until it reaches the number.  Instead of an event record on the b
// stream and a barrier packet on stream a: the cross-queue event wait measured
// ~50 us between the b stream's last kernel and stream a's next one, a kernel
// boundary on one queue ~8 us.  Flags only grow (one number per join, from
// the host), so they need no reset.  A join that has waited kJoinTimeout
// (100 MHz ticks) gives up and sets the error word (a page-locked host word,
// reported by the next rt_render or rt_ctx_stats): the stream goes on rather
// than hang the device.
constexpr uint64_t kJoinTimeout = 200000000ull;      // 2 s
__global__ __launch_bounds__(64) void wf_signal(uint64_t* flag, uint64_t n) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(64) void wf_join(uint64_t* flags, uint32_t mask, uint64_t n, uint64_t* err) {
    const uint32_t i = threadIdx.x;
    if (i < kDjFlags && ((mask >> i) & 1u)) {
        const uint64_t t0 = wall_clock64();
        while (__hip_atomic_load(&flags[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < n) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > kJoinTimeout) {       // err: a page-locked host word the host reads directly
                __hip_atomic_store(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
    }
}

hipError_t launch_signal(uint64_t* flag, uint64_t n, hipStream_t s) {
    hipLaunchKernelGGL(wf_signal, dim3(1), dim3(64), 0, s, flag, n);
    return hipGetLastError();
}

hipError_t launch_join(uint64_t* flags, uint32_t mask, uint64_t n, uint64_t* err, hipStream_t s) {
    hipLaunchKernelGGL(wf_join, dim3(1), dim3(64), 0, s, flags, mask, n, err);
    return hipGetLastError();
}

hipError_t launch_chain_segs(const FrameParams& fp, const WfBufs& b, uint32_t* segbits, uint32_t* rowcnt, uint32_t* rowoff,
                             hipStream_t s) {
    const dim3 grid((fp.rows + 3u) / 4u);
    hipLaunchKernelGGL(wf_chain_segs, grid, dim3(256), 0, s, fp, b, segbits, rowcnt);
    hipLaunchKernelGGL(wf_row_scan, dim3(1), dim3(1024), 0, s, rowcnt, fp.rows, rowoff);
    return hipGetLastError();
}

hipError_t launch_chain_pack(const FrameParams& fp, const uint32_t* segbits, const uint32_t* rowoff, uint8_t* pk_bgr,
                             float* pk_rgb, hipStream_t s) {
    hipLaunchKernelGGL(wf_chain_pack, dim3((fp.rows + 3u) / 4u), dim3(256), 0, s, fp, segbits, rowoff, pk_bgr, pk_rgb);
    return hipGetLastError();
}

#if RT_STAMP
}  // namespace rtamd
extern "C" int rt_debug_stamps(unsigned long long* out, int n, int reset) {
    // out: 16 fields per generation
    static unsigned long long a[rtamd::kMaxGenerations][12], b[rtamd::kMaxGenerations][4];
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(a, HIP_SYMBOL(rtamd::g_stamp), sizeof a) != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(b, HIP_SYMBOL(rtamd::g_stamp2), sizeof b) != hipSuccess) return -3;
    for (int i = 0; i < n && i < 16 * rtamd::kMaxGenerations; ++i)
        out[i] = (i % 16) < 12 ? a[i / 16][i % 16] : b[i / 16][i % 16 - 12];
    if (reset) {
        static unsigned long long za[rtamd::kMaxGenerations][12], zb[rtamd::kMaxGenerations][4];
        if (hipMemcpyToSymbol(HIP_SYMBOL(rtamd::g_stamp), za, sizeof za) != hipSuccess) return -3;
        if (hipMemcpyToSymbol(HIP_SYMBOL(rtamd::g_stamp2), zb, sizeof zb) != hipSuccess) return -3;
    }
    return 0;
}
namespace rtamd {
#endif

// rt_ctx_reserve: one launch on a stream loads this file's code object (its first launch does)
// and has the runtime set up the stream's hardware queue, including the queue's scratch, which
// it sizes at the first launch that needs private memory: kWarmScratch bytes per lane, at
// least what any wavefront kernel spills or stacks (128-208 B).
constexpr uint32_t kWarmScratch = 256;
__global__ __launch_bounds__(kWfThreads) void wf_warm(uint32_t* sink, uint32_t salt) {
    volatile uint32_t priv[kWarmScratch / 4];       // volatile + a lane-dependent index: kept in scratch
    const uint32_t i = (threadIdx.x * 7u + salt) % (kWarmScratch / 4);
    priv[i] = salt;
    if (priv[(i + salt) % (kWarmScratch / 4)] == 0xfeedf00du && sink) sink[blockIdx.x] = salt;
}

hipError_t launch_warmup(uint32_t workgroups, hipStream_t s) {
    hipLaunchKernelGGL(wf_warm, dim3(std::max(1u, workgroups)), dim3(kWfThreads), 0, s, nullptr, 1u);
    return hipGetLastError();
}

// Diagnostic (rt_div_a2_check): the sphere test's division t = x / (2a) as
// sphere_t computes it (sphere_k's hoisted reciprocal finished by div_a2) and
// as the compiler's own f64 division, side by side.
__global__ __launch_bounds__(256) void div_a2_probe(const double* x, const double* a, uint32_t n, double* fast,
                                                    double* slow) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const SphK k = sphere_k(a[i]);
        fast[i] = div_a2(x[i], k);
        slow[i] = x[i] / (2.0 * a[i]);
    }
}

// Diagnostic (rt_sqrt_check): the sphere test's square root as sphere_roots computes it
// (sqrt_win) and as the compiler's own f64 sqrt, side by side.
__global__ __launch_bounds__(256) void sqrt_probe(const double* x, uint32_t n, double* fast, double* slow) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        fast[i] = sqrt_win(x[i]);
        slow[i] = sqrt(x[i]);
    }
}

hipError_t launch_sqrt_probe(const double* x, uint32_t n, double* fast, double* slow, hipStream_t s) {
    const uint32_t blocks = std::max(1u, std::min(4096u, (n + 255u) / 256u));
    hipLaunchKernelGGL(sqrt_probe, dim3(blocks), dim3(256), 0, s, x, n, fast, slow);
    return hipGetLastError();
}

hipError_t launch_div_a2_probe(const double* x, const double* a, uint32_t n, double* fast, double* slow, hipStream_t s) {
    const uint32_t blocks = std::max(1u, std::min(4096u, (n + 255u) / 256u));
    hipLaunchKernelGGL(div_a2_probe, dim3(blocks), dim3(256), 0, s, x, a, n, fast, slow);
    return hipGetLastError();
}

hipError_t upload_srgb_table(const double* avg255) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_srgb_avg), avg255, 255 * sizeof(double));
}

}  // namespace rtamd
