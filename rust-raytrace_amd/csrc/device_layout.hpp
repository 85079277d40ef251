// Device (HBM) layout of a flattened scene.  Shared by the host upload code
// and the HIP kernels.  All geometry stays f64: the reference computes in f64
// (types.rs:11-25) and the self-intersection offset 1e-5 (raytrace.rs:43,62)
// is below f32 resolution for |coordinates| >~ 5.
#pragma once

#include <cstdint>

namespace rtamd {

// One sphere = 32 B, read by every ray-sphere test (shapes.rs:60-65).  rr is
// radius*radius computed once on the host with the same f64 multiply the
// reference does per test, so it is bit-identical.
struct alignas(16) DevSphere {
    double cx, cy, cz, rr;
};

// Plane as in the file: normal NOT normalised (shapes.rs:100-112).
struct DevPlane {
    double px, py, pz, nx, ny, nz;
};

// Per OBJECT (indexed by file-order object id), only what shading reads.
constexpr int32_t kMatPhong = 0;      // DevMaterial::kind (= rt_material_kind)
constexpr int32_t kMatIndirect = 1;   // IndirectPhongMaterial (path kernel only)
constexpr int32_t kMatFresnel = 2;
constexpr int32_t kMatTransparent = 3;   // TransparentMaterial (path kernel only)

// What the fold and the significance tests read (ks, ks_sig, kind) shares the
// first 64-B line.
struct alignas(64) DevMaterial {
    double ks[3];
    double ks_sig;                  // Color::significance, color.rs:637-639
    int32_t kind;                   // rt_material_kind
    uint32_t samples;               // IndirectPhongMaterial::samples
    double kd_sig;
    double ior;
    double kd[3], amb[3];
    double exponent;
};

constexpr int32_t kLightArea = 2;     // DevLight::kind (= rt_light_kind)

struct DevLight {
    double v[9];                    // point: location; directional: direction; area: origin, side1, side2
    double color[3];
    int32_t kind;                   // rt_light_kind
    int32_t _pad;
};

// One BVH2 node: the boxes of BOTH children (one 64-B fetch decides both),
// f32, rounded outward and padded on the host (host_bvh.cpp).  Child pointer
// c >= 0: inner node c; c < 0: leaf with spheres [(~c) >> 3, +((~c) & 7) + 1).
struct alignas(16) DevBvhNode {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t c0, c1;
    int32_t _pad[2];
};
static_assert(sizeof(DevBvhNode) == 64, "BVH node is one 64-B line");

// The same node with IEEE binary16 bounds (host_bvh.cpp half_nodes): each f32
// bound rounded OUTWARD to a half (lo down, hi up), so every half box contains
// the f32 box and the culling argument of DESIGN.md §4 carries over.  32 B:
// twice the nodes of an LDS prefix and half the bytes per L2 fetch below it.
// Built only when every bound is finite and within the half range (+-65504).
struct alignas(16) DevBvhNodeH {
    uint16_t b[12];                 // lo0 xyz, hi0 xyz, lo1 xyz, hi1 xyz (binary16 bits)
    int32_t c0, c1;
};
static_assert(sizeof(DevBvhNodeH) == 32, "half BVH node is 32 B");

// 4-wide BVH, plane-major: node i's child boxes and pointers are 7 16-byte
// planes, plane k at index k * n_nodes + i (lo.x, hi.x, lo.y, hi.y, lo.z,
// hi.z of the 4 children, then the 4 child pointers).  A wave's lanes reading
// plane k of 16 different nodes hit 16 different LDS bank slots (an
// array-of-nodes layout would put them on 2).  Child pointers as in
// DevBvhNode; kBvh4Empty marks an unused slot.
struct alignas(16) DevBvh4Plane {
    union {
        float f[4];
        int32_t i[4];
    };
};
constexpr int kBvh4Planes = 7;
constexpr int32_t kBvh4Empty = INT32_MIN;

// The 4-wide tree with child boxes quantised to 8 bits per bound in a per-node
// frame (host_bvh.cpp quantize_bvh4): 48 B per node, so C4's whole tree (10k
// spheres, 1510 nodes) fits one nearest-hit workgroup's LDS share.  Per axis a
// the frame is a power-of-two step s_a = 2^(e_a - 127) and an origin m_a * s_a
// (m_a a signed 24-bit integer); child k's bounds are (m_a + lo_a[k]) * s_a and
// (m_a + hi_a[k]) * s_a, which are exact f32 values (|m_a| + 255 < 2^24, normal
// range), rounded OUTWARD from the child's f32 box on the host: every decoded
// box contains the binary tree's f32 box, so the slab test on it culls a subset
// of what the f32 test culls.  Child refs (u16):
// < 0x8000 an inner node; 0x8000 | off << 3 | (count - 1) a leaf of spheres
// [base + off, + count); kQ4Empty an unused slot.
struct alignas(16) DevQNode4 {
    int32_t frame[3];               // m_a (low 24 bits, signed) | e_a << 24
    uint32_t base;                  // first sphere (leaf order) of the node's leaf children
    uint32_t lo[3];                 // per axis: byte k = child k's lower bound
    uint32_t hi[3];                 // per axis: byte k = child k's upper bound
    uint16_t child[4];
};
static_assert(sizeof(DevQNode4) == 48, "quantised 4-wide node is 48 B");
constexpr uint16_t kQ4Empty = 0xFFFF;
constexpr uint16_t kQ4Leaf = 0x8000;
constexpr int kQ4Stack = 32;          // nearest_q4's stack entries per lane (host: bvh4_stack_need <= this)

// One skybox face (texture.rs:22-26): RGB8 rows top-down at DevScene::tex + off.
struct DevTexFace {
    uint32_t w, h;
    uint64_t off;
};

// Light-view grid of one point light (host_lightgrid.cpp): a cube map of R x R
// cells per face centred on the light.  A direction d (from the light) maps to
// face 2a + (d_a < 0) with a = argmax |d_i|, and to face coordinates
// u = d_b / |d_a|, v = d_c / |d_a| (b = a+1, c = a+2 mod 3), cell
// (floor((u+1)/2 R), floor((v+1)/2 R)).  Only the face's rectangle of non-empty
// cells is stored: its cell offsets start at lg_off[off_base[f]].
struct DevLightGrid {
    double lx, ly, lz;              // the light's location
    int32_t R;                      // cells per face side; 0 = no grid for this light
    uint32_t always_begin, always_end;   // lg_ent entries tested for every query (spheres at the light)
    int32_t fx0[6], fy0[6], fw[6], fh[6];
    uint32_t off_base[6];
};

// One list entry: a sphere (leaf-order index) and a lower bound on the distance
// from the light to its padded box (f32, rounded down).
struct DevLgEntry {
    int32_t sph;
    float near;
};

struct DevScene {
    const DevSphere* spheres;       // file order among spheres (or BVH order, see sphere_obj)
    const int32_t* sphere_obj;      // object id of each sphere (tie-break key, material index)
    const DevPlane* planes;
    const int32_t* plane_obj;
    const DevMaterial* mats;        // indexed by object id
    const DevLight* lights;
    const DevBvhNode* bvh;          // sphere BVH (spheres[] are in its leaf order)
    int32_t bvh_root;               // encoded child pointer of the root (see DevBvhNode)
    int32_t n_spheres, n_planes, n_lights, n_bvh;
    const DevBvh4Plane* bvh4;       // the same tree collapsed 4-wide (DevBvh4Plane)
    int32_t bvh4_root, n_bvh4;
    const DevBvhNodeH* bvh_h;       // the binary BVH with binary16 bounds (null: not representable)
    int32_t has_fresnel;            // some object uses FresnelMaterial
    int32_t pfx2;                   // prefix sources: nodes of the binary tree staged in LDS (set per render)
    int32_t needs_path;             // a class only the path kernel implements (IndirectPhong, Transparent,
                                    // AreaLight, DepthOfFieldCamera)
    int32_t skybox;                 // SkyboxBackground (raytrace.rs:234-256; path kernel only)
    const uint8_t* tex;             // skybox texels
    const double* srgb_values;      // color.rs SRGB_VALUES (Color::from_srgb, color.rs:611-613)
    DevTexFace faces[6];            // px, nx, py, ny, pz, nz
    int32_t cam_dof;                // DepthOfFieldCamera (camera.rs:83-123)
    uint32_t cam_samples;           // Camera::samples() (1 for the simple camera)
    double cam_focus, cam_aperture, cam_im_dist;   // DepthOfFieldCamera focus, aperture, im_dist (camera.rs:98)
    double cam_pos[3];
    double cam_m[9];                // row-major
    double bg[3];
    const DevLightGrid* lgrid;       // per light (null: no grids)
    const uint32_t* lg_off;
    const DevLgEntry* lg_ent;
    const DevLightGrid* cgrid;       // the camera's view grid (camera rays' nearest hit; null: none)
    const uint32_t* cg_off;
    const DevLgEntry* cg_ent;
    const DevQNode4* q4;             // the quantised 4-wide tree (null: not representable)
    int32_t n_q4;                    // its nodes (breadth-first; root = node 0)
    int32_t pfxq;                    // nodes [0, pfxq) staged in LDS by the quantised-tree source (set per render)
};

struct FrameParams {
    double hw, hh, scale;           // main.rs:39-41
    uint32_t x0, tile_w, y0, tile_h;
    uint32_t band, band_stride, band_phase;
    uint32_t max_depth, spp;
    uint32_t bgr_pitch;
    uint32_t row0, rows;            // this launch covers local rows [row0, row0 + rows) of the tile
    float* out_rgb;                 // tile_h * tile_w * 3, may be null
    uint8_t* out_bgr;               // tile_h * bgr_pitch, may be null
    unsigned long long* counters;   // [kCounterShards] rays, then [kCounterShards] shadow rays
    float bg_rgb[3];                // output of a pixel whose camera ray misses: the background
    uint8_t bg_bgr[3];              //   averaged over spp (main.rs:56), f32 and sRGB B,G,R (host-computed)
    int32_t jitter;                 // rt_jitter: 0 centre, 1 keyed random draws (path kernel)
    uint64_t seed;                  // keyed RNG seed (path kernel)
    const double* srgb;             // the 255 sRGB thresholds in HBM (path kernel stages them in LDS)
    uint32_t path_group;            // path kernel: lanes per pixel (power of two <= 64), sharing its AA samples
};



#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

// Recursion stack of the path kernel: one frame per depth 0..max_depth for
// every work-item of the (persistent) grid, SoA so a wave's lanes at the same
// depth touch consecutive 8-B words: f64 fields [level][kPathF][T], then the
// key [level][T], then i32 fields [level][kPathI][T].  A frame whose child in
// flight is its last one stores only the compact part (what folding the
// child's colour needs: colour so far and the two fold factors); a frame with
// more children to spawn (IndirectPhong samples > 1, Transparent reflection
// before refraction) also stores the extension and the path key.
constexpr int kPathCompact = 5;       // colour 3, fold factor, second fold factor (IndirectPhong specular)
constexpr int kPathF = kPathCompact + 14;   // + point 3, normal 3, direction 3, significance, Schlick f, aux 3
constexpr int kPathI = 3;             // object, child in flight, flags
struct PathStack {
    unsigned char* mem;
    uint32_t T;                       // work-items of the grid (stride of every field)
    uint32_t levels;
    RT_HD double* f(int level, int field) const {
        return reinterpret_cast<double*>(mem) + (static_cast<uint64_t>(level) * kPathF + field) * T;
    }
    RT_HD uint64_t* key(int level) const {
        return reinterpret_cast<uint64_t*>(mem) + static_cast<uint64_t>(levels) * kPathF * T + static_cast<uint64_t>(level) * T;
    }
    RT_HD int32_t* i(int level, int field) const {
        return reinterpret_cast<int32_t*>(reinterpret_cast<uint64_t*>(mem) + static_cast<uint64_t>(levels) * (kPathF + 1) * T) +
               (static_cast<uint64_t>(level) * kPathI + field) * T;
    }
    static uint64_t bytes(uint32_t T, uint32_t levels) {
        return static_cast<uint64_t>(levels) * T * ((kPathF + 1) * 8 + kPathI * 4);
    }
};

// Wavefront working set for one chunk of a tile (HBM; sized by the host for
// `cap` pixels / `slots` generation-0 slots; 288 GB leaves room).
// Generation k = recursion depth k (raytrace.rs:33,63): queue Q_k holds the
// rays ray_color is called with at depth k.
//
// ONE allocation, addressed by offsets: a kernel keeps one base pointer and a
// few sizes live instead of ~40 array pointers (which the compiler holds in
// SGPRs and spills into the traversal loop's VGPRs).  Sections, each an SoA
// of arrays:
//   queues   [parity 2][field 8][qcap]: origin x,y,z, direction x,y,z,
//            significance (f64), owning chain (u32 in an 8-B slot); queues
//            ping-pong by generation parity;
//   records  shade records, f64 fields [7][levels*qcap] (hit point x,y,z,
//            incoming direction x,y,z, significance) then u32 fields
//            [4][levels*qcap] (object id, primitive: sphere >= 0 / ~plane,
//            chain, occlusion mask: bit l = light l shadowed).  One region
//            array per generation (generation k at k*qcap), so the nearest-hit
//            kernels never wait for the shadow / shading kernels of earlier
//            generations (the other stream);
//   levels   per-level local colour r,g,b and Schlick factor (f64)
//            [4][levels*capa], then object id (i32) [levels*capa]; [k*capa + c]
//            for chain c (chain = the entry of the lit camera hit's generation-0
//            record, capa >= qcap; its pixel is cpix[c]), so a generation's
//            levels are written in about its records' order;
//   term     terminal colour of each chain [3][capa] (f64), then nlev (u8,
//            levels pushed) [capa];
//   rq / rs  [k*G + r]: entries of region r of Q_k / of generation k's records;
//   cpix     the chunk pixel of each chain [qcap] (u32);
//   pmap     (compose) per chunk pixel [cap]: its chain, or kPixBackground /
//            kPixAmbient | object for a camera ray that ended without a chain;
//            With mark (sparse host copies) its first cap bytes are cmark
//            instead: 1 for a pixel that starts a chain, else 0;
//   ccol     (compose) per chain [capa]: final colour f32 r,g,b and the sRGB
//            bytes b | g << 8 | r << 16 (16 B), written by the fold in chain
//            order and read by wf_compose, which writes the frame row by row.
// Queue and record arrays are G regions of R entries (qcap = G*R); region r is
// written only by workgroup r of the producing kernel.
struct WfBufs {
    unsigned char* mem;
    unsigned long long* totals;     // [0] nearest queries, [1] shadow queries, [2..3] nearest box / sphere
                                    // tests, [4..5] shadow box / sphere tests (accumulated over chunks)
    unsigned long long* gen_totals; // per-generation queue / shade-record totals over the chunks of a render
    uint64_t qcap;                  // G * R
    uint64_t o_rec, o_lev, o_term, o_rq, o_rs, o_cpix, o_pmap, o_ccol;   // byte offsets of the sections
    uint32_t cap;                   // pixel capacity
    uint32_t capa;                  // qcap rounded up to 64: stride of the per-chain arrays (levels,
                                    // terminals; chain c = generation 0's record entry c)
    uint32_t levels;                // record generations / stack levels (max_depth + 1)
    uint32_t G;                     // regions per queue
    uint32_t R;                     // entries per region: ceil(slots / (G * 1024)) * 1024
    uint32_t slots;                 // generation-0 slots of this chunk (8x8 tiles, >= pixels)
    uint32_t tiles_x;               // 8x8 tiles per row of the chunk
    uint32_t spread_below;          // queues below this many items are dealt workgroup-first regardless
    uint32_t wg_major;              // chunk dealing: 1 = consecutive chunks to the waves of one
                                    // workgroup (idle workgroups exit at once), 0 = workgroup-first
    uint32_t compose;               // 1: final colours go through pmap / ccol and wf_compose writes the
                                    //   frame in row order; 0: the camera pass and the fold write pixels
    uint32_t mark;                  // 1 (sparse host copies, compose 0): the camera pass writes cmark

    // queues: f = 0..5 origin / direction, 6 significance
    RT_HD double* qf(int q, int f) const { return reinterpret_cast<double*>(mem) + (static_cast<uint64_t>(q) * 8 + f) * qcap; }
    RT_HD uint32_t* qpix(int q) const {
        return reinterpret_cast<uint32_t*>(reinterpret_cast<double*>(mem) + (static_cast<uint64_t>(q) * 8 + 7) * qcap);
    }
    // records (index = k * qcap + entry): f = 0..2 point, 3..5 direction, 6 significance
    RT_HD uint64_t rn() const { return static_cast<uint64_t>(levels) * qcap; }
    RT_HD double* rf(int f) const { return reinterpret_cast<double*>(mem + o_rec) + f * rn(); }
    RT_HD uint32_t* ru(int f) const {             // 0 object, 1 primitive, 2 chain, 3 occlusion
        return reinterpret_cast<uint32_t*>(reinterpret_cast<double*>(mem + o_rec) + 7 * rn()) + f * rn();
    }
    // levels (index = k * capa + chain): f = 0..2 colour, 3 Schlick factor
    RT_HD double* lf(int f) const { return reinterpret_cast<double*>(mem + o_lev) + static_cast<uint64_t>(f) * levels * capa; }
    RT_HD int32_t* lobj() const {
        return reinterpret_cast<int32_t*>(reinterpret_cast<double*>(mem + o_lev) + static_cast<uint64_t>(4) * levels * capa);
    }
    RT_HD double* term(int f) const { return reinterpret_cast<double*>(mem + o_term) + static_cast<uint64_t>(f) * capa; }
    RT_HD uint8_t* nlev() const { return reinterpret_cast<uint8_t*>(reinterpret_cast<double*>(mem + o_term) + 3ull * capa); }
    RT_HD uint32_t* cpix() const { return reinterpret_cast<uint32_t*>(mem + o_cpix); }   // chain -> chunk pixel
    RT_HD uint32_t* pmap() const { return reinterpret_cast<uint32_t*>(mem + o_pmap); }   // chunk pixel -> chain / code
    RT_HD uint32_t* ccol() const { return reinterpret_cast<uint32_t*>(mem + o_ccol); }   // chain c -> final colour [4c, 4c+4)
    // (mark) chunk pixel -> 1 if a chain starts there, 0 if the camera pass wrote its final colour
    // (the pmap section's bytes: compose and mark are never on together)
    RT_HD uint8_t* cmark() const { return mem + o_pmap; }
    RT_HD uint32_t* rq() const { return reinterpret_cast<uint32_t*>(mem + o_rq); }
    RT_HD uint32_t* rs() const { return reinterpret_cast<uint32_t*>(mem + o_rs); }
};
constexpr uint32_t kNlevRunning = 0xFFu;   // WfBufs::nlev of a chain that has not ended yet
constexpr uint32_t kPixBackground = 0xFFFFFFFFu;   // WfBufs::pmap: the camera ray missed every object
constexpr uint32_t kPixAmbient = 0x80000000u;      // ... | object: it ended on that object's ambient colour

constexpr int kWfThreads = 1024;      // workgroup size of the queue kernels
constexpr int kMaxRegions = 2048;     // upper bound of WfBufs::G
constexpr int kMaxScan = 4096;        // region sizes one region_scan covers (several generations' regions)
constexpr int kMaxGenerations = 34;   // RT_MAX_DEPTH_LIMIT + 2 generations, + 1 spare for the last producer
constexpr int kCntQ = 0;              // gen_totals layout: [kCntQ + k] queue sizes, [kCntS + k] shade records
constexpr int kCntS = 64;
constexpr int kCntWords = 128;
constexpr int kCounterShards = 256;
constexpr int kMaxLevels = 32;      // >= RT_MAX_DEPTH_LIMIT + 2

}  // namespace rtamd
