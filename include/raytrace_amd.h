/*
 * raytrace_amd.h -- C ABI of the MI355X-native per-pixel ray-tracing path.
 *
 * This is the drop-in boundary for j-dong/rust-raytrace's hot path.  The
 * reference has no FFI of its own: its "operator API" is Rust trait objects
 * (Shape / Material / LightModel / Background / Camera) called once per pixel
 * sample from the serial loop in main.rs:45-57.  A per-sample FFI call is far
 * too fine-grained for a GPU and `dyn` objects cannot cross a C ABI, so the
 * boundary sits one level up: the host parses and flattens the Scene, and the
 * library renders whole frames / tiles / row bands on one device.
 *
 * Entry point -> reference interface it replaces:
 *   rt_scene_parse        serialize.rs:427-441   pub fn deserialize(&String) -> Result<Scene, SyntaxError>
 *   rt_scene_from_desc    scene.rs:201-212       building a `Scene { objects, lights, camera, background, options }` in code
 *   rt_camera_simple_new  camera.rs:51-63        SimplePerspectiveCamera::new
 *   rt_camera_look_at     camera.rs:67-73        SimplePerspectiveCamera::look_at
 *   rt_render / rt_render_device
 *                         main.rs:39-57 + raytrace.rs:270-276 (raytrace) + raytrace.rs:261-267
 *                         (ray_color) + raytrace.rs:30-67 (PhongMaterial::color) + scene.rs:247-249
 *                         (Scene::intersect) + shapes.rs:50-112 (Sphere/Plane::intersect)
 *   rt_scene_set_skybox   scene.rs:174-188       SkyboxBackground { px, nx, py, ny, pz, nz }
 *   rt_texture_load       texture.rs:34-37       Texture::load (BMP and binary PPM here; the image crate decodes more)
 *   rt_to_srgb            color.rs:593-600       fn to_srgb (used by Color::write_bgr, color.rs:628-632)
 *   rt_bmp_header         bmp.rs:10-61           pub fn write_header
 *   rt_write_bmp          main.rs:34-59          header + bottom-up BGR rows to a file
 *
 * Conventions:
 *   - Every function returns RT_OK (0) or a negative RT_E_* code.  No C++
 *     exception or abort crosses the ABI.  rt_last_error() describes the last
 *     failure of a context (thread-local text for context-free calls).
 *   - All pointers are caller-owned; the library copies what it keeps.
 *   - One rt_ctx per device; calls on one context are not thread-safe;
 *     different contexts may be driven concurrently (one host thread per GPU).
 *   - A context's renders are ordered: each waits (on the device, not the
 *     host) for the context's previous render, whatever streams they were
 *     issued on, because they share the context's working set.  A stream
 *     passed to rt_render_device must outlive the renders issued on it (a
 *     render on the same stream as the previous one relies on stream order).
 *     rt_scene_upload waits for every render still reading the old scene.
 *   - Nothing is read from the environment: a render's schedule depends only
 *     on the scene, the options and the context's tuning (rt_ctx_set_tuning).
 *   - All scene arithmetic is IEEE f64 exactly as the reference (no FMA
 *     contraction); output colours are the f64 result rounded once to f32,
 *     and the u8 BGR bytes are quantised from the f64 value on the device.
 *   - Pixel row 0 is the image BOTTOM (the first row written, main.rs:45/58).
 */
#ifndef RAYTRACE_AMD_H
#define RAYTRACE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: rt_out_flags gained RT_OUT_FRAME_ROWS (rt_render writes a banded tile
 * straight into its rows of a whole-frame host buffer); rt_ctx_reserve added;
 * rt_sqrt_check added; rt_kernel_family index 6 is RT_KF_COMPOSE (earlier ABI-4 builds named it
 * RT_KF_SHADOW); the tuning keys fuse, lists,
 * lists0, fuse_from, prefix4_kb, cam_prefix_kb, tail_from, tail_max,
 * eager_fold, fold_split, bmerge, wave_max, tail_fold, tail_shade, fold_wgs and
 * shade_wgs (variants measured slower and removed) are gone:
 * rt_ctx_set_tuning answers RT_E_INVALID for them; tuning keys chain_on_caller,
 * copy_engine and dev_join added.  rt_stats unchanged (80 B); its kernel_ms is 0
 * after an rt_render_device without RT_TIME_KERNELS / RT_COUNT_WORK.
 * 4: rt_abi_version() added; RT_KF_TAIL (RT_KF_COUNT 8).  A caller checks
 * rt_abi_version() == RT_ABI_VERSION of the header it was built against before
 * passing any struct; any change of a struct, enum value or tuning key bumps it. */
#define RT_ABI_VERSION 5

enum rt_status {
    RT_OK = 0,
    RT_E_INVALID = -1,      /* bad argument */
    RT_E_NODEVICE = -2,     /* no HIP device / bad device index */
    RT_E_HIP = -3,          /* HIP runtime error (see rt_last_error) */
    RT_E_NOMEM = -4,
    RT_E_UNSUPPORTED = -5,  /* scene uses a class the device path does not implement yet */
    RT_E_PARSE = -6,        /* scene text failed to parse (SyntaxError) */
    RT_E_NOSCENE = -7,      /* render before upload */
    RT_E_IO = -8
};

/* ---- scene model (flattened mirror of scene.rs / shapes.rs / camera.rs) ---- */
enum rt_shape_kind { RT_SHAPE_SPHERE = 0, RT_SHAPE_PLANE = 1 };                 /* shapes.rs:42-112 */
enum rt_material_kind {                                                          /* scene.rs:32-89 */
    RT_MAT_PHONG = 0, RT_MAT_INDIRECT_PHONG = 1, RT_MAT_FRESNEL = 2, RT_MAT_TRANSPARENT = 3
};
enum rt_light_kind { RT_LIGHT_POINT = 0, RT_LIGHT_DIRECTIONAL = 1, RT_LIGHT_AREA = 2 };  /* scene.rs:117-155 */
enum rt_camera_kind { RT_CAMERA_SIMPLE = 0, RT_CAMERA_DOF = 1 };                 /* camera.rs:29-123 */
enum rt_background_kind { RT_BG_SOLID = 0, RT_BG_SKYBOX = 1 };                  /* scene.rs:164-188 */

typedef struct { double r, g, b; } rt_color;                                     /* color.rs:15-22 */

typedef struct {
    int32_t shape;          /* rt_shape_kind */
    int32_t material;       /* rt_material_kind */
    double geom[6];         /* sphere: center x,y,z, radius   plane: point x,y,z, normal x,y,z */
    rt_color diffuse;       /* Phong / IndirectPhong / Fresnel */
    rt_color specular;
    rt_color ambient;       /* Phong / IndirectPhong / Fresnel */
    double exponent;
    double ior;             /* Fresnel / Transparent */
    uint32_t samples;       /* IndirectPhong */
    uint32_t _pad;
} rt_object;

typedef struct {
    int32_t kind;           /* rt_light_kind */
    int32_t _pad;
    double v[9];            /* point: location; directional: direction; area: origin, side1, side2 */
    rt_color color;
} rt_light;

typedef struct {
    int32_t kind;           /* rt_camera_kind */
    uint32_t samples;       /* DepthOfFieldCamera samples (1 for simple) */
    double position[3];     /* SimplePerspectiveCamera.position */
    double matrix[9];       /* SimplePerspectiveCamera.matrix, row-major M[i][j] */
    double focus, aperture; /* DepthOfFieldCamera */
} rt_camera;

typedef struct {
    const rt_object* objects; uint32_t n_objects;
    const rt_light* lights;   uint32_t n_lights;
    rt_camera camera;
    int32_t background_kind;  /* a desc carries RT_BG_SOLID; textures go through rt_scene_set_skybox */
    rt_color background;
    uint32_t width, height, antialias;   /* scene.rs:191-198 Options */
} rt_scene_desc;

/* texture.rs:22-26: an RGB8 image, rows top-down, width*height*3 bytes (caller-owned). */
typedef struct {
    uint32_t width, height;
    const uint8_t* rgb;
} rt_texture;

typedef struct rt_scene rt_scene;   /* host-side parsed scene (opaque) */
typedef struct rt_ctx rt_ctx;       /* one device context (opaque) */

/* ---- host-side scene API ---- */
int rt_scene_parse(const char* text, size_t len, rt_scene** out, char* err, size_t err_len);
int rt_scene_from_desc(const rt_scene_desc* desc, rt_scene** out);
/* Borrow the flattened view of a scene (valid until rt_scene_free). */
int rt_scene_get_desc(const rt_scene* scene, rt_scene_desc* out);
void rt_scene_free(rt_scene* scene);
/* Make the scene's background a SkyboxBackground with faces px, nx, py, ny, pz, nz (copied). */
int rt_scene_set_skybox(rt_scene* scene, const rt_texture faces[6]);
/* Diagnostic, host only (no device): the spheres the light-view grid of point
 * light `light` (built as rt_scene_upload builds it) hands a
 * shadow query from each point of `points` (n_points x 3 doubles): the same
 * candidate list, in the same order, as the device tests after the planes and
 * the hint.  counts[i] = its length, or -1 when the device tests every sphere
 * (degenerate direction, or no grid for this light); ids = the candidates'
 * object ids (file order, scene.rs:248), concatenated, at most cap in all.
 * info[0..2] = cells per face side, stored cells, list entries.  resolution:
 * cells per face side (0 = the upload's automatic choice, else 1..4096).
 * Replaces nothing in the reference (its shadow query scans every object,
 * scene.rs:247-249); tests check the lists against that scan. */
int rt_light_grid_candidates(const rt_scene* scene, int light, int resolution, const double* points, uint32_t n_points,
                             int32_t* counts, int32_t* ids, size_t cap, int64_t* info);
/* Diagnostic, host only: the camera's view grid (built as
 * rt_scene_upload builds it, spheres in file order) for camera-ray directions
 * `dirs` (n_dirs x 3 doubles): for each direction the spheres the device may
 * test -- the always list, then the direction's whole cell list in increasing
 * distance bound (the device stops once a bound exceeds its best t) --
 * counts[i] = its length, or -1 when the device tests every sphere; ids = object
 * ids, nears = each entry's distance bound (f32), both concatenated, at most cap
 * in all.  info[0..2] = cells per face side, stored cells, list entries.
 * resolution: cells per face side (0: from the scene's frame size).  Replaces
 * nothing in the reference (scene.rs:247-249 scans every object); tests check
 * the lists against that scan. */
int rt_view_grid_candidates(const rt_scene* scene, int resolution, const double* dirs, uint32_t n_dirs,
                            int32_t* counts, int32_t* ids, float* nears, size_t cap, int64_t* info);
/* Diagnostic, host only: the quantised 4-wide sphere tree (DESIGN.md §3.10,
 * built as rt_scene_upload builds it; leaf_max 0: the upload's leaf size) and
 * the f32 child boxes it rounds outward.  nodes: 48 B per node (the device
 * layout, DevQNode4), at most cap_nodes; boxes: per node and child slot
 * lo x,y,z, hi x,y,z (f32; NaN for an unused slot), at most cap_nodes * 24
 * floats; sphere_first / sphere_count: per node and slot the leaf's spheres in
 * leaf order (-1 / 0 for an inner child or unused slot).  info[0..2] = nodes (0:
 * not representable, the device keeps the other trees), the traversal stack's
 * worst case, the leaf size; cap_nodes 0 is a size query (info only).  Replaces nothing in the reference (scene.rs:247-249
 * scans every object); tests decode the nodes and check every box contains its
 * f32 box. */
int rt_qtree_nodes(const rt_scene* scene, int leaf_max, void* nodes, float* boxes, int32_t* sphere_first,
                   int32_t* sphere_count, size_t cap_nodes, int64_t* info);
/* Decode an image file as Texture::load does (RGB8, rows top-down).  rgb == NULL: only the size.
 * Formats: uncompressed BMP (24/32 bit) and binary PPM; others -> RT_E_UNSUPPORTED. */
int rt_texture_load(const char* path, uint32_t* width, uint32_t* height, uint8_t* rgb, size_t cap);

int rt_camera_simple_new(const double position[3], const double look[3], const double up[3],
                         double im_dist, rt_camera* out);
int rt_camera_look_at(const double focus[3], const double look[3], const double up[3],
                      double pov, double h, rt_camera* out);

uint8_t rt_to_srgb(double v);
/* Writes the 122-byte BITMAPV4 header; *bytewidth = padded row pitch. */
int rt_bmp_header(uint8_t out[122], uint32_t width, uint32_t height, uint32_t* bytewidth);
/* Writes header + pixel array (bgr rows, bottom-up, `pitch` bytes each) to `path`. */
int rt_write_bmp(const char* path, uint32_t width, uint32_t height, const uint8_t* bgr, uint32_t pitch);

/* ---- device API ---- */
/* The RT_ABI_VERSION this library was built with. */
int rt_abi_version(void);
int rt_device_count(int* n);
int rt_ctx_create(int device, rt_ctx** out);
void rt_ctx_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);
/* Copies the scene to HBM in the device layout.  Classes the device path does
 * not implement -> RT_E_UNSUPPORTED. */
int rt_scene_upload(rt_ctx* ctx, const rt_scene* scene);

enum rt_jitter {
    RT_JITTER_CENTER = 0,   /* jx = jy = 0.5 (deterministic parity mode, main.rs:51-52) */
    RT_JITTER_RANDOM = 1    /* jx, jy drawn per AA sample (main.rs:51-52) from the keyed RNG (rt_render_opts.seed) */
};
enum rt_out_flags {
    RT_OUT_RGB_F32 = 1,
    RT_OUT_BGR_U8 = 2,
    RT_COUNT_WORK = 4,         /* also count box / sphere tests (instrumented kernels; wavefront only) */
    RT_TIME_KERNELS = 8,       /* record a timing event after every launch (wavefront, one stream) */
    RT_OUT_FRAME_ROWS = 16     /* rt_render only: out_rgb / out_bgr hold the WHOLE frame (height rows; f32
                                  rows of 3*width floats, BGR rows of bgr_pitch bytes, 0 -> 3*width) and the
                                  tile's pixel (x, local row j) lands in column x0 + x of its frame row
                                  y0 + ((j/band)*band_stride + band_phase)*band + j%band; nothing else of
                                  the buffers is written.  The multi-GPU host gather (main.rs:45-58 split
                                  over devices): each context renders its row bands straight into one
                                  shared page-locked frame, the copies overlapping its render. */
};
enum rt_algo {
    RT_ALGO_AUTO = 0,
    RT_ALGO_BRUTE_LDS = 1,      /* megakernel, sphere list staged in LDS */
    RT_ALGO_BRUTE_GLOBAL = 2,   /* megakernel, sphere list read through the caches */
    RT_ALGO_WAVEFRONT = 3,      /* per-depth launches over compacted ray queues, sphere BVH (default) */
    RT_ALGO_WAVEFRONT_BRUTE = 4, /* the same schedule, every sphere tested (linear scan like scene.rs:248) */
    RT_ALGO_PATH = 5            /* per-pixel recursion over an HBM stack: every material / light / camera class
                                   (IndirectPhong, Transparent, AreaLight, DepthOfField, random jitter); AUTO picks
                                   it whenever the scene or the jitter mode needs it */
};

typedef struct {
    uint32_t width, height;   /* full frame: defines the pixel -> (-1,1) mapping (main.rs:39-41) */
    uint32_t x0, tile_w;      /* columns [x0, x0 + tile_w) */
    uint32_t y0, tile_h;      /* local row j -> global row y0 + ((j/band)*band_stride + band_phase)*band + j%band */
    uint32_t band, band_stride, band_phase;   /* 0 -> 1: contiguous rows */
    uint32_t max_depth;       /* reference MAX_DEPTH = 4 (raytrace.rs:18); <= RT_MAX_DEPTH_LIMIT */
    uint32_t spp;             /* AA samples (Options.antialias); 0 -> the uploaded scene's value */
    int32_t jitter;           /* rt_jitter */
    uint32_t flags;           /* rt_out_flags */
    int32_t algo;             /* rt_algo */
    uint32_t bgr_pitch;       /* bytes per output BGR row; 0 -> 3*tile_w */
    uint32_t _pad;
    uint64_t seed;            /* keyed RNG seed: every random draw is a function of (seed, pixel, AA sample,
                                 camera sample, path through the ray tree, draw id), so a frame is
                                 reproducible and independent of tiling and GPU count.  The reference
                                 seeds one sequential XorShift stream from OS entropy (main.rs:43). */
} rt_render_opts;

#define RT_MAX_DEPTH_LIMIT 30

typedef struct {
    uint64_t rays;            /* every Scene::intersect query issued (camera + reflection + shadow) */
    uint64_t shadow_rays;
    uint64_t pixels;
    double kernel_ms;         /* hipEvent time from the first to the last launch of the render
                                 (rt_render, and rt_render_device with RT_TIME_KERNELS or
                                 RT_COUNT_WORK; 0 for other rt_render_device renders, which
                                 record no start event: one marker fewer between frames) */
    uint64_t box_tests;       /* RT_COUNT_WORK only: BVH slab tests (2 per inner node visited) */
    uint64_t sphere_tests;    /* RT_COUNT_WORK only: exact ray-sphere quadratics evaluated */
    uint64_t shadow_box_tests, shadow_sphere_tests;   /* the shadow-query share of the two above */
    uint64_t traced_rays;     /* queries the device actually traced: `rays` / spp when a chain schedule
                                 renders spp identical centre-jitter samples once, else `rays` */
    uint64_t chunks;          /* row chunks the wavefront schedule ran the tile as (sized to the
                                 working-set budget, tuning wf_budget_mb); 0 for other schedules */
} rt_stats;

void rt_render_opts_default(rt_render_opts* o, uint32_t width, uint32_t height);

/* Synchronous: renders into caller-owned HOST buffers (either may be NULL).
 * Page-locked buffers (hipHostMalloc / hipHostRegister) receive the DMA
 * directly; pageable ones are filled through four pinned 8 MiB staging slices,
 * the copy engine filling slices ahead while a pool of host threads empties
 * them in order.  Pass only the outputs needed: BGR alone moves 3 B per pixel
 * instead of 15 (C3, 4096^2: DESIGN.md §6 gives the measured end-to-end time). */
int rt_render(rt_ctx* ctx, const rt_render_opts* opts, float* out_rgb, uint8_t* out_bgr, rt_stats* stats);
/* Asynchronous on `stream` (a hipStream_t; NULL = the context's own stream):
 * renders into caller-owned DEVICE buffers.  Statistics of the most recent
 * render are read with rt_ctx_stats (which synchronises). */
int rt_render_device(rt_ctx* ctx, const rt_render_opts* opts, void* d_rgb, void* d_bgr, void* stream);
/* Prepare the context for renders with these options, synchronously and
 * without rendering: the schedule's streams and hardware queues, its working
 * set (sized exactly as the render sizes it), rt_render's device frame and
 * sparse-copy buffers (host = 1) and the kernels' code objects.  A later
 * rt_render / rt_render_device with the same options (or smaller ones) then
 * allocates nothing: a process that renders one frame (main.rs:13-60) calls
 * it after rt_scene_upload, e.g. while it parses or opens its output.  Needs
 * an uploaded scene (the schedule depends on it); RT_E_NOMEM if the working
 * set does not fit even as the smallest chunks.  stream: the hipStream_t the
 * rt_render_device calls will be issued on (its hardware queue is set up too;
 * NULL = the context's own stream, which rt_render uses). */
int rt_ctx_reserve(rt_ctx* ctx, const rt_render_opts* opts, int host, void* stream);
int rt_ctx_stats(rt_ctx* ctx, rt_stats* stats);
/* Diagnostic (device): the sphere test's division t = x / (2a) (shapes.rs:68,75)
 * computed as the device computes it (the per-ray reciprocal of 2a finished with
 * the division's own correction steps, DESIGN.md §4 "Division by 2a") -> fast[i],
 * and as the device's own f64 division -> slow[i], for n operand pairs.  Tests
 * compare both with IEEE division bit for bit.  Synchronous. */
int rt_div_a2_check(rt_ctx* ctx, const double* x, const double* a, uint32_t n, double* fast, double* slow);
/* Diagnostic (device): the sphere test's square root (shapes.rs:67) as the device
 * computes it (the f64 sqrt sequence without its scaling of operands below 2^-767,
 * DESIGN.md §4) -> fast[i], and the device's own sqrt -> slow[i].  Tests compare
 * both with IEEE sqrt bit for bit.  Synchronous. */
int rt_sqrt_check(rt_ctx* ctx, const double* x, uint32_t n, double* fast, double* slow);
/* Queue sizes of the last wavefront chunk: queue[k] = rays traced at depth k
 * (generation 0: 0, the camera rays are not queued), shaded[k] = hits that
 * issued shadow queries.  Diagnostic. */
int rt_ctx_generation_counts(rt_ctx* ctx, uint32_t* queue, uint32_t* shaded, int n);
/* Per kernel family, over every RT_TIME_KERNELS render since the previous
 * call: summed launch time (ms, hipEvent pairs around each launch) and launch
 * count; then resets.  Synchronises with the last timed launch.  Families:
 * rt_kernel_family.  Renders split over several chunk streams are not timed. */
enum rt_kernel_family {
    RT_KF_NEAREST = 0,      /* wf_nearest, generations >= 1 */
    RT_KF_OCCLUSION = 1,    /* wf_occlusion: every (record, light) pair of a generation */
    RT_KF_SHADE = 2,        /* wf_shade */
    RT_KF_FOLD = 3,         /* wf_fold */
    RT_KF_TALLY = 4,        /* wf_tally */
    RT_KF_CAMERA = 5,       /* wf_nearest, generation 0 (camera rays) */
    RT_KF_COMPOSE = 6,      /* wf_compose: the row-ordered frame pass (tuning compose) */
    RT_KF_TAIL = 7,         /* wf_tail: the fused generations >= tail_fuse */
    RT_KF_COUNT = 8
};
int rt_ctx_kernel_times(rt_ctx* ctx, double* ms, uint32_t* launches, int n);

/* Schedule tuning of a context (A/B measurement; the defaults are the measured
 * best).  Keys (rt_tuning_key(i) for i = 0, 1, ... until NULL):
 * chunk_pixels (wavefront chunk cap, 0: from the working-set budget), bvh_leaf, light_grids, light_grid_res
 * (these three take effect at the next rt_scene_upload), src, src_occ (the
 * nearest-hit and shadow sphere sources, trace_kernel.hip kSrc*; an unsupported
 * pair falls back to the binary tree through L2), prefix_kb (KB of the tree's
 * top staged in LDS for trees beyond LDS), lanes, stagger_gen, regions, split,
 * bstreams, cam (generation 0: 3 the camera's view grid, -1 where built, other
 * values per ray), deal, spread_below, path_group, cu_mask, prio, verbose,
 * grid_occ, compact_stack (small trees: 32-bit nearest-hit stack entries),
 * half_nodes (trees beyond LDS: binary16 node bounds for the prefix walk),
 * wf_budget_mb (wavefront working set of all chunk lanes, MB; 0: min(80 GB, 85%
 * of the device's free memory); a hipMalloc that still fails halves the chunks),
 * cam_grid_res (the view grid's cells per face side, 0 from the scene's frame
 * size, -1 none; at the next rt_scene_upload), a_queue (1: the nearest-hit
 * chain's stream gets a hardware queue of its own), tail_fuse (T >= 1: the
 * chains still running at generation T-1 of a frame on the src-9 tree whose
 * lights all have light-view grids finish in one launch, one chain per
 * work-item through its remaining bounces, folded there; 0 off, -1 auto),
 * tail_width (that launch's chains per wave, 0 auto), qtree (1: trees beyond
 * LDS take the quantised 4-wide tree for the nearest hit), compose (1: the
 * chains' final colours go to a per-chain buffer and one row-ordered pass,
 * RT_KF_COMPOSE, writes the frame with coalesced stores; 0: each chain writes
 * its pixel as it ends), host_chunks (rt_render into host memory: at least
 * this many chunks, the D2H copy of each chunk's rows overlapping the later
 * chunks), host_first (with host_chunks 2: the first chunk's percentage of
 * the rows, 0 equal), sparse_out (rt_render into host memory, a one-chunk
 * wavefront render: the frame is copied after the camera pass while the
 * generations run, then only the 16-pixel row segments holding pixels whose
 * chain was still running, packed on the device), chain_on_caller (1: a
 * one-lane render's nearest-hit chain runs on the caller's stream itself, no
 * fork and join between hardware queues; 0: on the context's high-priority
 * chain stream), copy_engine (rt_render's device -> host copies: 0
 * hipMemcpyAsync, e = 1..16 the device's SDMA engine e - 1 driven directly,
 * -1 its engines 0-3 in turn, -2 (default) -1 for a row-banded tile
 * (band_stride > 1) and 0 otherwise; a device without usable engines takes
 * hipMemcpyAsync), dev_join (1: the b streams join the chain's
 * stream on the device, a one-wave kernel polling flags that the b streams set
 * after their work; 0: through events; a join that waits 2 s gives up and
 * makes the next rt_render or rt_ctx_stats fail; the default is 0 in a process whose
 * kernels are serialised, ROCPROF_COUNTER_COLLECTION or AMD_SERIALIZE_KERNEL
 * set, where the b streams could not run beside the join).
 * cu_mask, prio and a_queue rebuild the context's streams (after pending work) when changed.
 * Unknown key or value out of range -> RT_E_INVALID.  Results never depend on
 * them (tests/test_gpu_parity.py renders under several and compares bits). */
int rt_ctx_set_tuning(rt_ctx* ctx, const char* key, int64_t value);
int rt_ctx_get_tuning(const rt_ctx* ctx, const char* key, int64_t* value);
const char* rt_tuning_key(int index);

#ifdef __cplusplus
}
#endif
#endif
