/*
 * ref64 -- CPU ORACLE for the per-pixel ray-tracing path of j-dong/rust-raytrace.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline).  The product path (librtamd.so) never links,
 * loads or calls it.
 *
 * It is a plain-C f64 restatement of the reference algorithm, following:
 *   main.rs:39-59        pixel mapping, AA loop and average, BGR row write
 *   camera.rs:51-80      SimplePerspectiveCamera new / look_at / project
 *   camera.rs:83-123     DepthOfFieldCamera (stochastic: keyed draws = the device's, REF_RNG_KEYED)
 *   raytrace.rs:17-28    MIN_SIGNIFICANCE, MAX_DEPTH (a parameter here), clamps
 *   raytrace.rs:30-67    PhongMaterial::color
 *   raytrace.rs:69-121   IndirectPhongMaterial::color (stochastic; keyed or XorShift draws)
 *   raytrace.rs:123-167  FresnelMaterial::color
 *   raytrace.rs:169-226  TransparentMaterial::color
 *   raytrace.rs:228-256  SolidColorBackground, SkyboxBackground (texture.rs:46-58 sampling)
 *   raytrace.rs:261-276  ray_color / raytrace
 *   scene.rs:117-155     Point / Directional / Area lights
 *   scene.rs:223-249     Scene::intersect (first-wins ties, NaN-t wins)
 *   shapes.rs:22-24,50-112  Ray::cast, Sphere::intersect, Plane::intersect
 *   color.rs:27-67,593-600,628-639  Color ops, to_srgb, write_bgr, significance
 *   bmp.rs:10-61         BMP header
 * All arithmetic is IEEE f64 with no contraction (built -ffp-contract=off).
 * nalgebra ^0.4 op order is ASSUMED (source absent): dot = (x*x'+y*y')+z*z',
 * normalize = v / sqrt(sqnorm) per component, Mat3*Vec3 = row dot products.
 *
 * Pinning (see DESIGN.md "Oracle"): the sRGB tables and BMP header are pinned
 * bit-exactly by the reference's own data (color.rs tables, out.bmp header);
 * the camera/plane/sphere/intersect/IndirectPhong semantics are pinned
 * STATISTICALLY by out.bmp (the reference's only render).  The Phong hot path
 * itself has no golden in the reference: parity there is against this
 * restatement ("parity unpinned" beyond the shared sub-paths above).
 */
#ifndef REF64_H
#define REF64_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { REF_SPHERE = 0, REF_PLANE = 1 };
enum { REF_PHONG = 0, REF_INDIRECT_PHONG = 1, REF_FRESNEL = 2, REF_TRANSPARENT = 3 };
enum { REF_POINT = 0, REF_DIRECTIONAL = 1, REF_AREA = 2 };
enum { REF_CAM_NEW = 0, REF_CAM_LOOK_AT = 1 };

typedef struct {
    int32_t shape;       /* REF_SPHERE / REF_PLANE */
    int32_t material;    /* REF_PHONG ... */
    double geom[6];      /* sphere: center xyz, radius;  plane: point xyz, normal xyz */
    double diffuse[3], specular[3], ambient[3];
    double exponent, ior;
    uint32_t samples;
} ref_object;

typedef struct {
    int32_t kind;        /* REF_POINT / REF_DIRECTIONAL / REF_AREA */
    double v[9];         /* point: location; directional: direction; area: origin, side1, side2 */
    double color[3];
} ref_light;

typedef struct {
    int32_t ctor;        /* REF_CAM_NEW: p0=position p1=look p2=up s0=im_dist
                            REF_CAM_LOOK_AT: p0=focus p1=look p2=up s0=pov(rad) s1=h */
    double p0[3], p1[3], p2[3];
    double s0, s1;
    int32_t dof;         /* 1 = DepthOfFieldCamera wrapping the above */
    double focus, aperture;
    uint32_t dof_samples;
} ref_camera;

/* texture.rs:22-26: RGB8, rows top-down (what image::open(..).to_rgb() yields) */
typedef struct {
    uint32_t width, height;
    const uint8_t* rgb;
} ref_texture;

typedef struct {
    const ref_object* objects; uint32_t n_objects;
    const ref_light* lights;   uint32_t n_lights;
    ref_camera camera;
    double background[3];
    uint32_t width, height, antialias;
    const ref_texture* skybox;   /* NULL: SolidColorBackground; else SkyboxBackground px, nx, py, ny, pz, nz */
} ref_scene;

enum { REF_JITTER_CENTER = 0, REF_JITTER_RANDOM = 1 };
/* Where the random draws come from.  XORSHIFT: the reference's rand 0.3
 * XorShiftRng consumed sequentially (per row here; the reference seeds it from
 * OS entropy, main.rs:43, so only its distribution is reproducible).  KEYED:
 * a counter-based stream keyed on the draw's place in the recursion (pixel,
 * AA sample, camera sample, path through the ray tree, draw id) -- the same
 * specification the device path implements (trace_common.hpp "keyed RNG"),
 * so device and oracle agree draw for draw, in any traversal order. */
enum { REF_RNG_XORSHIFT = 0, REF_RNG_KEYED = 1 };

typedef struct {
    uint32_t max_depth;      /* reference MAX_DEPTH = 4 (raytrace.rs:18) */
    int32_t jitter;          /* REF_JITTER_CENTER: jx = jy = 0.5 (deterministic parity mode) */
    uint64_t seed;           /* stochastic paths only */
    uint32_t x0, tile_w;     /* columns [x0, x0+tile_w) */
    uint32_t y0, tile_h;     /* local row j -> global row y0 + ((j/band)*stride + phase)*band + j%band */
    uint32_t band, band_stride, band_phase;
    int32_t threads;         /* <=0: all online CPUs */
    int32_t rng;             /* REF_RNG_XORSHIFT / REF_RNG_KEYED */
} ref_opts;

typedef struct {
    uint64_t rays;           /* every Scene::intersect call (nearest-hit + shadow) */
    uint64_t shadow_rays;
    uint64_t sphere_tests;
    uint64_t plane_tests;
} ref_counts;

/* Render a tile.  Any output pointer may be NULL.
 *   out_rgb64 / out_rgb32: tile_h rows of tile_w RGB triples (row 0 = first local row)
 *   out_bgr: tile_h rows of bgr_pitch bytes, B,G,R per pixel (color.rs:628-632)
 * Returns 0, or -1 on invalid arguments. */
int ref_render(const ref_scene* scene, const ref_opts* opts,
               double* out_rgb64, float* out_rgb32, uint8_t* out_bgr, uint32_t bgr_pitch,
               ref_counts* counts);

/* Building blocks, exported for known-answer tests. */
int ref_sphere_intersect(const double center[3], double radius, const double o[3], const double d[3],
                         double* t, double normal[3]);          /* 1 = hit */
int ref_plane_intersect(const double point[3], const double n[3], const double o[3], const double d[3],
                        double* t, double normal[3]);           /* 1 = hit */
int ref_camera_build(const ref_camera* cam, double position[3], double matrix[9]);
uint8_t ref_to_srgb(double v);
double ref_srgb_average(int i);
double ref_srgb_value(int i);
uint32_t ref_bmp_header(uint8_t out[122], uint32_t width, uint32_t height);   /* returns bytewidth */

#ifdef __cplusplus
}
#endif
#endif
