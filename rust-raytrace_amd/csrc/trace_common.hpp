// Device-side exact restatement of the reference's per-ray math, shared by the
// megakernel and the wavefront kernels (trace_kernel.hip).
//
// Exactness: every operation is the reference's f64 operation in the
// reference's order, compiled with -ffp-contract=off (no FMA fusion; Rust never
// fuses).  f64 add/mul/div/sqrt are IEEE correctly rounded on gfx950, so the
// only possible difference from the CPU is pow() (raytrace.rs:55): OCML vs
// glibc, <= 1 ulp (measured: bit-identical on every parity scene so far).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device_layout.hpp"

namespace rtamd {

extern __constant__ double c_srgb_avg[255];

constexpr double kMinSignificance = 1.0 / 256.0 / 2.0;            // raytrace.rs:17
constexpr double kEps = 0.00001;                                   // raytrace.rs:43,62
constexpr double kFrac1Pi = 0.318309886183790671537767526745028724; // f64::consts::FRAC_1_PI

struct Ray {
    double ox, oy, oz, dx, dy, dz;
};

struct Hit {
    double t;
    int32_t obj;        // object id, INT32_MAX = no hit
    int32_t prim;       // sphere index (>= 0) or ~plane index (< 0)
    bool nan_t;
};

struct Col {
    double r, g, b;
};

// ---- keyed RNG --------------------------------------------------------------
// The reference draws from ONE sequential XorShiftRng seeded from OS entropy
// (main.rs:43): no run can be reproduced and the stream order is the serial
// pixel loop's.  The device path instead makes every draw a pure function of
// its place in the recursion, so any schedule gives the same image and the
// oracle (oracle/ref64.c, REF_RNG_KEYED) reproduces it draw for draw:
//   pixel      kp = mix(mix(seed) + (y << 32 | x))        (frame coordinates)
//   AA sample  ka = child(kp, a)    jitter jx = f64(ka, 0), jy = f64(ka, 1)  (main.rs:51-52)
//   camera     kc = child(ka, cs)   DoF theta = f64(kc, 0), r2 = closed01(kc, 1)  (camera.rs:115-117)
//   a hit with path key K draws     AreaLight l: u = f64(K, 2+2l), w = f64(K, 3+2l)  (scene.rs:153)
//                                   indirect sample i: f64(K, 128+2i), f64(K, 129+2i)  (raytrace.rs:101-102)
//   child ray i of a hit has key child(K, i) (mirror reflection 0, refraction 1,
//   indirect sample i).
// f64 / closed01 follow rand 0.3's bit recipes (52 mantissa bits; 53 bits over 2^53 - 1).
__device__ __forceinline__ uint64_t kmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t key_child(uint64_t k, uint64_t i) { return kmix(k + (i + 1) * 0x9E3779B97F4A7C15ull); }
__device__ __forceinline__ uint64_t key_bits(uint64_t k, uint32_t id) {
    return kmix(k ^ (static_cast<uint64_t>(id + 1) * 0xD1B54A32D192ED03ull));
}
__device__ __forceinline__ double key_f64(uint64_t k, uint32_t id) {
    return __longlong_as_double(static_cast<long long>(0x3FF0000000000000ull | (key_bits(k, id) & 0xFFFFFFFFFFFFFull))) - 1.0;
}
__device__ __forceinline__ double key_closed01(uint64_t k, uint32_t id) {
    return static_cast<double>(key_bits(k, id) >> 11) / 9007199254740991.0;
}
__device__ __forceinline__ uint64_t key_pixel(uint64_t seed, uint32_t x, uint32_t y) {
    return kmix(kmix(seed) + ((static_cast<uint64_t>(y) << 32) | x));
}

__device__ __forceinline__ double clamp_zero(double x) { return x < 0.0 ? 0.0 : x; }   // raytrace.rs:20-23

// color.rs:593-600 as a binary search over the strictly increasing table.
__device__ __forceinline__ uint8_t to_srgb(double v, const double* table) {
    if (!(v < table[254])) return 255;           // also NaN
    int lo = 0, hi = 254;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int mid = (lo + hi) >> 1;
        bool lt = v < table[mid];
        hi = lt ? mid : hi;
        lo = lt ? lo : mid + 1;
    }
    return static_cast<uint8_t>(lo);
}

__device__ __forceinline__ uint8_t to_srgb(double v) { return to_srgb(v, c_srgb_avg); }

// The per-ray constants of shapes.rs:60-89's quadratic: a2 = 2.0*a and
// a4 = 4.0*a (the same f64 products the reference forms per test) and the
// reciprocal of a2 refined exactly as gfx950's f64 division refines its
// denominator (v_rcp_f64, then two Newton steps r += r*(1 - a2*r)).  `win` is
// the exponent window of numerators div_a2 may finish with that hoisted
// reciprocal (0: none, the ray's a2 is outside [2^-100, 2^101)).
struct SphK {
    double a2, a4, ra2;
    uint32_t win;
};

// Any denominator d (RT_DIVK: the normalisations' three divisions by one length): the same
// reciprocal and window, and div_by below the same three operations as div_a2 -- which is
// div_by with d = 2a, so rt_div_a2_check pins both.
struct DivK {
    double d, rd;
    uint32_t win;
};

__device__ __forceinline__ DivK div_k(double d) {
    DivK k;
    k.d = d;
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    k.rd = fma(r, e, r);
    const uint32_t ed = (static_cast<uint32_t>(__double2hiint(d)) >> 20) & 0x7FFu;
    k.win = ed - 923u < 201u ? 1500u : 0u;
    return k;
}

__device__ __forceinline__ SphK sphere_k(double a) {
    const DivK d = div_k(2.0 * a);
    SphK k;
    k.a2 = d.d;
    k.a4 = 4.0 * a;
    k.ra2 = d.rd;
    k.win = d.win;
    return k;
}

// x / a2, correctly rounded.  The compiler's f64 division is v_div_scale (of
// numerator and denominator), that reciprocal, q0 = x*r, e = fma(-a2, q0, x),
// v_div_fmas = fma(e, r, q0), v_div_fixup.  With a2 in [2^-100, 2^101) and
// |x| in [2^-900, 2^600) (biased exponent 123..1622) div_scale scales neither
// operand (exponent gap < 768, no denormal quotient or reciprocal, x not tiny)
// and div_fixup returns q with sign(x), so the three operations below give the
// division's bits; any other x (0, denormal, huge, inf, NaN) takes the division.
__device__ __forceinline__ double div_by(double x, const DivK& k) {
    const uint32_t ex = (static_cast<uint32_t>(__double2hiint(x)) >> 20) & 0x7FFu;
    if (ex - 123u < k.win) {
        const double q0 = x * k.rd;
        const double e = fma(-k.d, q0, x);
        return fma(e, k.rd, q0);
    }
    return x / k.d;
}

__device__ __forceinline__ double div_a2(double x, const SphK& k) { return div_by(x, DivK{k.a2, k.ra2, k.win}); }

// sqrt(x) as gfx950's correctly rounded f64 square root computes it (the compiler's
// sequence: v_rsq_f64 refined by Goldschmidt / Newton steps), without the parts that
// do nothing for x in [2^-767, +inf): the sequence scales x by 2^256 when x < 2^-767
// (and its result by 2^-128), which is ldexp by 0 here, and returns x itself for +-0
// and +inf, which x is not.  So for those x the core below gives the sequence's bits
// (pinned on the device against sqrt(): rt_sqrt_check, tests/test_gpu_division.py);
// any other x (tiny, denormal, 0, inf, NaN, negative) takes sqrt().
#ifndef RT_WSQRT
#define RT_WSQRT 1
#endif
// RT_DIVK: the normalisations (hit normal, light direction, half vector, camera ray) as
// div_k / div_by and sqrt_win (round 6, same box: C3 2.790 vs 2.806 ms, 8-way share 0.655-0.658
// vs 0.658-0.662 ms, C4 49.05 vs 49.24 ms, C5 291.0 vs 294.9 ms; exact: the GPU suite is green)
#ifndef RT_DIVK
#define RT_DIVK 1
#endif
__device__ __forceinline__ double sqrt_win(double x) {
    if (RT_WSQRT && x >= 0x1p-767 && x < __builtin_huge_val()) {
        const double y = __builtin_amdgcn_rsq(x);
        double g = x * y, h = y * 0.5;
        const double r = fma(-h, g, 0.5);
        g = fma(g, r, g);
        h = fma(h, r, h);
        double d = fma(-g, g, x);
        g = fma(d, h, g);
        d = fma(-g, g, x);
        return fma(d, h, g);
    }
    return sqrt(x);
}

// shapes.rs:60-89, split in two: sphere_disc forms b and the discriminant (the
// miss path, every test), sphere_roots the rest for disc > 0: t1, or t2 when t1 <= 0.
__device__ __forceinline__ double sphere_disc(const DevSphere& s, const Ray& r, const SphK& k, double& b) {
    const double ocx = r.ox - s.cx, ocy = r.oy - s.cy, ocz = r.oz - s.cz;
    b = 2.0 * (r.dx * ocx + r.dy * ocy + r.dz * ocz);
    const double cc = (ocx * ocx + ocy * ocy + ocz * ocz) - s.rr;
    return b * b - k.a4 * cc;
}

// kBF: the branch-free form (both quotients straight-line) or the branchy one (a division only
// for a positive numerator, the second root only when the first is behind).  Round 6, same box:
// C3 2.912-2.917 vs 2.924-2.930 ms branch-free everywhere, but C5 305.3 vs 294.6 ms and C4 49.46 vs
// 49.27 ms; the binary16 walk of trees beyond LDS (RT_BF_HALF) takes the branchy form.
#ifndef RT_ROOTS_BF
#define RT_ROOTS_BF 1
#endif
#ifndef RT_BF_HALF
#define RT_BF_HALF 0
#endif
#ifndef RT_BF_LDS
#define RT_BF_LDS 1
#endif
template <bool kBF = (RT_ROOTS_BF != 0)>
__device__ __forceinline__ bool sphere_roots(double b, double disc, const SphK& k, double& t) {
    const double sq = sqrt_win(disc);
    if constexpr (kBF) {
    // both roots' quotients straight-line (div_a2's three operations, whose result for x <= 0 or NaN is
    // never > 0), the real division only for a positive numerator outside the window (rare)
    const double x1 = -b - sq, x2 = -b + sq;
    auto fast = [&](double x) {
        const double q0 = x * k.ra2;
        const double e = fma(-k.a2, q0, x);
        return fma(e, k.ra2, q0);
    };
    auto in_win = [&](double x) { return ((static_cast<uint32_t>(__double2hiint(x)) >> 20) & 0x7FFu) - 123u < k.win; };
    double t1 = fast(x1), t2 = fast(x2);
    const bool slow1 = x1 > 0.0 && !in_win(x1), slow2 = x2 > 0.0 && !in_win(x2);
    if (slow1 || slow2) {
        if (slow1) t1 = x1 / k.a2;
        if (slow2) t2 = x2 / k.a2;
    }
    const bool h1 = t1 > 0.0;
    t = h1 ? t1 : t2;
    return h1 || t2 > 0.0;
    } else {
    // a2 >= 0 (or NaN): x <= 0 or NaN gives x / a2 <= 0, -0 or NaN, never > 0, so the
    // division is skipped there (a root behind the origin)
    const double x1 = -b - sq;
    if (x1 > 0.0) {
        const double t1 = div_a2(x1, k);
        if (t1 > 0.0) { t = t1; return true; }
    }
    const double x2 = -b + sq;
    if (x2 > 0.0) {
        const double t2 = div_a2(x2, k);
        if (t2 > 0.0) { t = t2; return true; }
    }
    return false;
    }
}

// The exact quadratic; true + the t the reference returns, or false for None.
template <bool kBF = (RT_ROOTS_BF != 0)>
__device__ __forceinline__ bool sphere_t(const DevSphere& s, const Ray& r, const SphK& k, double& t) {
    double b;
    const double disc = sphere_disc(s, r, k, b);
    return disc > 0.0 && sphere_roots<kBF>(b, disc, k, t);
}

// shapes.rs:100-112: t = n.(p - o) / n.d ; None iff t <= 0 (a NaN t is a hit).
__device__ __forceinline__ bool plane_t(const DevPlane& p, const Ray& r, double& t) {
    const double ex = p.px - r.ox, ey = p.py - r.oy, ez = p.pz - r.oz;
    t = (p.nx * ex + p.ny * ey + p.nz * ez) / (p.nx * r.dx + p.ny * r.dy + p.nz * r.dz);
    return !(t <= 0.0);
}

// Scene::intersect (scene.rs:247-249), brute force: every object tested.
// min_by_key(FloatNotNan(t)): a NaN t (only a plane can produce one) is the
// minimum key and the first in file order wins outright; otherwise smallest t,
// ties to the FIRST object in file order.
// Work counters (only in the kCount instantiations): boxes = slab tests,
// spheres = exact quadratic tests.
struct Work {
    uint32_t boxes = 0, spheres = 0;
#if RT_STAMP
    unsigned long long cyc[3] = {0, 0, 0};     // RT_STAMP builds: nearest_bvh_bl's descend / leaf / pop loops
    uint32_t wsteps[3] = {0, 0, 0};            // ... and the wave's iterations of them (counted by its first active lane)
#endif
};
#if RT_STAMP
#define RT_WSTAMP(v)                                                              \
    do {                                                                          \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");              \
        v = __builtin_amdgcn_s_memtime();                                         \
    } while (0)
#define RT_WSTEP(i) \
    do {                                                                          \
        if (static_cast<unsigned>(__builtin_amdgcn_readfirstlane(__lane_id())) == __lane_id()) ++w->wsteps[i]; \
    } while (0)
#else
#define RT_WSTAMP(v) ((void)0)
#define RT_WSTEP(i) ((void)0)
#endif

template <bool kCount = false, class SpherePtr>
__device__ __forceinline__ Hit nearest_brute(const DevScene& sc, SpherePtr S, const Ray& r, Work* w = nullptr) {
    Hit h;
    h.t = __builtin_huge_val();
    h.obj = INT32_MAX;
    h.prim = 0;
    h.nan_t = false;
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        const int32_t obj = sc.plane_obj[i];
        if (t != t) {
            if (!h.nan_t) { h.nan_t = true; h.t = t; h.obj = obj; h.prim = ~i; }
        } else if (!h.nan_t && (t < h.t || (t == h.t && obj < h.obj))) {
            h.t = t; h.obj = obj; h.prim = ~i;
        }
    }
    if (h.nan_t) return h;      // no sphere can produce a NaN t
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;     // direction.sqnorm()
    const SphK sk = sphere_k(a);
    const int n = sc.n_spheres;
    if constexpr (kCount) w->spheres += n;
#pragma unroll 2
    for (int i = 0; i < n; ++i) {
        const DevSphere s = S[i];
        double t;
        if (sphere_t(s, r, sk, t)) {
            const int32_t obj = sc.sphere_obj[i];
            if (t < h.t || (t == h.t && obj < h.obj)) { h.t = t; h.obj = obj; h.prim = i; }
        }
    }
    return h;
}

// The shadow test of raytrace.rs:41-49: `intersect(shadow ray)` is Some and
// (range is None or t*t < range).  Equivalent any-hit form:
//  * no range (directional light): shadowed iff ANY object reports a hit;
//  * with range (point light): if any plane reports a NaN t the nearest hit
//    is that NaN hit and NaN*NaN < r2 is false -> lit; otherwise shadowed iff
//    SOME hit has t*t < r2 (t_min <= t_i and rounding is monotone, so the
//    nearest one then qualifies too).
template <bool kCount = false, class SpherePtr>
__device__ __forceinline__ bool occluded_brute(const DevScene& sc, SpherePtr S, const Ray& r, bool has_range, double r2,
                                               Work* w = nullptr) {
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
    const SphK sk = sphere_k(a);
    const int n = sc.n_spheres;
    for (int i = 0; i < n; ++i) {
        const DevSphere s = S[i];
        double t;
        if constexpr (kCount) ++w->spheres;
        if (sphere_t(s, r, sk, t)) {
            if (!has_range || t * t < r2) return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------ BVH
//
// Culling must never skip a sphere the exact f64 test would report, or the
// result would differ from the reference's linear scan.  Boxes are padded and
// rounded outward on the host; here every slab interval is computed in f32
// from the f32-rounded ray and then widened by a relative kBoxTol, which
// covers the f32 rounding of origin, direction and slab arithmetic (each a few
// ulps, relative to the t values they perturb).  The slab test runs on the
// direction scaled by a power of two 2^-te that brings its largest component
// into [0.5, 1) whenever that component lies outside [2^-20, 2^20] (te = 0,
// no scaling, for the unit-length camera, reflection and point-light shadow
// rays): t' = t 2^te, exactly, and every t limit handed to the box tests is
// scaled the same way (t_limit(rb, t)).  Without it the f32 direction of a
// directional light's unnormalised shadow ray (-direction, raytrace.rs:41,
// scene.rs:131-139) or of a reflection off a plane whose normal is far from
// unit length over- or underflows, or has every component clamped (round 5:
// a light of magnitude 1e-35 culled occluders).  Direction components below
// 1e-20 of the scaled direction are clamped (no 0 * inf NaNs); such a ray
// moves < 1e-14 relative to its largest component along that axis over any
// relevant t, far below the box padding.  DESIGN.md "BVH exactness" has the
// argument in full.
constexpr float kBoxTol = 1e-5f;
constexpr int kBvhStack = 64;      // host builder bounds the depth (median splits past depth 40)
constexpr int kBvh4Stack = 64;     // 4-wide: the host checks the tree's worst case (bvh4_stack_need) against it

// f32 image of a ray for the slab tests: 1/d per axis and -o/d, so each slab
// bound is one FMA, fma(lo, 1/d, -o/d).  The FMA's rounding terms are of the
// same two kinds the tolerance argument covers: relative to t (rounding of
// 1/d and of the result) and a spatial 2^-24 |o| from rounding o/d.  te: the
// slab t values are t 2^te (see above).
struct RayBox {
    float ix, iy, iz, nox, noy, noz;
    int32_t te;
};

__device__ __forceinline__ float inv_dir(double d) {
    float f = static_cast<float>(d);
    if (!(fabsf(f) >= 1e-20f)) f = copysignf(1e-20f, f);
    return 1.0f / f;
}

#ifndef RT_DIR_SCALE
#define RT_DIR_SCALE 1      // (A/B builds only: 0 = the round-4 unscaled slab tests, not exact for such rays)
#endif
__device__ __forceinline__ RayBox make_raybox(const Ray& r) {
    const double m = fmax(fmax(fabs(r.dx), fabs(r.dy)), fabs(r.dz));
    // m = f 2^te with f in [0.5, 1) (v_frexp_exp_i32_f64); NaN and infinite directions keep
    // te = 0 (their t values are NaN anyway)
    const int32_t te = RT_DIR_SCALE && ((m > 0x1p20 && m < __builtin_huge_val()) || (m < 0x1p-20 && m > 0.0))
                           ? __builtin_amdgcn_frexp_exp(m) : 0;
    const float ix = inv_dir(ldexp(r.dx, -te)), iy = inv_dir(ldexp(r.dy, -te)), iz = inv_dir(ldexp(r.dz, -te));
    return RayBox{ix, iy, iz, -(static_cast<float>(r.ox) * ix), -(static_cast<float>(r.oy) * iy),
                  -(static_cast<float>(r.oz) * iz), te};
}

// Slab bound t at coordinate v along the axis with (1/d, -o/d) = (i, no).
__device__ __forceinline__ float slab_t(float v, float i, float no) { return __builtin_fmaf(v, i, no); }

// Interval widening by the relative kBoxTol (one FMA with an |x| modifier), or as
// one multiply by these factors where the sign cases do not matter (RT_WIDEN_MUL).
#ifndef RT_WIDEN_MUL
#define RT_WIDEN_MUL 1
#endif
constexpr float kWidenLo = 1.0f - kBoxTol;
constexpr float kWidenHi = 1.0f + kBoxTol;
__device__ __forceinline__ float widen_lo(float t) { return __builtin_fmaf(-kBoxTol, fabsf(t), t); }
__device__ __forceinline__ float widen_hi(float t) { return __builtin_fmaf(kBoxTol, fabsf(t), t); }

// Conservative slab test; tlim = largest t still of interest.
__device__ __forceinline__ bool box_hit(const float* lo, const float* hi, const RayBox& rb, float tlim, float& tnear) {
    const float ax = slab_t(lo[0], rb.ix, rb.nox), bx = slab_t(hi[0], rb.ix, rb.nox);
    const float ay = slab_t(lo[1], rb.iy, rb.noy), by = slab_t(hi[1], rb.iy, rb.noy);
    const float az = slab_t(lo[2], rb.iz, rb.noz), bz = slab_t(hi[2], rb.iz, rb.noz);
    float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    tn = widen_lo(tn);
    tf = widen_hi(tf);
    tnear = tn;
    // tn <= tf && tf >= 0 && tn <= tlim, as one compare: every caller's tlim is
    // >= 0 (+inf or t_limit of a positive t), so max(tn, 0) <= min(tf, tlim)
    // states exactly the same three conditions (fewer compares and mask ANDs)
#ifndef RT_BOXFOLD
#define RT_BOXFOLD 1
#endif
    if (RT_BOXFOLD) return fmaxf(tn, 0.0f) <= fminf(tf, tlim);
    return tn <= tf && tf >= 0.0f && tn <= tlim;
}

// An f32 bound >= t (t >= 0 or +inf), for culling boxes that start beyond t.
__device__ __forceinline__ float t_limit(double t) {
    float f = static_cast<float>(t);
    if (static_cast<double>(f) < t) f = __uint_as_float(__float_as_uint(f) + 1u);   // next f32 up (t >= 0)
    return f + kBoxTol * f;
}
// ... in the scaled t of the ray's slab tests (t 2^te, exact; te = 0 for unit-length rays)
__device__ __forceinline__ float t_limit(const RayBox& rb, double t) { return t_limit(ldexp(t, rb.te)); }

// Planes of the scene (always brute force: few, and they carry the NaN quirk).
__device__ __forceinline__ Hit nearest_planes(const DevScene& sc, const Ray& r) {
    Hit h;
    h.t = __builtin_huge_val();
    h.obj = INT32_MAX;
    h.prim = 0;
    h.nan_t = false;
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        const int32_t obj = sc.plane_obj[i];
        if (t != t) {
            if (!h.nan_t) { h.nan_t = true; h.t = t; h.obj = obj; h.prim = ~i; }
        } else if (!h.nan_t && (t < h.t || (t == h.t && obj < h.obj))) {
            h.t = t; h.obj = obj; h.prim = ~i;
        }
    }
    return h;
}

// Where the traversal reads its data: the first `nl` BVH nodes (breadth-first
// order, i.e. the top of the tree) from an LDS copy, the rest from HBM/L2;
// spheres and their object ids from LDS when the whole list fits, else HBM.
struct BvhView {
    const float2* lnodes;        // LDS nodes, axis-pair-major (stage_node_planes): 6 bound-pair arrays then the child pairs
    int32_t nl;
    const DevBvhNode* pnodes;    // prefix sources: nodes [0, nl) in LDS as DevBvhNode (array of nodes)
    const DevBvhNode* gnodes;
    const DevSphere* sph;
    const int32_t* obj;
    const DevBvh4Plane* p4;      // 4-wide tree planes (LDS or HBM), stride n4
    int32_t n4;
    const DevBvhNodeH* hpnodes;  // half-node prefix source: nodes [0, nl) in LDS (binary16 bounds)
    const DevBvhNodeH* hgnodes;  // ... and the whole half-node tree in HBM/L2
    const DevQNode4* q4l;        // quantised 4-wide tree: nodes [0, nq) in LDS, the rest from q4g (HBM/L2)
    const DevQNode4* q4g;
    int32_t nq;
};

// The view of the scene's trees and spheres in HBM (what a source does not stage in LDS).
__device__ __forceinline__ BvhView global_view(const DevScene& sc) {
    BvhView v{};
    v.gnodes = sc.bvh;
    v.sph = sc.spheres;
    v.obj = sc.sphere_obj;
    v.p4 = sc.bvh4;
    v.n4 = sc.n_bvh4;
    v.q4g = sc.q4;
    return v;
}

// LDS copy of binary nodes [0, n), AXIS-PAIR-MAJOR: for axis a the lo_a
// bounds of the two children of node i as one pair at L[(2a) * n + i] and
// the hi_a bounds at L[(2a + 1) * n + i] (float2), the child pair at
// ((int2*)(L + 6n))[i]; 56 B per node.  A ray reads only the pairs its slab
// test needs: per axis the NEAR pair (lo when 1/d_a >= 0, else hi) and the
// FAR pair, both children at once (nearest_bvh_bl), and every 8-B read of a
// wave spreads over all 32 8-B bank slots (the pair arrays have an 8-B stride).
__host__ __device__ constexpr size_t node_planes_bytes(int32_t n) { return (static_cast<size_t>(n) * 56u + 15u) / 16u * 16u; }

// kByteOff (nearest_bvh_bl's walk): an inner child c is stored as the byte
// offset (c + 1) * 8 of its pairs, so a visit addresses every array with one add
// and no shift, and 0 (an inline constant) is free to mean "no node"; leaf codes
// (negative) are unchanged.
__host__ __device__ constexpr int32_t node_byte_off(int32_t c) { return c >= 0 ? (c + 1) * 8 : c; }

template <int kThreads, bool kByteOff = false>
__device__ __forceinline__ const float2* stage_node_planes(const DevBvhNode* src, int32_t n, unsigned char* lds) {
    float2* L = reinterpret_cast<float2*>(lds);
    int2* C = reinterpret_cast<int2*>(L + 6 * n);
    for (int i = threadIdx.x; i < n; i += kThreads) {
        const DevBvhNode nd = src[i];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            L[(2 * a) * n + i] = make_float2(nd.lo0[a], nd.lo1[a]);
            L[(2 * a + 1) * n + i] = make_float2(nd.hi0[a], nd.hi1[a]);
        }
        C[i] = kByteOff ? make_int2(node_byte_off(nd.c0), node_byte_off(nd.c1)) : make_int2(nd.c0, nd.c1);
    }
    return L;
}

__device__ __forceinline__ DevBvhNode lds_node(const float2* L, int32_t n, int32_t i) {
    DevBvhNode nd;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float2 lo = L[(2 * a) * n + i], hi = L[(2 * a + 1) * n + i];
        nd.lo0[a] = lo.x; nd.lo1[a] = lo.y;
        nd.hi0[a] = hi.x; nd.hi1[a] = hi.y;
    }
    const int2 cc = reinterpret_cast<const int2*>(L + 6 * n)[i];
    nd.c0 = cc.x; nd.c1 = cc.y;
    return nd;
}

__device__ __forceinline__ float half_bits_f(uint16_t h) {
    return static_cast<float>(__builtin_bit_cast(_Float16, h));     // exact (v_cvt_f32_f16)
}

// kNodes: 0 = every node from HBM/L2, 1 = LDS prefix + HBM, 2 = every node in LDS,
// 3 = LDS prefix + HBM of binary16 nodes (DevBvhNodeH, bounds rounded outward:
// decoded exactly, each box contains the f32 node's box)
template <int kNodes>
__device__ __forceinline__ DevBvhNode fetch_node(const BvhView& v, int32_t i) {
    if constexpr (kNodes == 3) {
        const DevBvhNodeH h = *(i < v.nl ? v.hpnodes + i : v.hgnodes + i);
        DevBvhNode nd;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            nd.lo0[a] = half_bits_f(h.b[a]); nd.hi0[a] = half_bits_f(h.b[3 + a]);
            nd.lo1[a] = half_bits_f(h.b[6 + a]); nd.hi1[a] = half_bits_f(h.b[9 + a]);
        }
        nd.c0 = h.c0; nd.c1 = h.c1;
        return nd;
    } else if constexpr (kNodes == 2) {
        return lds_node(v.lnodes, v.nl, i);
    } else if constexpr (kNodes == 1) {
        // one flat load from LDS or HBM/L2: the same layout on both sides, so no
        // divergent branch (a plane-major prefix measured C4 70.8 -> 79.0 ms)
        return *(i < v.nl ? v.pnodes + i : v.gnodes + i);
    } else {
        return v.gnodes[i];
    }
}

// The private stack array must stay in scratch: an array small enough for the
// compiler to promote to registers is indexed per lane with divergent indices,
// which compiles to a waterfall loop over the wave's distinct indices (the
// 128-B compact stack measured 130x slower that way).  Passing its address to
// an empty asm statement makes it escape, so it is never promoted.  (Its 32-bit
// scratch offset, not the 64-bit generic pointer: the generic cast's null check
// hit an instruction-selection error in one kernel.)
template <class T>
__device__ __forceinline__ void rt_keep_in_scratch(T* p) {
    asm volatile("" : : "v"(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p))));
}

// Traversal stacks, declared as plain locals so the compiler keeps the stack
// pointer (and the register part) in registers.  The top kReg entries live in
// registers, shifted with v_mov on push/pop (constant indices after
// unrolling); deeper entries live in a private array (scratch, cached in
// L1/L2).  A pop refills the register part from scratch, so the load's
// latency overlaps the traversal work before the entry is needed; with
// kReg = 0 every pop waits for its scratch load.  The nearest query packs
// (node, entry t) into one 64-bit entry: one scratch access per push / pop.
// The host bounds the tree depth, so kBvhStack entries always suffice.
#define RT_STACK_DECL(kReg, E) RT_STACK_DECL_N(kReg, E, kBvhStack)
#define RT_STACK_DECL_N(kReg, E, kN)                                                   \
    E stk_m[kN];                                                                       \
    E stk_r[(kReg) > 0 ? (kReg) : 1];                                                  \
    int stk_n = 0;                                                                     \
    auto stk_push = [&](E v) {                                                         \
        if constexpr ((kReg) > 0) {                                                    \
            if (stk_n >= (kReg)) stk_m[stk_n - (kReg)] = stk_r[(kReg) - 1];            \
            _Pragma("unroll") for (int q = (kReg) - 1; q > 0; --q) stk_r[q] = stk_r[q - 1]; \
            stk_r[0] = v;                                                              \
        } else {                                                                       \
            stk_m[stk_n] = v;                                                          \
        }                                                                              \
        ++stk_n;                                                                       \
    };                                                                                 \
    auto stk_pop = [&]() -> E {                                                        \
        --stk_n;                                                                       \
        if constexpr ((kReg) > 0) {                                                    \
            const E v = stk_r[0];                                                      \
            _Pragma("unroll") for (int q = 0; q < (kReg) - 1; ++q) stk_r[q] = stk_r[q + 1]; \
            if (stk_n >= (kReg)) stk_r[(kReg) - 1] = stk_m[stk_n - (kReg)];            \
            return v;                                                                  \
        } else {                                                                       \
            return stk_m[stk_n];                                                       \
        }                                                                              \
    }

__device__ __forceinline__ uint64_t stk_entry(int32_t node, float t) {
    return (static_cast<uint64_t>(__float_as_uint(t)) << 32) | static_cast<uint32_t>(node);
}
__device__ __forceinline__ int32_t stk_node(uint64_t e) { return static_cast<int32_t>(static_cast<uint32_t>(e)); }
__device__ __forceinline__ float stk_t(uint64_t e) { return __uint_as_float(static_cast<uint32_t>(e >> 32)); }

// Compact 32-bit entries (host: every node index and leaf code fits kBits
// bits signed, depth <= kShortStack): the low kBits bits are the node / leaf
// code (sign-extended), the rest the entry t's top 32 - kBits bits (sign,
// exponent, 23 - kBits mantissa bits: 16 -> 7, 18 -> 5).  Dropping the low
// mantissa bits moves t toward zero: a non-negative t can only get smaller and
// a negative one stays negative, so `t <= tlim` (tlim > 0) culls a subset of
// what the exact t would: the same leaves that can hold the winner are
// visited, and the (t, object) winner does not depend on order.
constexpr int kShortStack = 32;
template <int kBits>
__device__ __forceinline__ uint32_t stk_entry_c(int32_t node, float t) {
    constexpr uint32_t kMask = (1u << kBits) - 1u;
    return (__float_as_uint(t) & ~kMask) | (static_cast<uint32_t>(node) & kMask);
}
template <int kBits>
__device__ __forceinline__ int32_t stk_node_c(uint32_t e) { return static_cast<int32_t>(e << (32 - kBits)) >> (32 - kBits); }
template <int kBits>
__device__ __forceinline__ float stk_t_c(uint32_t e) { return __uint_as_float(e & ~((1u << kBits) - 1u)); }

// Scene::intersect through the BVH.  Same winner as nearest_brute: candidates
// compete on (t, object id), independent of visiting order.
template <bool kCount = false, int kNodes = 0, int kReg = 0>
__device__ __forceinline__ Hit nearest_bvh(const DevScene& sc, const BvhView& v, const Ray& r, Work* w = nullptr) {
    Hit h = nearest_planes(sc, r);
    if (h.nan_t || sc.n_spheres == 0) return h;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    const RayBox rb = make_raybox(r);
    float tlim = h.obj == INT32_MAX ? __builtin_inff() : t_limit(rb, h.t);
    RT_STACK_DECL(kReg, uint64_t);
    int32_t cur = sc.bvh_root;
    for (;;) {
        if (cur >= 0) {
            const DevBvhNode nd = fetch_node<kNodes>(v, cur);
            if constexpr (kCount) w->boxes += 2;
            float t0, t1;
            const bool h0 = box_hit(nd.lo0, nd.hi0, rb, tlim, t0);
            const bool h1 = box_hit(nd.lo1, nd.hi1, rb, tlim, t1);
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                stk_push(stk_entry(first0 ? nd.c1 : nd.c0, first0 ? t1 : t0));
                cur = first0 ? nd.c0 : nd.c1;
                continue;
            }
            if (h0) { cur = nd.c0; continue; }
            if (h1) { cur = nd.c1; continue; }
        } else {
            const int first = (~cur) >> 3, cnt = ((~cur) & 7) + 1;
            if constexpr (kCount) w->spheres += cnt;
            for (int k = first; k < first + cnt; ++k) {
                double t;
                if (sphere_t(v.sph[k], r, sk, t)) {
                    const int32_t obj = v.obj[k];
                    if (t < h.t || (t == h.t && obj < h.obj)) {
                        h.t = t; h.obj = obj; h.prim = k;
                        tlim = t_limit(rb, t);
                    }
                }
            }
        }
        // pop, skipping entries that the current best already rules out
        for (;;) {
            if (stk_n == 0) return h;
            const uint64_t e = stk_pop();
            cur = stk_node(e);
            if (stk_t(e) <= tlim) break;
        }
    }
}

// nearest_bvh with the inner-node step written branch-light:
// a wave descends inner nodes in one tight loop whose only divergent
// statement is the masked push of the far child, then tests its leaf, then
// pops past the entries the current best rules out.  Same visiting order,
// culling and result as nearest_bvh.
template <bool kCount = false, int kNodes = 0, int kReg = 0, int kCompactBits = 0>
__device__ __forceinline__ Hit nearest_bvh_bl(const DevScene& sc, const BvhView& v, const Ray& r, Work* w = nullptr) {
    Hit h = nearest_planes(sc, r);
    if (h.nan_t || sc.n_spheres == 0) return h;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    const RayBox rb = make_raybox(r);
    float tlim = h.obj == INT32_MAX ? __builtin_inff() : t_limit(rb, h.t);
    // not a node and no leaf code: INT32_MIN (~cur would list 8 spheres at 2^28), or 0 for the
    // byte-offset nodes of the whole-LDS walk (node c is (c + 1) * 8)
    constexpr int32_t kNone = kNodes == 2 ? 0 : INT32_MIN;
    // kReg newest entries in registers (the LDS-prefix source), the rest in scratch;
    // kCompactBits > 0: 32-bit entries with that many code bits, kShortStack of them
    // (128 B of scratch per lane); 0: 64-bit (node, t) entries
    constexpr bool kCompact = kCompactBits > 0;
    using StkE = std::conditional_t<kCompact, uint32_t, uint64_t>;
    RT_STACK_DECL_N(kReg, StkE, (kCompact ? kShortStack : kBvhStack));
    if constexpr (kCompact) rt_keep_in_scratch(stk_m);
    auto mk_entry = [](int32_t node, float t) -> StkE {
        if constexpr (kCompact) return stk_entry_c<kCompactBits>(node, t); else return stk_entry(node, t);
    };
    auto e_node = [](StkE e) -> int32_t {
        if constexpr (kCompact) return stk_node_c<kCompactBits>(e); else return stk_node(e);
    };
    auto e_t = [](StkE e) -> float {
        if constexpr (kCompact) return stk_t_c<kCompactBits>(e); else return stk_t(e);
    };
    // whole tree in LDS (kNodes 2): nodes as byte offsets (stage_node_planes<., true>), 0 = none
    int32_t cur = kNodes == 2 ? node_byte_off(sc.bvh_root) : sc.bvh_root;
    [[maybe_unused]] unsigned long long q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    // whole tree in LDS: per axis the array of NEAR bound pairs (lo when 1/d >= 0,
    // else hi) and of FAR pairs.  fma(v, 1/d, -o/d) is monotone in v for a fixed
    // ray (1/d != 0), so fma(near) = min(fma(lo), fma(hi)) exactly: box_hit's
    // interval, without its six min/max per child.  Byte bases one pair before
    // node 0, so node byte offset (c + 1) * 8 addresses pair c.
    [[maybe_unused]] const char *nxa = nullptr, *fxa = nullptr, *nya = nullptr, *fya = nullptr, *nza = nullptr,
                                *fza = nullptr, *ca = nullptr;
    if constexpr (kNodes == 2) {
        const char* L = reinterpret_cast<const char*>(v.lnodes) - 8;
        const size_t n8 = static_cast<size_t>(v.nl) * 8;
        nxa = L + (rb.ix >= 0.0f ? 0 : n8); fxa = L + (rb.ix >= 0.0f ? n8 : 0);
        nya = L + 2 * n8 + (rb.iy >= 0.0f ? 0 : n8); fya = L + 2 * n8 + (rb.iy >= 0.0f ? n8 : 0);
        nza = L + 4 * n8 + (rb.iz >= 0.0f ? 0 : n8); fza = L + 4 * n8 + (rb.iz >= 0.0f ? n8 : 0);
        ca = L + 6 * n8;
    }
    for (;;) {
        RT_WSTAMP(q0);
        while (kNodes == 2 ? cur > 0 : cur >= 0) {
            RT_WSTEP(0);
            float t0, t1;
            bool h0, h1;
            int32_t c0, c1;
            if constexpr (kNodes == 2) {
                auto pair = [cur](const char* base) { return *reinterpret_cast<const float2*>(base + cur); };
                const float2 nx = pair(nxa), fx = pair(fxa), ny = pair(nya), fy = pair(fya), nz = pair(nza), fz = pair(fza);
                const int2 cc = *reinterpret_cast<const int2*>(ca + cur);
                const float a0 = fmaxf(fmaxf(slab_t(nx.x, rb.ix, rb.nox), slab_t(ny.x, rb.iy, rb.noy)), slab_t(nz.x, rb.iz, rb.noz));
                const float a1 = fmaxf(fmaxf(slab_t(nx.y, rb.ix, rb.nox), slab_t(ny.y, rb.iy, rb.noy)), slab_t(nz.y, rb.iz, rb.noz));
                const float b0 = fminf(fminf(slab_t(fx.x, rb.ix, rb.nox), slab_t(fy.x, rb.iy, rb.noy)), slab_t(fz.x, rb.iz, rb.noz));
                const float b1 = fminf(fminf(slab_t(fx.y, rb.ix, rb.nox), slab_t(fy.y, rb.iy, rb.noy)), slab_t(fz.y, rb.iz, rb.noz));
#if RT_WIDEN_MUL
                // the relative widening as one multiply per bound (§4 item 2): t (1 - tol) for the
                // entry, f (1 + tol) for the exit.  Where the two forms differ (t or f < 0) the
                // compare below clamps t to 0 and a negative exit fails either way; +inf stays +inf
                t0 = a0 * kWidenLo; t1 = a1 * kWidenLo;
                const float f0 = b0 * kWidenHi, f1 = b1 * kWidenHi;
#else
                t0 = widen_lo(a0); t1 = widen_lo(a1);
                const float f0 = widen_hi(b0), f1 = widen_hi(b1);
#endif
                // box_hit's folded test max(t, 0) <= min(f, tlim) as two compares: tlim is never
                // NaN, and !(x > f) holds for a NaN f as min(f, tlim) = tlim does (no
                // canonicalisation of tlim per visit, no min)
                const float x0 = fmaxf(t0, 0.0f), x1 = fmaxf(t1, 0.0f);
                h0 = x0 <= tlim && !(x0 > f0);
                h1 = x1 <= tlim && !(x1 > f1);
                c0 = cc.x;
                c1 = cc.y;
            } else {
                const DevBvhNode nd = fetch_node<kNodes>(v, cur);
                h0 = box_hit(nd.lo0, nd.hi0, rb, tlim, t0);
                h1 = box_hit(nd.lo1, nd.hi1, rb, tlim, t1);
                c0 = nd.c0;
                c1 = nd.c1;
            }
            if constexpr (kCount) w->boxes += 2;
            const bool first0 = t0 <= t1;
            if (h0 && h1) stk_push(mk_entry(first0 ? c1 : c0, first0 ? t1 : t0));
            cur = (h0 && (!h1 || first0)) ? c0 : (h1 ? c1 : kNone);
        }
        RT_WSTAMP(q1);
        if (cur != kNone) {
            const int first = (~cur) >> 3, cnt = ((~cur) & 7) + 1;
            if constexpr (kCount) w->spheres += cnt;
            for (int k = first; k < first + cnt; ++k) {
                RT_WSTEP(1);
                double t;
                if (sphere_t<kNodes == 3 ? (RT_BF_HALF != 0) : kNodes == 2 ? (RT_BF_LDS != 0) : (RT_ROOTS_BF != 0)>(v.sph[k], r, sk, t)) {
                    const int32_t obj = v.obj[k];
                    if (t < h.t || (t == h.t && obj < h.obj)) {
                        h.t = t; h.obj = obj; h.prim = k;
                        tlim = t_limit(rb, t);
                    }
                }
            }
        }
        RT_WSTAMP(q2);
        cur = kNone;
        while (stk_n > 0) {
            RT_WSTEP(2);
            const StkE e = stk_pop();
            if (e_t(e) <= tlim) { cur = e_node(e); break; }
        }
        RT_WSTAMP(q3);
#if RT_STAMP
        w->cyc[0] += q1 - q0; w->cyc[1] += q2 - q1; w->cyc[2] += q3 - q2;
#endif
        if (cur == kNone) return h;
    }
}

// The shadow query (see occluded_brute for the any-hit equivalence).
template <bool kCount = false, int kNodes = 0, int kReg = 0>
__device__ __forceinline__ bool occluded_bvh(const DevScene& sc, const BvhView& v, const Ray& r, bool has_range,
                                             double r2, int32_t hint = -1, Work* w = nullptr) {
    bool plane_block = false;
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        if (!has_range) return true;
        if (t != t) return false;
        plane_block |= t * t < r2;
    }
    if (plane_block) return true;
    if (sc.n_spheres == 0) return false;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    if (hint >= 0) {                     // see occluded_bvh4
        if constexpr (kCount) ++w->spheres;
        double t;
        if (sphere_t(v.sph[hint], r, sk, t) && (!has_range || t * t < r2)) return true;
    }
    const RayBox rb = make_raybox(r);
    // t*t < r2 implies t < sqrt(r2) (up to rounding, covered by t_limit's margin)
    const float tlim = has_range ? t_limit(rb, sqrt(r2)) : __builtin_inff();
    RT_STACK_DECL(kReg, int32_t);
    int32_t cur = sc.bvh_root;
    for (;;) {
        if (cur >= 0) {
            const DevBvhNode nd = fetch_node<kNodes>(v, cur);
            if constexpr (kCount) w->boxes += 2;
            float t0, t1;
            const bool h0 = box_hit(nd.lo0, nd.hi0, rb, tlim, t0);
            const bool h1 = box_hit(nd.lo1, nd.hi1, rb, tlim, t1);
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                stk_push(first0 ? nd.c1 : nd.c0);
                cur = first0 ? nd.c0 : nd.c1;
                continue;
            }
            if (h0) { cur = nd.c0; continue; }
            if (h1) { cur = nd.c1; continue; }
        } else {
            const int first = (~cur) >> 3, cnt = ((~cur) & 7) + 1;
            if constexpr (kCount) w->spheres += cnt;
            for (int k = first; k < first + cnt; ++k) {
                double t;
                if (sphere_t(v.sph[k], r, sk, t) && (!has_range || t * t < r2)) return true;
            }
        }
        if (stk_n == 0) return false;
        cur = stk_pop();
    }
}

// ---- 4-wide BVH --------------------------------------------------------
// One node visit tests the 4 child boxes (same conservative slab test); the
// shadow query takes the hit children in slot order.  Misses are marked by the child pointer (kBvh4Empty), never by t, so a box
// hit at t = +inf is still visited.
struct Node4Hits {
    float t[4];
    int32_t c[4];
};

__device__ __forceinline__ Node4Hits node4_test(const BvhView& v, int32_t node, const RayBox& rb, float tlim) {
    // axis by axis (as box_hit, same operations), so only two planes are live at a time
    const int32_t N = v.n4;
    const DevBvh4Plane* P = v.p4 + node;
    float tn[4], tf[4];
    {
        const DevBvh4Plane lo = P[0], hi = P[N];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = slab_t(lo.f[k], rb.ix, rb.nox), b = slab_t(hi.f[k], rb.ix, rb.nox);
            tn[k] = fminf(a, b);
            tf[k] = fmaxf(a, b);
        }
    }
    {
        const DevBvh4Plane lo = P[2 * N], hi = P[3 * N];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = slab_t(lo.f[k], rb.iy, rb.noy), b = slab_t(hi.f[k], rb.iy, rb.noy);
            tn[k] = fmaxf(tn[k], fminf(a, b));
            tf[k] = fminf(tf[k], fmaxf(a, b));
        }
    }
    {
        const DevBvh4Plane lo = P[4 * N], hi = P[5 * N];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = slab_t(lo.f[k], rb.iz, rb.noz), b = slab_t(hi.f[k], rb.iz, rb.noz);
            tn[k] = fmaxf(tn[k], fminf(a, b));
            tf[k] = fminf(tf[k], fmaxf(a, b));
        }
    }
    const DevBvh4Plane ch = P[6 * N];
    Node4Hits o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float n = widen_lo(tn[k]);
        const float f = widen_hi(tf[k]);
        const bool hit = n <= f && f >= 0.0f && n <= tlim && ch.i[k] != kBvh4Empty;
        o.t[k] = hit ? n : __builtin_inff();
        o.c[k] = hit ? ch.i[k] : kBvh4Empty;
    }
    return o;
}

// ---- quantised 4-wide tree (DevQNode4) -----------------------------------------
// Scene::intersect (scene.rs:247-249) through the 4-wide tree whose child boxes
// are 8-bit multiples of a per-node power-of-two step (host_bvh.cpp
// quantize_bvh4).  A bound decodes exactly: fma(q, s, m * s) = (m + q) * s is an
// f32 value (|m + q| < 2^24, s a power of two in the normal range), and it lies
// outside the f32 child box (rounded outward), so the slab test below is the
// f32 tree's test on a box that contains that one: it culls a subset of what
// the f32 test culls.  The nearest hit child is
// entered first, the other hit children pushed far-to-near (64-bit entries:
// the entry t and the node index, or kQ4LeafTag | first << 3 | count - 1);
// leaves get the exact f64 test and the winner is the lexicographic (t,
// object id) minimum over every tested sphere, as for the binary tree.
// kAll: every node in LDS (ds reads); else nodes [0, nq) from LDS and the rest
// through L2 by one flat load (the same 48-B layout on both sides).
constexpr uint32_t kQ4LeafTag = 0x80000000u;

__device__ __forceinline__ float q4_step(int32_t f) { return __uint_as_float((static_cast<uint32_t>(f) >> 24) << 23); }
__device__ __forceinline__ float q4_byte(uint32_t w, int k) { return static_cast<float>((w >> (8 * k)) & 0xFFu); }

template <bool kCount = false, bool kAll = true>
__device__ __forceinline__ Hit nearest_q4(const DevScene& sc, const BvhView& v, const Ray& r, Work* w = nullptr) {
    Hit h = nearest_planes(sc, r);
    if (h.nan_t || sc.n_spheres == 0) return h;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    const RayBox rb = make_raybox(r);
    float tlim = h.obj == INT32_MAX ? __builtin_inff() : t_limit(rb, h.t);
    const bool fx = rb.ix < 0.0f, fy = rb.iy < 0.0f, fz = rb.iz < 0.0f;     // near slab bound = hi
    RT_STACK_DECL_N(0, uint64_t, kQ4Stack);
    rt_keep_in_scratch(stk_m);
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    uint32_t cur = 0;                                            // the root: inner node 0
    for (;;) {
        while (cur < kQ4LeafTag) {
            DevQNode4 nd;
            if constexpr (kAll) nd = v.q4l[cur];
            else nd = *(static_cast<int32_t>(cur) < v.nq ? v.q4l + cur : v.q4g + cur);
            const float sx = q4_step(nd.frame[0]), sy = q4_step(nd.frame[1]), sz = q4_step(nd.frame[2]);
            const float ox = static_cast<float>((nd.frame[0] << 8) >> 8) * sx;      // m * s, exact
            const float oy = static_cast<float>((nd.frame[1] << 8) >> 8) * sy;
            const float oz = static_cast<float>((nd.frame[2] << 8) >> 8) * sz;
            const uint32_t nxw = fx ? nd.hi[0] : nd.lo[0], fxw = fx ? nd.lo[0] : nd.hi[0];
            const uint32_t nyw = fy ? nd.hi[1] : nd.lo[1], fyw = fy ? nd.lo[1] : nd.hi[1];
            const uint32_t nzw = fz ? nd.hi[2] : nd.lo[2], fzw = fz ? nd.lo[2] : nd.hi[2];
            float t[4];
            uint32_t c[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float tn = fmaxf(fmaxf(slab_t(__builtin_fmaf(q4_byte(nxw, k), sx, ox), rb.ix, rb.nox),
                                             slab_t(__builtin_fmaf(q4_byte(nyw, k), sy, oy), rb.iy, rb.noy)),
                                       slab_t(__builtin_fmaf(q4_byte(nzw, k), sz, oz), rb.iz, rb.noz));
                const float tf = fminf(fminf(slab_t(__builtin_fmaf(q4_byte(fxw, k), sx, ox), rb.ix, rb.nox),
                                             slab_t(__builtin_fmaf(q4_byte(fyw, k), sy, oy), rb.iy, rb.noy)),
                                       slab_t(__builtin_fmaf(q4_byte(fzw, k), sz, oz), rb.iz, rb.noz));
                const float n = widen_lo(tn);
                const uint32_t ref = nd.child[k];
                const bool hit = fmaxf(n, 0.0f) <= fminf(widen_hi(tf), tlim) && ref != kQ4Empty;
                t[k] = hit ? n : __builtin_inff();
                c[k] = !hit ? kNone
                       : ref < kQ4Leaf ? ref
                                       : kQ4LeafTag | ((nd.base + ((ref >> 3) & 0xFFFu)) << 3) | (ref & 7u);
            }
            if constexpr (kCount) w->boxes += 4;
            // near-to-far: misses (t = +inf, c = kNone) sort last
#define RT_Q4CAS(i, j)                                                              \
            {                                                                       \
                const bool sw = t[j] < t[i];                                        \
                const float ti = t[i]; const uint32_t ci = c[i];                    \
                t[i] = sw ? t[j] : ti; c[i] = sw ? c[j] : ci;                       \
                t[j] = sw ? ti : t[j]; c[j] = sw ? ci : c[j];                       \
            }
            RT_Q4CAS(0, 1) RT_Q4CAS(2, 3) RT_Q4CAS(0, 2) RT_Q4CAS(1, 3) RT_Q4CAS(1, 2)
#undef RT_Q4CAS
#pragma unroll
            for (int k = 3; k >= 1; --k)
                if (c[k] != kNone) stk_push(stk_entry(static_cast<int32_t>(c[k]), t[k]));
            cur = c[0];
        }
        if (cur != kNone) {
            const int first = static_cast<int>((cur & ~kQ4LeafTag) >> 3), cnt = static_cast<int>(cur & 7u) + 1;
            if constexpr (kCount) w->spheres += cnt;
            for (int k = first; k < first + cnt; ++k) {
                double tt;
                if (sphere_t(v.sph[k], r, sk, tt)) {
                    const int32_t obj = v.obj[k];
                    if (tt < h.t || (tt == h.t && obj < h.obj)) {
                        h.t = tt; h.obj = obj; h.prim = k;
                        tlim = t_limit(rb, tt);
                    }
                }
            }
        }
        cur = kNone;
        while (stk_n > 0) {
            const uint64_t e = stk_pop();
            if (stk_t(e) <= tlim) { cur = static_cast<uint32_t>(stk_node(e)); break; }
        }
        if (cur == kNone) return h;
    }
}

// `hint`: a sphere (leaf-order index, or -1) tested before the traversal: the
// sphere the shadow ray starts on, which occludes it whenever the light is
// behind that surface.  Any-hit: testing one sphere early cannot change the
// answer (and the planes, with the NaN rule, are decided before it).
template <bool kCount = false>
__device__ __forceinline__ bool occluded_bvh4(const DevScene& sc, const BvhView& v, const Ray& r, bool has_range,
                                              double r2, int32_t hint, Work* w = nullptr) {
    bool plane_block = false;
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        if (!has_range) return true;
        if (t != t) return false;
        plane_block |= t * t < r2;
    }
    if (plane_block) return true;
    if (sc.n_spheres == 0) return false;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    if (hint >= 0) {
        if constexpr (kCount) ++w->spheres;
        double t;
        if (sphere_t(v.sph[hint], r, sk, t) && (!has_range || t * t < r2)) return true;
    }
    const RayBox rb = make_raybox(r);
    const float tlim = has_range ? t_limit(rb, sqrt(r2)) : __builtin_inff();
    // pushes are unconditional stores at the stack top (junk when nothing is
    // pushed; the next push overwrites it): no branch per child
    int32_t stk_m[kBvh4Stack];
    int stk_n = 0;
    int32_t cur = sc.bvh4_root;
    for (;;) {
        if (cur >= 0) {
            // slot order (measured: near-to-far sorting costs more than it saves here)
            const Node4Hits n = node4_test(v, cur, rb, tlim);
            if constexpr (kCount) w->boxes += 4;
            int32_t next = kBvh4Empty;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool hk = n.c[k] != kBvh4Empty;
                if (hk && next != kBvh4Empty) stk_m[stk_n++] = next;
                next = hk ? n.c[k] : next;
            }
            if (next != kBvh4Empty) { cur = next; continue; }
        } else {
            const int first = (~cur) >> 3, cnt = ((~cur) & 7) + 1;
            if constexpr (kCount) w->spheres += cnt;
            for (int k = first; k < first + cnt; ++k) {
                double t;
                if (sphere_t(v.sph[k], r, sk, t) && (!has_range || t * t < r2)) return true;
            }
        }
        if (stk_n == 0) return false;
        cur = stk_m[--stk_n];
    }
}

// ---- point-light shadows through the light-view grid ---------------------
// The shadow query of occluded_bvh4 for a point light (has_range), with the
// spheres taken from the light's grid (host_lightgrid.cpp) instead of a tree:
// the always list, then the list of the cell that p's direction from the light
// falls in, in increasing box distance from the light, stopping at the first
// box farther than p (no blocker can be farther from the light than p is).
// Every sphere that could report a blocking hit is on those lists, and each is
// tested with the exact quadratic, so the any-hit answer is the linear scan's.
// A degenerate direction (p at the light, non-finite) tests every sphere.
template <bool kCount = false>
__device__ __forceinline__ bool occluded_lgrid(const DevScene& sc, const BvhView& v, const DevLightGrid& g,
                                               const Ray& r, double r2, double ptx, double pty, double ptz,
                                               int32_t hint, Work* w = nullptr) {
    bool plane_block = false;
    for (int i = 0; i < sc.n_planes; ++i) {
        double t;
        if (!plane_t(sc.planes[i], r, t)) continue;
        if (t != t) return false;                  // the NaN hit is the nearest: t*t < r2 fails (lit)
        plane_block |= t * t < r2;
    }
    if (plane_block) return true;
    if (sc.n_spheres == 0) return false;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    auto blocks = [&](int32_t k) {
        if constexpr (kCount) ++w->spheres;
        double t;
        return sphere_t(v.sph[k], r, sk, t) && t * t < r2;
    };
    if (hint >= 0 && blocks(hint)) return true;
    for (uint32_t e = g.always_begin; e < g.always_end; ++e)
        if (blocks(sc.lg_ent[e].sph)) return true;
    const float dx = static_cast<float>(ptx - g.lx), dy = static_cast<float>(pty - g.ly),
                dz = static_cast<float>(ptz - g.lz);
    const float ax = fabsf(dx), ay = fabsf(dy), az = fabsf(dz);
    const int fa = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    const float da = fa == 0 ? dx : fa == 1 ? dy : dz;
    const float db = fa == 0 ? dy : fa == 1 ? dz : dx;
    const float dc = fa == 0 ? dz : fa == 1 ? dx : dy;
    if (!(fabsf(da) > 0.0f && fabsf(da) < 3.0e38f)) {
        for (int32_t k = 0; k < sc.n_spheres; ++k)
            if (blocks(k)) return true;
        return false;
    }
    const int f = 2 * fa + (da < 0.0f ? 1 : 0);
    const float inv = 1.0f / fabsf(da);
    const float R = static_cast<float>(g.R);
    const int ci = min(max(static_cast<int>(floorf((db * inv + 1.0f) * 0.5f * R)), 0), g.R - 1);
    const int cj = min(max(static_cast<int>(floorf((dc * inv + 1.0f) * 0.5f * R)), 0), g.R - 1);
    const int li = ci - g.fx0[f], lj = cj - g.fy0[f];
    if (li < 0 || lj < 0 || li >= g.fw[f] || lj >= g.fh[f]) return false;    // no sphere in this direction
    const uint32_t cell = g.off_base[f] + static_cast<uint32_t>(lj * g.fw[f] + li);
    const uint32_t e0 = sc.lg_off[cell], e1 = sc.lg_off[cell + 1];
    const float dist = sqrtf(dx * dx + dy * dy + dz * dz) * 1.00001f + 1e-5f;     // >= |p - L|
    for (uint32_t e = e0; e < e1; ++e) {
        const DevLgEntry en = sc.lg_ent[e];
        if (en.near > dist) break;
        if (blocks(en.sph)) return true;
    }
    return false;
}

// ---- generation 0: the camera's view grid --------------------------------
// Scene::intersect for a camera ray (origin = the camera position) through the
// camera's view grid (host_lightgrid.cpp build_view_grid): the planes, the
// always list, then the ray direction's cell in increasing box distance from
// the camera, stopping at the first entry whose distance bound exceeds the
// current best t (t_limit margin).  A reported hit point lies in its sphere's
// padded box and in the ray direction from the camera, so its sphere is on
// that cell's list, and its distance from the camera (t |d|, |d| = 1 up to
// rounding) is at least the entry's bound: every sphere that could win or tie
// is tested with the exact quadratic, and the (t, object id) minimum is the
// linear scan's (scene.rs:247-249).  A degenerate direction
// tests every sphere.
template <bool kCount = false>
__device__ __forceinline__ Hit nearest_cgrid(const DevScene& sc, const BvhView& v, const Ray& r, Work* w = nullptr) {
    Hit h = nearest_planes(sc, r);
    if (h.nan_t || sc.n_spheres == 0) return h;
    const double a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    const SphK sk = sphere_k(a);
    const DevLightGrid& g = *sc.cgrid;
    float lim = h.obj == INT32_MAX ? __builtin_inff() : t_limit(h.t);
    auto test = [&](int32_t k) {
        if constexpr (kCount) ++w->spheres;
        double t;
        if (sphere_t(v.sph[k], r, sk, t)) {
            const int32_t obj = v.obj[k];
            if (t < h.t || (t == h.t && obj < h.obj)) { h.t = t; h.obj = obj; h.prim = k; lim = t_limit(t); }
        }
    };
    for (uint32_t e = g.always_begin; e < g.always_end; ++e) test(sc.cg_ent[e].sph);
    const float dx = static_cast<float>(r.dx), dy = static_cast<float>(r.dy), dz = static_cast<float>(r.dz);
    const float ax = fabsf(dx), ay = fabsf(dy), az = fabsf(dz);
    const int fa = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    const float da = fa == 0 ? dx : fa == 1 ? dy : dz;
    const float db = fa == 0 ? dy : fa == 1 ? dz : dx;
    const float dc = fa == 0 ? dz : fa == 1 ? dx : dy;
    if (!(fabsf(da) > 0.0f && fabsf(da) < 3.0e38f)) {
        for (int32_t k = 0; k < sc.n_spheres; ++k) test(k);
        return h;
    }
    const int f = 2 * fa + (da < 0.0f ? 1 : 0);
    const float inv = 1.0f / fabsf(da);
    const float R = static_cast<float>(g.R);
    const int ci = min(max(static_cast<int>(floorf((db * inv + 1.0f) * 0.5f * R)), 0), g.R - 1);
    const int cj = min(max(static_cast<int>(floorf((dc * inv + 1.0f) * 0.5f * R)), 0), g.R - 1);
    const int li = ci - g.fx0[f], lj = cj - g.fy0[f];
    if (li < 0 || lj < 0 || li >= g.fw[f] || lj >= g.fh[f]) return h;        // no sphere box in this direction
    const uint32_t cell = g.off_base[f] + static_cast<uint32_t>(lj * g.fw[f] + li);
    const uint32_t e0 = sc.cg_off[cell], e1 = sc.cg_off[cell + 1];
    for (uint32_t e = e0; e < e1; ++e) {
        const DevLgEntry en = sc.cg_ent[e];
        if (en.near > lim) break;
        test(en.sph);
    }
    return h;
}

// The surface normal the reference's intersect() returned for the winner:
// sphere normalize(ray.cast(t) - center) (shapes.rs:61,66); plane: as in the
// file (shapes.rs:108).  pt == ray.cast(t) bit-for-bit.
__device__ __forceinline__ void hit_normal(const DevScene& sc, const DevSphere* S, int32_t prim, double ptx, double pty,
                                           double ptz, double& nx, double& ny, double& nz) {
    if (prim >= 0) {
        const DevSphere s = S[prim];
        const double ux = ptx - s.cx, uy = pty - s.cy, uz = ptz - s.cz;
#if RT_DIVK
        const DivK l = div_k(sqrt_win(ux * ux + uy * uy + uz * uz));
        nx = div_by(ux, l); ny = div_by(uy, l); nz = div_by(uz, l);
#else
        const double l = sqrt(ux * ux + uy * uy + uz * uz);
        nx = ux / l; ny = uy / l; nz = uz / l;
#endif
    } else {
        const DevPlane& p = sc.planes[~prim];
        nx = p.nx; ny = p.ny; nz = p.nz;
    }
}

// Light direction and squared range (scene.rs:122-138).  Returns has_range.
__device__ __forceinline__ bool light_dir(const DevLight& L, double ptx, double pty, double ptz, double& lx, double& ly,
                                          double& lz, double& r2) {
    if (L.kind == 0) {                       // PointLight
        const double vx = L.v[0] - ptx, vy = L.v[1] - pty, vz = L.v[2] - ptz;
        r2 = vx * vx + vy * vy + vz * vz;    // location.sqdist(pt)
#if RT_DIVK
        const DivK l = div_k(sqrt_win(r2));  // == norm of the same vector
        lx = div_by(vx, l); ly = div_by(vy, l); lz = div_by(vz, l);
#else
        const double l = sqrt(r2);           // == norm of the same vector
        lx = vx / l; ly = vy / l; lz = vz / l;
#endif
        return true;
    }
    lx = -L.v[0]; ly = -L.v[1]; lz = -L.v[2];  // DirectionalLight: -direction, not normalised
    r2 = 0.0;
    return false;
}

// FresnelMaterial's Schlick factor from the UNflipped n.d (raytrace.rs:128-136),
// in the reference's operation order.
__device__ __forceinline__ double fresnel_factor(const DevMaterial& m, double nd) {
    double r0 = (m.ior - 1.0) / (m.ior + 1.0);
    r0 = r0 * r0;
    const double omcos = 1.0 - fabs(nd);
    const double omcos2 = omcos * omcos;
    const double f = r0 + (((1.0 - r0) * omcos2) * omcos2) * omcos;
    return f > 1.0 ? 1.0 : f;                                       // clamp_one, raytrace.rs:26-28
}

// The per-hit flags of PhongMaterial / FresnelMaterial::color.  `f` is the
// Fresnel factor (1.0 for Phong): every Fresnel expression multiplies the
// Phong one by f in a position where x * 1.0 == x exactly, so one code path
// reproduces both materials bit for bit.
struct Shading {
    bool diffuse, specular;
    double f;
};

// kFresnel = false: the scene has no FresnelMaterial (f is the constant 1.0).
template <bool kFresnel = true>
__device__ __forceinline__ Shading shading_flags(const DevMaterial& m, double sig, double nd) {
    Shading s;
    s.f = kFresnel && m.kind == kMatFresnel ? fresnel_factor(m, nd) : 1.0;
    s.diffuse = m.kd_sig * sig > kMinSignificance;                  // raytrace.rs:35 / 137
    s.specular = (m.ks_sig * s.f) * sig > kMinSignificance;         // raytrace.rs:36 / 138
    return s;
}

// The diffuse and specular terms of one unshadowed light (raytrace.rs:51-56,
// Fresnel: 151-156, where the specular term is ((ks * lc) * f) * pow).
__device__ __forceinline__ void add_light(Col& res, const DevMaterial& m, const DevLight& L, bool diffuse, bool specular,
                                          double f, double lx, double ly, double lz, double nx, double ny, double nz,
                                          double dx, double dy, double dz) {
    if (diffuse) {
        const double s = clamp_zero(lx * nx + ly * ny + lz * nz);
        res.r = res.r + ((m.kd[0] * L.color[0]) * s) * kFrac1Pi;
        res.g = res.g + ((m.kd[1] * L.color[1]) * s) * kFrac1Pi;
        res.b = res.b + ((m.kd[2] * L.color[2]) * s) * kFrac1Pi;
    }
    if (specular) {
        const double hx = lx - dx, hy = ly - dy, hz = lz - dz;
#if RT_DIVK
        const DivK hl = div_k(sqrt_win(hx * hx + hy * hy + hz * hz));
        const double c = clamp_zero(nx * div_by(hx, hl) + ny * div_by(hy, hl) + nz * div_by(hz, hl));
#else
        const double hl = sqrt(hx * hx + hy * hy + hz * hz);
        const double c = clamp_zero(nx * (hx / hl) + ny * (hy / hl) + nz * (hz / hl));
#endif
        const double p = pow(c, m.exponent);
        res.r = res.r + ((m.ks[0] * L.color[0]) * f) * p;
        res.g = res.g + ((m.ks[1] * L.color[1]) * f) * p;
        res.b = res.b + ((m.ks[2] * L.color[2]) * f) * p;
    }
}

// Pixel -> camera ray (main.rs:50-53; camera.rs:78) of AA sample 0: the
// centre jitter, or the keyed draws of the pixel's first sample (fp.jitter;
// the chain schedules take random jitter only with one sample per pixel).
__device__ __forceinline__ Ray camera_ray(const DevScene& sc, const FrameParams& fp, uint32_t lx, uint32_t local_row) {
    const uint32_t x = fp.x0 + lx;
    const uint32_t y = fp.y0 + ((local_row / fp.band) * fp.band_stride + fp.band_phase) * fp.band + local_row % fp.band;
    double jx = 0.5, jy = 0.5;
    if (fp.jitter) {
        const uint64_t ka = key_child(key_pixel(fp.seed, x, y), 0);
        jx = key_f64(ka, 0);
        jy = key_f64(ka, 1);
    }
    const double px = ((static_cast<double>(x) + jx) - fp.hw) * fp.scale;
    const double py = ((static_cast<double>(y) + jy) - fp.hh) * fp.scale;
    const double* M = sc.cam_m;
    const double dx = M[0] * px + M[1] * py + M[2] * 1.0;
    const double dy = M[3] * px + M[4] * py + M[5] * 1.0;
    const double dz = M[6] * px + M[7] * py + M[8] * 1.0;
#if RT_DIVK
    const DivK l = div_k(sqrt_win(dx * dx + dy * dy + dz * dz));
    return Ray{sc.cam_pos[0], sc.cam_pos[1], sc.cam_pos[2], div_by(dx, l), div_by(dy, l), div_by(dz, l)};
#else
    const double l = sqrt(dx * dx + dy * dy + dz * dz);
    return Ray{sc.cam_pos[0], sc.cam_pos[1], sc.cam_pos[2], dx / l, dy / l, dz / l};
#endif
}

// Mirror direction and the offset origin of raytrace.rs:60-62.
__device__ __forceinline__ Ray reflect_ray(const Ray& r, double ptx, double pty, double ptz, double nx, double ny,
                                           double nz) {
    const double dn = r.dx * nx + r.dy * ny + r.dz * nz;
    const double k2 = 2.0 * dn;
    const double rdx = r.dx - nx * k2, rdy = r.dy - ny * k2, rdz = r.dz - nz * k2;
    return Ray{ptx + rdx * kEps, pty + rdy * kEps, ptz + rdz * kEps, rdx, rdy, rdz};
}

// Final colour of a pixel from its spp identical centre-jitter samples
// (raytrace.rs:271-275, main.rs:47-56): res = BLACK; res += (BLACK + c)/1 per
// sample; res / spp.
__device__ __forceinline__ Col average_samples(Col c, uint32_t spp) {
    c = Col{(0.0 + c.r) / 1.0, (0.0 + c.g) / 1.0, (0.0 + c.b) / 1.0};
    Col res{0.0, 0.0, 0.0};
    for (uint32_t k = 0; k < spp; ++k) res = Col{res.r + c.r, res.g + c.g, res.b + c.b};
    const double aa = static_cast<double>(spp);
    return Col{res.r / aa, res.g / aa, res.b / aa};
}

__device__ __forceinline__ void write_pixel(const FrameParams& fp, uint32_t lx, uint32_t out_row, Col res,
                                            const double* srgb = c_srgb_avg) {
    const size_t p = static_cast<size_t>(out_row) * fp.tile_w + lx;
    if (fp.out_rgb) {
        fp.out_rgb[3 * p + 0] = static_cast<float>(res.r);
        fp.out_rgb[3 * p + 1] = static_cast<float>(res.g);
        fp.out_rgb[3 * p + 2] = static_cast<float>(res.b);
    }
    if (fp.out_bgr) {
        uint8_t* q = fp.out_bgr + static_cast<size_t>(out_row) * fp.bgr_pitch + 3u * lx;
        q[0] = to_srgb(res.b, srgb);
        q[1] = to_srgb(res.g, srgb);
        q[2] = to_srgb(res.r, srgb);
        if (lx == fp.tile_w - 1)       // BMP row padding is zero (main.rs:42)
            for (uint32_t k = 3u * fp.tile_w; k < fp.bgr_pitch; ++k)
                fp.out_bgr[static_cast<size_t>(out_row) * fp.bgr_pitch + k] = 0;
    }
}

// AreaLight (scene.rs:142-155): a PointLight at origin + side1*u + side2*w, u
// drawn before w, both keyed on the hit's path key and the light's index.
__device__ __forceinline__ bool light_dir_keyed(const DevLight& L, int l, uint64_t key, double ptx, double pty, double ptz,
                                                double& lx, double& ly, double& lz, double& r2) {
    if (L.kind != kLightArea) return light_dir(L, ptx, pty, ptz, lx, ly, lz, r2);
    const double u = key_f64(key, 2u + 2u * static_cast<uint32_t>(l));
    const double w = key_f64(key, 3u + 2u * static_cast<uint32_t>(l));
    const double qx = (L.v[0] + L.v[3] * u) + L.v[6] * w;
    const double qy = (L.v[1] + L.v[4] * u) + L.v[7] * w;
    const double qz = (L.v[2] + L.v[5] * u) + L.v[8] * w;
    const double vx = qx - ptx, vy = qy - pty, vz = qz - ptz;
    r2 = vx * vx + vy * vy + vz * vz;
    const double n = sqrt(r2);
    lx = vx / n; ly = vy / n; lz = vz / n;
    return true;
}

}  // namespace rtamd
