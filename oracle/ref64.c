/*
 * ref64.c -- CPU ORACLE (test infrastructure only; see ref64.h for the rules
 * and the list of reference files this restates).  Plain C, IEEE f64, built
 * with -ffp-contract=off -fno-fast-math so that every expression below rounds
 * exactly like the reference's Rust (which never contracts a*b+c into an FMA).
 */
#define _GNU_SOURCE
#include "ref64.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* raytrace.rs:17 */
static const double MIN_SIGNIFICANCE = 1.0 / 256.0 / 2.0;
/* raytrace.rs:43,62 ... the self-intersection offset */
static const double EPS_OFFSET = 0.00001;
/* std::f64::consts::FRAC_1_PI, raytrace.rs:52 */
static const double FRAC_1_PI_ = 0.318309886183790671537767526745028724;
static const double PI_ = 3.14159265358979323846264338327950288;

typedef struct { double x, y, z; } v3;
typedef struct { double r, g, b; } col;

static inline v3 V(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
/* nalgebra 0.4 dot: (x*x' + y*y') + z*z'  (assumed op order) */
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double sqnorm(v3 a) { return dot(a, a); }
/* normalize = divide each component by sqrt(sqnorm) */
static inline v3 normalize(v3 a) { double l = sqrt(sqnorm(a)); return V(a.x / l, a.y / l, a.z / l); }
static inline v3 cross(v3 a, v3 b) {
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline v3 from3(const double* p) { return V(p[0], p[1], p[2]); }

static inline col C(double r, double g, double b) { col c = {r, g, b}; return c; }
static inline col cadd(col a, col b) { return C(a.r + b.r, a.g + b.g, a.b + b.b); }
static inline col cmulc(col a, col b) { return C(a.r * b.r, a.g * b.g, a.b * b.b); }
static inline col cmul(col a, double s) { return C(a.r * s, a.g * s, a.b * s); }
static inline col cdiv(col a, double s) { return C(a.r / s, a.g / s, a.b / s); }
static inline col cfrom3(const double* p) { return C(p[0], p[1], p[2]); }
/* color.rs:637-639 */
static inline double significance(col c) { return c.r + c.g + c.b; }
static const col BLACK = {0.0, 0.0, 0.0};

/* raytrace.rs:20-28 */
static inline double clamp_zero(double x) { return x < 0.0 ? 0.0 : x; }
static inline double clamp_one(double x) { return x > 1.0 ? 1.0 : x; }

/* ---- RNG: rand 0.3 XorShiftRng (statistical paths only; the reference seeds
 * it from OS entropy, main.rs:43, so only its distribution matters) ---- */
typedef struct { uint32_t x, y, z, w; } rng_t;
static inline uint32_t rng_u32(rng_t* r) {
    uint32_t t = r->x ^ (r->x << 11);
    r->x = r->y; r->y = r->z; r->z = r->w;
    r->w = r->w ^ (r->w >> 19) ^ (t ^ (t >> 8));
    return r->w;
}
static inline uint64_t rng_u64(rng_t* r) { uint64_t hi = rng_u32(r); return (hi << 32) | rng_u32(r); }
static inline double rng_f64(rng_t* r) {
    uint64_t bits = 0x3FF0000000000000ull | (rng_u64(r) & 0xFFFFFFFFFFFFFull);
    double d; memcpy(&d, &bits, 8); return d - 1.0;
}
static inline double rng_closed01(rng_t* r) { return (double)(rng_u64(r) >> 11) / 9007199254740991.0; }
static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t* r, uint64_t seed) {
    uint64_t s = seed;
    uint64_t a = splitmix64(&s), b = splitmix64(&s);
    r->x = (uint32_t)a; r->y = (uint32_t)(a >> 32); r->z = (uint32_t)b; r->w = (uint32_t)(b >> 32) | 1u;
}

/* ---- keyed counter-based RNG (REF_RNG_KEYED): the specification shared with
 * the device path (trace_common.hpp).  A draw is a pure function of a 64-bit
 * key and a draw id; keys follow the recursion:
 *   pixel      kp = mix(mix(seed) + (y << 32 | x))         (frame coordinates)
 *   AA sample  ka = child(kp, aa)      jitter: jx = f64(ka, 0), jy = f64(ka, 1)
 *   camera     kc = child(ka, cs)      DoF: theta = f64(kc, 0) * 2pi, r2 = closed01(kc, 1)
 *   path key of the camera ray = kc; a hit with path key K draws
 *     AreaLight l:         u = f64(K, 2 + 2l), w = f64(K, 3 + 2l)
 *     indirect sample i:   r1 = f64(K, 128 + 2i), r2 = f64(K, 129 + 2i)
 *   child ray i of a hit (indirect sample i; mirror reflection 0,
 *   Transparent refraction 1): key child(K, i).
 * f64 / closed01 use the bit recipes of rand 0.3 (rng_f64 / rng_closed01). */
static inline uint64_t kmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t key_child(uint64_t k, uint64_t i) { return kmix(k + (i + 1) * 0x9E3779B97F4A7C15ull); }
static inline uint64_t key_bits(uint64_t k, uint32_t id) { return kmix(k ^ ((uint64_t)(id + 1) * 0xD1B54A32D192ED03ull)); }
static inline double key_f64(uint64_t k, uint32_t id) {
    uint64_t bits = 0x3FF0000000000000ull | (key_bits(k, id) & 0xFFFFFFFFFFFFFull);
    double d; memcpy(&d, &bits, 8); return d - 1.0;
}
static inline double key_closed01(uint64_t k, uint32_t id) { return (double)(key_bits(k, id) >> 11) / 9007199254740991.0; }
static inline uint64_t key_pixel(uint64_t seed, uint32_t x, uint32_t y) {
    return kmix(kmix(seed) + (((uint64_t)y << 32) | x));
}

/* ---- shapes.rs ---- */
typedef struct { v3 origin, direction; } ray_t;
/* shapes.rs:22-24 */
static inline v3 cast(const ray_t* r, double t) { return vadd(r->origin, vmul(r->direction, t)); }

/* shapes.rs:50-89 */
static int sphere_intersect(v3 c, double radius, const ray_t* ray, double* t_out, v3* n_out) {
    v3 oc = vsub(ray->origin, c);
    double a = sqnorm(ray->direction);
    double b = 2.0 * dot(ray->direction, oc);
    double cc = sqnorm(oc) - radius * radius;
    double disc = b * b - 4.0 * a * cc;
    if (disc > 0.0) {
        double s = sqrt(disc);
        double t = (-b - s) / (2.0 * a);
        if (t > 0.0) {
            *t_out = t; if (n_out) *n_out = normalize(vsub(cast(ray, t), c));
            return 1;
        }
        double t2 = (-b + s) / (2.0 * a);
        if (t2 > 0.0) {
            *t_out = t2; if (n_out) *n_out = normalize(vsub(cast(ray, t2), c));
            return 1;
        }
        return 0;
    }
    return 0;
}

/* shapes.rs:100-112 -- the normal is returned as written in the file (not normalised) */
static int plane_intersect(v3 p, v3 n, const ray_t* ray, double* t_out, v3* n_out) {
    double t = dot(n, vsub(p, ray->origin)) / dot(n, ray->direction);
    if (t <= 0.0) return 0;          /* NaN <= 0 is false: a NaN t IS a hit */
    *t_out = t; if (n_out) *n_out = n;
    return 1;
}

/* ---- scene ---- */
typedef struct {
    const ref_scene* s;
    uint32_t max_depth;
    v3 cam_pos; double cam_m[9];
    double cam_im_dist;
    ref_counts cnt;
    rng_t rng;
    int keyed;              /* REF_RNG_KEYED */
} ctx_t;

/* A [0,1) draw: the next XorShift output, or the keyed draw (key, id). */
static inline double draw_f64(ctx_t* c, uint64_t key, uint32_t id) {
    return c->keyed ? key_f64(key, id) : rng_f64(&c->rng);
}

typedef struct { int hit; uint32_t obj; double t; v3 normal; } hit_t;

/* scene.rs:223-249: filter_map over all objects in file order, then
 * min_by_key(FloatNotNan::new(t)).  Option ordering puts None (a NaN t) BELOW
 * every Some, and min_by_key keeps the FIRST minimum, so: a NaN-t hit wins
 * (the first one in file order), otherwise the smallest t, ties -> first. */
static hit_t scene_intersect(ctx_t* c, const ray_t* ray) {
    hit_t best; best.hit = 0; best.obj = 0; best.t = 0.0; best.normal = V(0, 0, 0);
    int best_nan = 0;
    c->cnt.rays++;
    for (uint32_t i = 0; i < c->s->n_objects; ++i) {
        const ref_object* o = &c->s->objects[i];
        double t; v3 n; int h;
        if (o->shape == REF_SPHERE) {
            c->cnt.sphere_tests++;
            h = sphere_intersect(from3(o->geom), o->geom[3], ray, &t, &n);
        } else {
            c->cnt.plane_tests++;
            h = plane_intersect(from3(o->geom), from3(o->geom + 3), ray, &t, &n);
        }
        if (!h) continue;
        int cnan = isnan(t);
        int better;
        if (!best.hit) better = 1;
        else if (best_nan) better = 0;                 /* None is the minimum; first one stays */
        else if (cnan) better = 1;
        else better = t < best.t;                      /* strict: ties keep the first */
        if (better) { best.hit = 1; best.obj = i; best.t = t; best.normal = n; best_nan = cnan; }
    }
    return best;
}

/* scene.rs:117-155: returns 1 if the light has a range (Some(sq)) */
static int light_dir(ctx_t* c, const ref_light* L, uint32_t li, uint64_t key, v3 pt, v3* ldir, double* sq) {
    if (L->kind == REF_POINT || L->kind == REF_AREA) {
        v3 loc;
        if (L->kind == REF_POINT) loc = from3(L->v);
        else {
            double u = draw_f64(c, key, 2 + 2 * li), w = draw_f64(c, key, 3 + 2 * li);
            loc = vadd(vadd(from3(L->v), vmul(from3(L->v + 3), u)), vmul(from3(L->v + 6), w));
        }
        v3 dv = V(loc.x - pt.x, loc.y - pt.y, loc.z - pt.z);
        *ldir = normalize(dv);
        *sq = sqnorm(vsub(loc, pt));   /* FloatPnt::sqdist */
        return 1;
    }
    *ldir = vneg(from3(L->v));         /* DirectionalLight: -direction, NOT normalised */
    return 0;
}

/* The shadow test shared by every material (raytrace.rs:41-49 and copies). */
static int in_shadow(ctx_t* c, v3 pt, v3 ldir, int has_range, double sq) {
    ray_t sr; sr.origin = vadd(pt, vmul(ldir, EPS_OFFSET)); sr.direction = ldir;
    hit_t h = scene_intersect(c, &sr);
    c->cnt.shadow_rays++;
    if (!h.hit) return 0;
    if (has_range) return h.t * h.t < sq;
    return 1;
}

static col ray_color(ctx_t* c, const ray_t* ray, double sig, uint32_t depth, uint64_t key);

static col shade(ctx_t* c, const ref_object* m, const hit_t* hit, const ray_t* ray, double sig, uint32_t depth,
                 uint64_t key) {
    col kd = cfrom3(m->diffuse), ks = cfrom3(m->specular), amb = cfrom3(m->ambient);
    switch (m->material) {
    case REF_PHONG: {                                  /* raytrace.rs:30-67 */
        col res = amb;
        if (depth > c->max_depth) return res;
        v3 pt = cast(ray, hit->t);
        int diffuse = significance(kd) * sig > MIN_SIGNIFICANCE;
        int specular = significance(ks) * sig > MIN_SIGNIFICANCE;
        v3 normal = dot(hit->normal, ray->direction) > 0.0 ? vneg(hit->normal) : hit->normal;
        for (uint32_t li = 0; li < c->s->n_lights; ++li) {
            if (!(diffuse || specular)) continue;
            const ref_light* L = &c->s->lights[li];
            v3 ldir; double sq = 0.0;
            int rng_ = light_dir(c, L, li, key, pt, &ldir, &sq);
            if (in_shadow(c, pt, ldir, rng_, sq)) continue;
            col lc = cfrom3(L->color);
            if (diffuse)
                res = cadd(res, cmul(cmul(cmulc(kd, lc), clamp_zero(dot(ldir, normal))), FRAC_1_PI_));
            if (specular)
                res = cadd(res, cmul(cmulc(ks, lc),
                                     pow(clamp_zero(dot(normal, normalize(vsub(ldir, ray->direction)))), m->exponent)));
        }
        if (specular) {
            v3 d = ray->direction;
            v3 rd = vsub(d, vmul(normal, 2.0 * dot(d, normal)));
            ray_t refl; refl.origin = vadd(pt, vmul(rd, EPS_OFFSET)); refl.direction = rd;
            res = cadd(res, cmulc(ks, ray_color(c, &refl, sig * significance(ks), depth + 1, key_child(key, 0))));
        }
        return res;
    }
    case REF_INDIRECT_PHONG: {                         /* raytrace.rs:69-121 */
        col res = amb;
        if (depth > c->max_depth) return res;
        v3 pt = cast(ray, hit->t);
        int diffuse = significance(kd) * sig > MIN_SIGNIFICANCE;
        int specular = significance(ks) * sig > MIN_SIGNIFICANCE;
        v3 normal = dot(hit->normal, ray->direction) > 0.0 ? vneg(hit->normal) : hit->normal;
        if (diffuse || specular) {
            for (uint32_t li = 0; li < c->s->n_lights; ++li) {
                const ref_light* L = &c->s->lights[li];
                v3 ldir; double sq = 0.0;
                int rng_ = light_dir(c, L, li, key, pt, &ldir, &sq);
                if (in_shadow(c, pt, ldir, rng_, sq)) continue;
                col lc = cfrom3(L->color);
                if (diffuse)
                    res = cadd(res, cmul(cmul(cmulc(kd, lc), clamp_zero(dot(ldir, normal))), FRAC_1_PI_));
                if (specular)
                    res = cadd(res, cmul(cmulc(ks, lc),
                                         pow(clamp_zero(dot(normal, normalize(vsub(ldir, ray->direction)))), m->exponent)));
            }
            for (uint32_t si = 0; si < m->samples; ++si) {
                double r1 = draw_f64(c, key, 128 + 2 * si) * 2.0 - 1.0;
                double r2 = draw_f64(c, key, 129 + 2 * si) * (2.0 * PI_);
                double sin_theta = 1.0 - r1 * r1;          /* quirk: no sqrt (raytrace.rs:103) */
                double phi = r2;
                double x = sin_theta * cos(phi), z = sin_theta * sin(phi);
                v3 d0 = V(x, r1, z);
                v3 dir = dot(d0, normal) >= 0.0 ? d0 : vneg(d0);
                ray_t nr; nr.origin = vadd(pt, vmul(dir, EPS_OFFSET)); nr.direction = dir;
                col cl = ray_color(c, &nr, sig, depth + 1, key_child(key, si));
                double fac = (double)m->samples * 0.5;
                if (diffuse) res = cadd(res, cdiv(cmul(cmulc(kd, cl), dot(normal, dir)), fac));
                if (specular)   /* quirk: `ray` here is the NEW ray, so dir - dir = 0 (raytrace.rs:108,115) */
                    res = cadd(res, cdiv(cmul(cmulc(ks, cl),
                                              pow(clamp_zero(dot(normal, normalize(vsub(dir, nr.direction)))), m->exponent)), fac));
            }
        }
        return res;
    }
    case REF_FRESNEL: {                                /* raytrace.rs:123-167 */
        col res = amb;
        if (depth > c->max_depth) return res;
        v3 pt = cast(ray, hit->t);
        double nd = dot(hit->normal, ray->direction);
        v3 normal = nd > 0.0 ? vneg(hit->normal) : hit->normal;
        double r0 = (m->ior - 1.0) / (m->ior + 1.0);
        r0 = r0 * r0;
        double omcos = 1.0 - fabs(nd);
        double omcos2 = omcos * omcos;
        double fresnel = clamp_one(r0 + (1.0 - r0) * omcos2 * omcos2 * omcos);
        int diffuse = significance(kd) * sig > MIN_SIGNIFICANCE;
        int specular = significance(ks) * fresnel * sig > MIN_SIGNIFICANCE;
        for (uint32_t li = 0; li < c->s->n_lights; ++li) {
            if (!(diffuse || specular)) continue;
            const ref_light* L = &c->s->lights[li];
            v3 ldir; double sq = 0.0;
            int rng_ = light_dir(c, L, li, key, pt, &ldir, &sq);
            if (in_shadow(c, pt, ldir, rng_, sq)) continue;
            col lc = cfrom3(L->color);
            if (diffuse)
                res = cadd(res, cmul(cmul(cmulc(kd, lc), clamp_zero(dot(ldir, normal))), FRAC_1_PI_));
            if (specular)
                res = cadd(res, cmul(cmul(cmulc(ks, lc), fresnel),
                                     pow(clamp_zero(dot(normal, normalize(vsub(ldir, ray->direction)))), m->exponent)));
        }
        if (specular) {
            v3 d = ray->direction;
            v3 rd = vsub(d, vmul(normal, 2.0 * dot(d, normal)));
            ray_t refl; refl.origin = vadd(pt, vmul(rd, EPS_OFFSET)); refl.direction = rd;
            res = cadd(res, cmul(cmulc(ks, ray_color(c, &refl, fresnel * sig * significance(ks), depth + 1, key_child(key, 0))),
                                 fresnel));
        }
        return res;
    }
    case REF_TRANSPARENT: {                            /* raytrace.rs:169-226 */
        col res = BLACK;
        if (depth > c->max_depth) return res;
        v3 pt = cast(ray, hit->t);
        double nd = dot(hit->normal, ray->direction);
        v3 normal = nd > 0.0 ? vneg(hit->normal) : hit->normal;
        double ndv = dot(normal, ray->direction);
        double n = nd > 0.0 ? m->ior : 1.0 / m->ior;
        double sin2 = n * n * (1.0 - nd * nd);
        int has_refract = sin2 < 1.0;
        v3 refract = V(0, 0, 0);
        if (has_refract) {
            double cs = sqrt(1.0 - sin2);
            refract = vsub(vmul(ray->direction, n), vmul(normal, n * fabs(nd) + cs));
        }
        double r0 = (m->ior - 1.0) / (m->ior + 1.0);
        r0 = r0 * r0;
        double omcos = nd > 0.0 ? (has_refract ? 1.0 - dot(normal, refract) : 0.0) : 1.0 - fabs(nd);
        double omcos2 = omcos * omcos;
        double fresnel = has_refract ? clamp_one(r0 + (1.0 - r0) * omcos2 * omcos2 * omcos) : 1.0;
        int specular = significance(ks) * fresnel * sig > MIN_SIGNIFICANCE;
        for (uint32_t li = 0; li < c->s->n_lights; ++li) {
            if (!specular) continue;
            const ref_light* L = &c->s->lights[li];
            v3 ldir; double sq = 0.0;
            int rng_ = light_dir(c, L, li, key, pt, &ldir, &sq);
            if (in_shadow(c, pt, ldir, rng_, sq)) continue;
            col lc = cfrom3(L->color);
            res = cadd(res, cmul(cmul(cmulc(ks, lc), fresnel),
                                 pow(clamp_zero(dot(normal, normalize(vsub(ldir, ray->direction)))), m->exponent)));
        }
        if (specular) {
            v3 rd = vsub(ray->direction, vmul(normal, 2.0 * ndv));
            ray_t refl; refl.origin = vadd(pt, vmul(rd, EPS_OFFSET)); refl.direction = rd;
            res = cadd(res, cmul(cmulc(ks, ray_color(c, &refl, fresnel * sig * significance(ks), depth + 1, key_child(key, 0))),
                                 fresnel));
        }
        if (fresnel < 1.0 && has_refract) {
            double omf = clamp_one(1.0 - fresnel);
            v3 r = normalize(refract);
            ray_t rr; rr.origin = vadd(pt, vmul(r, EPS_OFFSET)); rr.direction = r;
            res = cadd(res, cmul(ray_color(c, &rr, omf * sig, depth + 1, key_child(key, 1)), omf));
        }
        return res;
    }
    }
    return BLACK;
}

/* texture.rs:28-31, 40-58 and color.rs:611-613 (Color::from_srgb) */
static double SRGB_VALUES_[256];
static double tex_clamp(double x) { return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x); }
static col tex_at(const ref_texture* t, uint32_t x, uint32_t y) {
    const uint8_t* p = t->rgb + 3 * ((size_t)x + (size_t)y * t->width);
    col c; c.r = SRGB_VALUES_[p[0]]; c.g = SRGB_VALUES_[p[1]]; c.b = SRGB_VALUES_[p[2]];
    return c;
}
static uint32_t as_u32(double x) { return x >= 0.0 ? (uint32_t)x : 0u; }   /* Rust `as u32`: NaN -> 0 */
static col tex_sample(const ref_texture* t, double xs, double ys) {
    double x = tex_clamp(xs) * (double)(t->width - 1);
    double y = tex_clamp(ys) * (double)(t->height - 1);
    uint32_t x0 = as_u32(x), y0 = as_u32(y);
    uint32_t x1 = x0 >= t->width - 1 ? t->width - 1 : x0 + 1;
    uint32_t y1 = y0 >= t->height - 1 ? t->height - 1 : y0 + 1;
    double xx = x - (double)x0, yy = y - (double)y0;
    col cx0 = cadd(cmul(tex_at(t, x0, y0), 1.0 - yy), cmul(tex_at(t, x0, y1), yy));
    col cx1 = cadd(cmul(tex_at(t, x1, y0), 1.0 - yy), cmul(tex_at(t, x1, y1), yy));
    return cadd(cmul(cx0, 1.0 - xx), cmul(cx1, xx));
}
/* raytrace.rs:234-256: x axis, then y, then z (skybox_axis! macro order) */
static col skybox_color(const ref_texture* f, v3 d) {
    if (fabs(d.x) > fabs(d.z) && fabs(d.x) > fabs(d.y)) {
        double px = -d.z / d.x, py = -d.y / fabs(d.x);
        return tex_sample(&f[d.x > 0.0 ? 0 : 1], px * 0.5 + 0.5, py * 0.5 + 0.5);
    }
    if (fabs(d.y) > fabs(d.x) && fabs(d.y) > fabs(d.z)) {
        double px = d.x / fabs(d.y), py = d.z / d.y;
        return tex_sample(&f[d.y > 0.0 ? 2 : 3], px * 0.5 + 0.5, py * 0.5 + 0.5);
    }
    if (fabs(d.z) > fabs(d.x) && fabs(d.z) > fabs(d.y)) {
        double px = d.x / d.z, py = -d.y / fabs(d.z);
        return tex_sample(&f[d.z > 0.0 ? 4 : 5], px * 0.5 + 0.5, py * 0.5 + 0.5);
    }
    return BLACK;
}

/* raytrace.rs:261-267 */
static col ray_color(ctx_t* c, const ray_t* ray, double sig, uint32_t depth, uint64_t key) {
    hit_t h = scene_intersect(c, ray);
    if (!h.hit)                                         /* raytrace.rs:228-256 */
        return c->s->skybox ? skybox_color(c->s->skybox, ray->direction) : cfrom3(c->s->background);
    return shade(c, &c->s->objects[h.obj], &h, ray, sig, depth, key);
}

/* camera.rs:51-73 */
int ref_camera_build(const ref_camera* cam, double position[3], double matrix[9]) {
    v3 pos, look = from3(cam->p1), up = from3(cam->p2);
    double im_dist;
    if (cam->ctor == REF_CAM_LOOK_AT) {
        double cot = 1.0 / tan(cam->s0 / 2.0);           /* (pov/2).tan().recip() */
        im_dist = cot;
        double d = cam->s1 * cot;
        pos = vsub(from3(cam->p0), vmul(normalize(look), d));
    } else {
        pos = from3(cam->p0);
        im_dist = cam->s0;
    }
    v3 u = normalize(cross(look, up));
    v3 v = normalize(cross(u, look));
    v3 w = vmul(normalize(look), im_dist);
    position[0] = pos.x; position[1] = pos.y; position[2] = pos.z;
    double m[9] = {u.x, v.x, w.x, u.y, v.y, w.y, u.z, v.z, w.z};
    memcpy(matrix, m, sizeof m);
    return 0;
}

static inline v3 mat_mul(const double* m, v3 p) {
    return V(m[0] * p.x + m[1] * p.y + m[2] * p.z,
             m[3] * p.x + m[4] * p.y + m[5] * p.z,
             m[6] * p.x + m[7] * p.y + m[8] * p.z);
}

/* camera.rs:76-80 (simple) and camera.rs:109-122 (depth of field) */
static ray_t camera_project(ctx_t* c, double px, double py, uint64_t key) {
    ray_t r;
    v3 dir = mat_mul(c->cam_m, V(px, py, 1.0));
    if (!c->s->camera.dof) {
        r.origin = c->cam_pos; r.direction = normalize(dir);
        return r;
    }
    v3 ip = vadd(c->cam_pos, dir);
    v3 fp = vadd(c->cam_pos, vmul(dir, c->s->camera.focus / c->cam_im_dist));
    double theta = draw_f64(c, key, 0) * (2.0 * PI_);
    double r2 = c->keyed ? key_closed01(key, 1) : rng_closed01(&c->rng);
    double rad = sqrt(r2) * c->s->camera.aperture;
    v3 orig = vadd(ip, mat_mul(c->cam_m, V(cos(theta) * rad, sin(theta) * rad, 0.0)));
    r.origin = orig; r.direction = normalize(vsub(fp, orig));
    return r;
}

/* ---- color.rs sRGB quantiser: tables generated, asserted against the
 * reference's literal tables by tests/test_oracle.py ---- */
static double SRGB_AVERAGE_[255];
static pthread_once_t srgb_once = PTHREAD_ONCE_INIT;
static void srgb_init(void) {
    for (int i = 0; i < 256; ++i) {
        double cc = (double)i / 255.0;
        SRGB_VALUES_[i] = cc <= 0.04045 ? cc / 12.92 : pow((cc + 0.055) / 1.055, 2.4);
    }
    for (int i = 0; i < 255; ++i) SRGB_AVERAGE_[i] = (SRGB_VALUES_[i] + SRGB_VALUES_[i + 1]) / 2.0;
}
double ref_srgb_value(int i) { pthread_once(&srgb_once, srgb_init); return SRGB_VALUES_[i]; }
double ref_srgb_average(int i) { pthread_once(&srgb_once, srgb_init); return SRGB_AVERAGE_[i]; }
/* color.rs:593-600: linear scan, first i with val < AVERAGE[i]; NaN -> 255 */
uint8_t ref_to_srgb(double v) {
    pthread_once(&srgb_once, srgb_init);
    for (int i = 0; i < 255; ++i)
        if (v < SRGB_AVERAGE_[i]) return (uint8_t)i;
    return 255;
}

/* bmp.rs:10-61 */
uint32_t ref_bmp_header(uint8_t out[122], uint32_t width, uint32_t height) {
    uint32_t bytewidth = (3u * width + 3u) & 0xFFFFFFFCu;
    uint32_t pasize = bytewidth * height;
    uint32_t fsize = 14u + 108u + pasize;
    memset(out, 0, 122);
    out[0] = 0x42; out[1] = 0x4D;
    for (int k = 0; k < 4; ++k) out[2 + k] = (uint8_t)(fsize >> (8 * k));
    out[10] = 0x7A; out[14] = 0x6C;
    for (int k = 0; k < 4; ++k) out[18 + k] = (uint8_t)(width >> (8 * k));
    for (int k = 0; k < 4; ++k) out[22 + k] = (uint8_t)(height >> (8 * k));
    out[26] = 1; out[28] = 0x18;
    for (int k = 0; k < 4; ++k) out[34 + k] = (uint8_t)(pasize >> (8 * k));
    out[38] = 0x13; out[39] = 0x0B; out[42] = 0x13; out[43] = 0x0B;
    out[70] = 0x42; out[71] = 0x47; out[72] = 0x52; out[73] = 0x73;
    return bytewidth;
}

/* ---- exported known-answer building blocks ---- */
int ref_sphere_intersect(const double center[3], double radius, const double o[3], const double d[3],
                         double* t, double normal[3]) {
    ray_t r; r.origin = from3(o); r.direction = from3(d);
    v3 n; int h = sphere_intersect(from3(center), radius, &r, t, &n);
    if (h && normal) { normal[0] = n.x; normal[1] = n.y; normal[2] = n.z; }
    return h;
}
int ref_plane_intersect(const double point[3], const double nrm[3], const double o[3], const double d[3],
                        double* t, double normal[3]) {
    ray_t r; r.origin = from3(o); r.direction = from3(d);
    v3 n; int h = plane_intersect(from3(point), from3(nrm), &r, t, &n);
    if (h && normal) { normal[0] = n.x; normal[1] = n.y; normal[2] = n.z; }
    return h;
}

/* ---- the pixel loop, main.rs:39-59, over a tile, multi-threaded by rows ---- */
typedef struct {
    const ref_scene* s; const ref_opts* o;
    double* rgb64; float* rgb32; uint8_t* bgr; uint32_t pitch;
    uint32_t next_row;             /* atomic work counter */
    pthread_mutex_t mu;
    ref_counts total;
} job_t;

static uint32_t global_row(const ref_opts* o, uint32_t j) {
    uint32_t band = o->band ? o->band : 1, stride = o->band_stride ? o->band_stride : 1;
    return o->y0 + ((j / band) * stride + o->band_phase) * band + j % band;
}

static void* worker(void* arg) {
    job_t* jb = (job_t*)arg;
    const ref_scene* s = jb->s; const ref_opts* o = jb->o;
    ctx_t c; memset(&c, 0, sizeof c);
    c.s = s; c.max_depth = o->max_depth;
    c.keyed = o->rng == REF_RNG_KEYED;
    double cpos[3];
    ref_camera_build(&s->camera, cpos, c.cam_m);
    c.cam_pos = from3(cpos);
    {   /* camera.rs:98 DepthOfFieldCamera::new: im_dist = (M*(0,0,1)).norm() */
        v3 z = mat_mul(c.cam_m, V(0.0, 0.0, 1.0));
        c.cam_im_dist = sqrt(sqnorm(z));
    }
    double hw = (double)s->width / 2.0, hh = (double)s->height / 2.0;   /* main.rs:39-41 */
    double a = 1.0 / hw, b = 1.0 / hh;
    double scale = a > b ? a : b;      /* f64::max; NaN-free here */
    uint32_t aa = s->antialias;
    uint32_t cam_samples = s->camera.dof ? s->camera.dof_samples : 1;
    for (;;) {
        uint32_t j = __atomic_fetch_add(&jb->next_row, 1, __ATOMIC_RELAXED);
        if (j >= o->tile_h) break;
        uint32_t y = global_row(o, j);
        rng_seed(&c.rng, o->seed * 0x100000001B3ull + y);
        for (uint32_t i = 0; i < o->tile_w; ++i) {
            uint32_t x = o->x0 + i;
            const uint64_t kp = key_pixel(o->seed, x, y);
            col res = BLACK;
            for (uint32_t k = 0; k < aa; ++k) {
                const uint64_t ka = key_child(kp, k);
                double jx, jy;
                if (o->jitter == REF_JITTER_CENTER) { jx = 0.5; jy = 0.5; }
                else { jx = draw_f64(&c, ka, 0); jy = draw_f64(&c, ka, 1); }   /* x drawn before y */
                double px = (((double)x + jx) - hw) * scale;
                double py = (((double)y + jy) - hh) * scale;
                /* raytrace.rs:270-276 */
                col r = BLACK;
                for (uint32_t cs = 0; cs < cam_samples; ++cs) {
                    const uint64_t kc = key_child(ka, cs);
                    ray_t ray = camera_project(&c, px, py, kc);
                    r = cadd(r, ray_color(&c, &ray, 1.0, 0, kc));
                }
                r = cdiv(r, (double)cam_samples);
                res = cadd(res, r);
            }
            res = cdiv(res, (double)aa);
            size_t p = (size_t)j * o->tile_w + i;
            if (jb->rgb64) { jb->rgb64[3 * p] = res.r; jb->rgb64[3 * p + 1] = res.g; jb->rgb64[3 * p + 2] = res.b; }
            if (jb->rgb32) { jb->rgb32[3 * p] = (float)res.r; jb->rgb32[3 * p + 1] = (float)res.g; jb->rgb32[3 * p + 2] = (float)res.b; }
            if (jb->bgr) {                                  /* color.rs:628-632 */
                uint8_t* q = jb->bgr + (size_t)j * jb->pitch + 3 * (size_t)i;
                q[0] = ref_to_srgb(res.b); q[1] = ref_to_srgb(res.g); q[2] = ref_to_srgb(res.r);
            }
        }
    }
    pthread_mutex_lock(&jb->mu);
    jb->total.rays += c.cnt.rays; jb->total.shadow_rays += c.cnt.shadow_rays;
    jb->total.sphere_tests += c.cnt.sphere_tests; jb->total.plane_tests += c.cnt.plane_tests;
    pthread_mutex_unlock(&jb->mu);
    return NULL;
}

int ref_render(const ref_scene* scene, const ref_opts* opts,
               double* out_rgb64, float* out_rgb32, uint8_t* out_bgr, uint32_t bgr_pitch,
               ref_counts* counts) {
    if (!scene || !opts || scene->width == 0 || scene->height == 0 || scene->antialias == 0) return -1;
    if (opts->x0 + opts->tile_w > scene->width) return -1;
    if (opts->tile_h && global_row(opts, opts->tile_h - 1) >= scene->height) return -1;
    if (out_bgr && bgr_pitch < 3 * opts->tile_w) return -1;
    pthread_once(&srgb_once, srgb_init);
    job_t jb; memset(&jb, 0, sizeof jb);
    jb.s = scene; jb.o = opts; jb.rgb64 = out_rgb64; jb.rgb32 = out_rgb32; jb.bgr = out_bgr; jb.pitch = bgr_pitch;
    pthread_mutex_init(&jb.mu, NULL);
    if (out_bgr)   /* BMP rows are zero padded (main.rs:42 vec![0; bytewidth]) */
        for (uint32_t j = 0; j < opts->tile_h; ++j)
            memset(out_bgr + (size_t)j * bgr_pitch + 3 * (size_t)opts->tile_w, 0, bgr_pitch - 3 * opts->tile_w);
    int nt = opts->threads > 0 ? opts->threads : (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nt < 1) nt = 1;
    if ((uint32_t)nt > opts->tile_h) nt = opts->tile_h ? (int)opts->tile_h : 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nt);
    for (int k = 1; k < nt; ++k) pthread_create(&th[k], NULL, worker, &jb);
    worker(&jb);
    for (int k = 1; k < nt; ++k) pthread_join(th[k], NULL);
    free(th);
    pthread_mutex_destroy(&jb.mu);
    if (counts) *counts = jb.total;
    return 0;
}
