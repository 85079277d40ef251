// sRGB quantiser, BMP header / writer and cameras: the host-side pieces of the
// path that stay on the CPU.
//
// All arithmetic is f64 without contraction (this file is compiled with
// -ffp-contract=off), matching the reference's Rust.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "host_scene.hpp"

namespace rtamd {

namespace {
double g_values[256];
double g_average[255];
std::once_flag g_once;

// color.rs:75-332 holds SRGB_VALUES[i] as literals; they are exactly the sRGB
// EOTF of i/255 in f64, and SRGB_AVERAGE[i] (color.rs:335-591) is exactly the
// midpoint of neighbours.  tests/test_host.py asserts both tables bit-for-bit
// against the reference's literals (tests/golden/srgb_tables.json).
void init_tables() {
    for (int i = 0; i < 256; ++i) {
        double c = static_cast<double>(i) / 255.0;
        g_values[i] = c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4);
    }
    for (int i = 0; i < 255; ++i) g_average[i] = (g_values[i] + g_values[i + 1]) / 2.0;
}
}  // namespace

const double* srgb_values_table() { std::call_once(g_once, init_tables); return g_values; }
const double* srgb_average_table() { std::call_once(g_once, init_tables); return g_average; }

// color.rs:593-600: the smallest i with v < SRGB_AVERAGE[i], else 255.  The
// table is strictly increasing, so a binary search is the same function; NaN
// compares false everywhere and lands on 255 like the linear scan.
uint8_t to_srgb(double v) {
    const double* a = srgb_average_table();
    if (!(v < a[254])) return 255;
    int lo = 0, hi = 254;               // answer in [lo, hi]
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (v < a[mid]) hi = mid; else lo = mid + 1;
    }
    return static_cast<uint8_t>(lo);
}

namespace {
struct V3 { double x, y, z; };
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 mul(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 normalize(V3 a) { double l = std::sqrt(dot(a, a)); return {a.x / l, a.y / l, a.z / l}; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V3 from(const double* p) { return {p[0], p[1], p[2]}; }
}  // namespace

// camera.rs:51-63
void camera_simple_new(const double position[3], const double look[3], const double up[3],
                       double im_dist, rt_camera& out) {
    V3 lk = from(look), u = normalize(cross(lk, from(up)));
    V3 v = normalize(cross(u, lk));
    V3 w = mul(normalize(lk), im_dist);
    out = rt_camera{};
    out.kind = RT_CAMERA_SIMPLE;
    out.samples = 1;
    for (int i = 0; i < 3; ++i) out.position[i] = position[i];
    const double m[9] = {u.x, v.x, w.x, u.y, v.y, w.y, u.z, v.z, w.z};
    std::memcpy(out.matrix, m, sizeof m);
}

// camera.rs:67-73
void camera_look_at(const double focus[3], const double look[3], const double up[3],
                    double pov, double h, rt_camera& out) {
    double cot = 1.0 / std::tan(pov / 2.0);
    double d = h * cot;
    V3 pos = sub(from(focus), mul(normalize(from(look)), d));
    const double p[3] = {pos.x, pos.y, pos.z};
    camera_simple_new(p, look, up, cot, out);
}

namespace {
thread_local std::string t_err;
}
void set_thread_error(const std::string& msg) { t_err = msg; }
const char* thread_error() { return t_err.c_str(); }

}  // namespace rtamd

extern "C" {

uint8_t rt_to_srgb(double v) { return rtamd::to_srgb(v); }

// bmp.rs:10-61
int rt_bmp_header(uint8_t out[122], uint32_t width, uint32_t height, uint32_t* bytewidth) {
    if (!out) return RT_E_INVALID;
    uint32_t bw = (3u * width + 3u) & 0xFFFFFFFCu;
    uint32_t pasize = bw * height;
    uint32_t fsize = 14u + 108u + pasize;
    std::memset(out, 0, 122);
    auto le32 = [&](int at, uint32_t v) { for (int k = 0; k < 4; ++k) out[at + k] = uint8_t(v >> (8 * k)); };
    out[0] = 'B'; out[1] = 'M';
    le32(2, fsize);
    le32(10, 122);            // offset of pixel array
    le32(14, 108);            // BITMAPV4HEADER size
    le32(18, width);
    le32(22, height);
    out[26] = 1;              // planes
    out[28] = 24;             // bpp
    le32(34, pasize);
    le32(38, 0x0B13);         // 72 DPI
    le32(42, 0x0B13);
    out[70] = 0x42; out[71] = 0x47; out[72] = 0x52; out[73] = 0x73;   // 'sRGB' (LCS_sRGB, little endian)
    if (bytewidth) *bytewidth = bw;
    return RT_OK;
}

// main.rs:34-59: header, then rows bottom-up (row 0 first).
int rt_write_bmp(const char* path, uint32_t width, uint32_t height, const uint8_t* bgr, uint32_t pitch) {
    if (!path || !bgr) return RT_E_INVALID;
    uint8_t hdr[122];
    uint32_t bw = 0;
    rt_bmp_header(hdr, width, height, &bw);
    if (pitch < 3 * width) return RT_E_INVALID;
    FILE* f = std::fopen(path, "wb");
    if (!f) { rtamd::set_thread_error(std::string("cannot create ") + path); return RT_E_IO; }
    bool ok = std::fwrite(hdr, 1, 122, f) == 122;
    std::string row(bw, '\0');
    for (uint32_t y = 0; ok && y < height; ++y) {
        std::memcpy(&row[0], bgr + static_cast<size_t>(y) * pitch, 3u * width);
        ok = std::fwrite(row.data(), 1, bw, f) == bw;
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) { rtamd::set_thread_error(std::string("error writing ") + path); return RT_E_IO; }
    return RT_OK;
}

int rt_camera_simple_new(const double position[3], const double look[3], const double up[3],
                         double im_dist, rt_camera* out) {
    if (!position || !look || !up || !out) return RT_E_INVALID;
    rtamd::camera_simple_new(position, look, up, im_dist, *out);
    return RT_OK;
}

int rt_camera_look_at(const double focus[3], const double look[3], const double up[3],
                      double pov, double h, rt_camera* out) {
    if (!focus || !look || !up || !out) return RT_E_INVALID;
    rtamd::camera_look_at(focus, look, up, pov, h, *out);
    return RT_OK;
}

}  // extern "C"
