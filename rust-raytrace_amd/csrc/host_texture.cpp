// Texture loading for SkyboxBackground (texture.rs:34-37).  The reference
// decodes through the `image` crate (PNG, JPEG, BMP, PPM, ...); no image
// library is available to this build, so the host decodes the two formats
// that need none: uncompressed BMP (24 or 32 bit, either row order) and binary
// PPM (P6, maxval 255).  The result is what `image::open(path).to_rgb()`
// yields: RGB8, rows top-down.
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "host_scene.hpp"

namespace rtamd {
namespace {

uint32_t le16(const uint8_t* p) { return p[0] | (p[1] << 8); }
uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | (static_cast<uint32_t>(p[3]) << 24); }

// Largest side accepted (a texture is at most 2^15 x 2^15 texels = 3 GiB of
// RGB8): every size product below then fits in 64 bits without wrapping.
constexpr uint64_t kMaxSide = 1u << 15;

int decode_bmp(const std::vector<uint8_t>& f, HostTexture& t, std::string& err) {
    if (f.size() < 54) { err = "truncated BMP header"; return RT_E_IO; }
    const uint32_t data_off = le32(&f[10]), hdr = le32(&f[14]);
    if (hdr < 40) { err = "unsupported BMP header (OS/2)"; return RT_E_UNSUPPORTED; }
    const int32_t w = static_cast<int32_t>(le32(&f[18])), h = static_cast<int32_t>(le32(&f[22]));
    const uint32_t bpp = le16(&f[28]), comp = le32(&f[30]);
    if ((bpp != 24 && bpp != 32) || (comp != 0 && !(comp == 3 && bpp == 32))) {
        err = "unsupported BMP encoding (" + std::to_string(bpp) + " bpp, compression " + std::to_string(comp) + ")";
        return RT_E_UNSUPPORTED;
    }
    if (w <= 0 || h == 0 || h == INT32_MIN) { err = "empty BMP"; return RT_E_IO; }
    const bool bottom_up = h > 0;
    const uint32_t H = static_cast<uint32_t>(bottom_up ? h : -static_cast<int64_t>(h)), W = static_cast<uint32_t>(w);
    if (W > kMaxSide || H > kMaxSide) { err = "BMP larger than 32768 x 32768"; return RT_E_UNSUPPORTED; }
    const uint64_t pitch = (static_cast<uint64_t>(W) * (bpp / 8) + 3) & ~3ull;
    if (static_cast<uint64_t>(data_off) + pitch * H > f.size()) { err = "truncated BMP pixel data"; return RT_E_IO; }
    t.width = W;
    t.height = H;
    t.rgb.assign(static_cast<size_t>(W) * H * 3, 0);
    for (uint32_t y = 0; y < H; ++y) {
        const uint32_t src_row = bottom_up ? H - 1 - y : y;
        const uint8_t* row = f.data() + data_off + src_row * pitch;
        for (uint32_t x = 0; x < W; ++x) {
            const uint8_t* px = row + static_cast<size_t>(x) * (bpp / 8);
            uint8_t* q = &t.rgb[(static_cast<size_t>(y) * W + x) * 3];
            q[0] = px[2]; q[1] = px[1]; q[2] = px[0];          // BGR(A) -> RGB
        }
    }
    return RT_OK;
}

int decode_ppm(const std::vector<uint8_t>& f, HostTexture& t, std::string& err) {
    size_t i = 2;
    auto skip = [&]() {
        for (;;) {
            while (i < f.size() && std::isspace(f[i])) ++i;
            if (i < f.size() && f[i] == '#') { while (i < f.size() && f[i] != '\n') ++i; continue; }
            return;
        }
    };
    auto num = [&](uint64_t& v) {
        skip();
        if (i >= f.size() || !std::isdigit(f[i])) return false;
        v = 0;
        while (i < f.size() && std::isdigit(f[i]) && v < (1ull << 32)) v = v * 10 + (f[i++] - '0');
        return true;
    };
    uint64_t w, h, mx;
    if (!num(w) || !num(h) || !num(mx) || i >= f.size()) { err = "bad PPM header"; return RT_E_IO; }
    if (mx != 255) { err = "unsupported PPM maxval " + std::to_string(mx); return RT_E_UNSUPPORTED; }
    ++i;                                               // one whitespace byte ends the header
    if (w == 0 || h == 0) { err = "empty PPM"; return RT_E_IO; }
    if (w > kMaxSide || h > kMaxSide) { err = "PPM larger than 32768 x 32768"; return RT_E_UNSUPPORTED; }
    if (w * h * 3 > f.size() - i) { err = "truncated PPM"; return RT_E_IO; }
    t.width = static_cast<uint32_t>(w);
    t.height = static_cast<uint32_t>(h);
    t.rgb.assign(f.begin() + i, f.begin() + i + w * h * 3);
    return RT_OK;
}

}  // namespace

int load_texture_file(const std::string& path, HostTexture& out, std::string& err) {
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) { err = "cannot open " + path; return RT_E_IO; }
    std::vector<uint8_t> f;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) f.insert(f.end(), buf, buf + n);
    std::fclose(fp);
    HostTexture t;
    int rc;
    if (f.size() >= 2 && f[0] == 'B' && f[1] == 'M') rc = decode_bmp(f, t, err);
    else if (f.size() >= 2 && f[0] == 'P' && f[1] == '6') rc = decode_ppm(f, t, err);
    else { err = "unsupported image format (this build decodes BMP and binary PPM)"; rc = RT_E_UNSUPPORTED; }
    if (rc == RT_OK) out = std::move(t);
    return rc;
}

}  // namespace rtamd

extern "C" {

int rt_texture_load(const char* path, uint32_t* width, uint32_t* height, uint8_t* rgb, size_t cap) {
    if (!path || !width || !height) return RT_E_INVALID;
    ::HostTexture t;
    std::string err;
    const int rc = rtamd::load_texture_file(path, t, err);
    if (rc != RT_OK) { rtamd::set_thread_error(err); return rc; }
    *width = t.width;
    *height = t.height;
    if (rgb) {
        if (cap < t.rgb.size()) { rtamd::set_thread_error("rgb buffer too small"); return RT_E_INVALID; }
        std::memcpy(rgb, t.rgb.data(), t.rgb.size());
    }
    return RT_OK;
}

int rt_scene_set_skybox(rt_scene* s, const rt_texture faces[6]) {
    if (!s || !faces) return RT_E_INVALID;
    ::HostTexture tex[6];
    for (int k = 0; k < 6; ++k) {
        if (!faces[k].rgb || faces[k].width == 0 || faces[k].height == 0) return RT_E_INVALID;
        tex[k].width = faces[k].width;
        tex[k].height = faces[k].height;
        tex[k].rgb.assign(faces[k].rgb, faces[k].rgb + static_cast<size_t>(faces[k].width) * faces[k].height * 3);
    }
    for (int k = 0; k < 6; ++k) s->skybox[k] = std::move(tex[k]);
    s->background_kind = RT_BG_SKYBOX;
    return RT_OK;
}

}  // extern "C"
