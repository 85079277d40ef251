// `raytrace` -- the replacement for the reference's main.rs:13-60.
//
// Reads a scene file in the reference grammar (default test_scene.txt, as
// main.rs:16), renders it on one or more GPUs through the C ABI, and writes the
// reference's BMP (default out.bmp, main.rs:34).  Multi-GPU: image rows are
// dealt in interleaved bands, one host thread + one rt_ctx per device, each
// device renders its bands into its own buffer and the host gathers them into
// the frame (no collective: pixels are independent, main.rs:45-57).
//
//   raytrace [--scene FILE] [--out FILE] [--width W] [--height H] [--spp N]
//            [--max-depth D] [--gpus N] [--band ROWS] [--jitter random|center] [--seed N]
//            [--algo auto|wavefront|path|lds|global]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "raytrace_amd.h"

namespace {

struct Args {
    std::string scene = "test_scene.txt", out = "out.bmp";
    long width = -1, height = -1, spp = -1;
    unsigned max_depth = 4;        // raytrace.rs:18
    int gpus = 1;
    unsigned band = 16;
    int algo = RT_ALGO_AUTO;
    int jitter = RT_JITTER_RANDOM;     // main.rs:51-52 jitters every sample; --jitter center = parity mode
    unsigned long long seed = 1;       // keyed draws (the reference seeds from OS entropy, main.rs:43)
};

bool parse_args(int argc, char** argv, Args& a) {
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        auto val = [&]() -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        const char* v = nullptr;
        if (k == "--scene" && (v = val())) a.scene = v;
        else if (k == "--out" && (v = val())) a.out = v;
        else if (k == "--width" && (v = val())) a.width = std::atol(v);
        else if (k == "--height" && (v = val())) a.height = std::atol(v);
        else if (k == "--spp" && (v = val())) a.spp = std::atol(v);
        else if (k == "--max-depth" && (v = val())) a.max_depth = static_cast<unsigned>(std::atol(v));
        else if (k == "--gpus" && (v = val())) a.gpus = std::atoi(v);
        else if (k == "--band" && (v = val())) a.band = static_cast<unsigned>(std::atol(v));
        else if (k == "--seed" && (v = val())) a.seed = std::strtoull(v, nullptr, 0);
        else if (k == "--jitter" && (v = val())) a.jitter = std::string(v) == "center" ? RT_JITTER_CENTER : RT_JITTER_RANDOM;
        else if (k == "--algo" && (v = val())) {
            std::string s = v;
            a.algo = s == "lds" ? RT_ALGO_BRUTE_LDS : s == "global" ? RT_ALGO_BRUTE_GLOBAL
                   : s == "wavefront" ? RT_ALGO_WAVEFRONT : s == "path" ? RT_ALGO_PATH : RT_ALGO_AUTO;
        } else {
            std::fprintf(stderr, "usage: raytrace [--scene FILE] [--out FILE] [--width W] [--height H] [--spp N]\n"
                                 "                [--max-depth D] [--gpus N] [--band ROWS] [--jitter random|center]\n"
                                 "                [--seed N] [--algo auto|wavefront|path|lds|global]\n");
            return false;
        }
    }
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    if (!parse_args(argc, argv, a)) return 2;
    std::ifstream f(a.scene, std::ios::binary);
    if (!f) { std::printf("error: cannot open %s\n", a.scene.c_str()); return 1; }   // main.rs:18
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    rt_scene* scene = nullptr;
    char err[512];
    if (rt_scene_parse(text.data(), text.size(), &scene, err, sizeof err) != RT_OK) {
        std::printf("error: %s\n", err);                                              // main.rs:28
        return 1;
    }
    rt_scene_desc d;
    rt_scene_get_desc(scene, &d);
    const uint32_t W = a.width > 0 ? static_cast<uint32_t>(a.width) : d.width;
    const uint32_t H = a.height > 0 ? static_cast<uint32_t>(a.height) : d.height;
    const uint32_t spp = a.spp > 0 ? static_cast<uint32_t>(a.spp) : d.antialias;
    int ndev = 0;
    rt_device_count(&ndev);
    if (ndev < 1) { std::printf("error: no GPU\n"); return 1; }
    const int G = std::max(1, std::min(a.gpus, ndev));
    const uint32_t band = std::max(1u, a.band);
    uint32_t pitch = 0;
    uint8_t hdr[122];
    rt_bmp_header(hdr, W, H, &pitch);
    std::vector<uint8_t> frame(static_cast<size_t>(pitch) * H, 0);
    std::vector<int> rc(G, RT_OK);
    std::vector<rt_stats> st(G);
    std::vector<std::string> errs(G);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g) {
        th.emplace_back([&, g]() {
            rt_ctx* ctx = nullptr;
            if ((rc[g] = rt_ctx_create(g, &ctx)) != RT_OK) { errs[g] = rt_last_error(nullptr); return; }
            if ((rc[g] = rt_scene_upload(ctx, scene)) != RT_OK) { errs[g] = rt_last_error(ctx); rt_ctx_destroy(ctx); return; }
            // rows of this device: bands g, g+G, g+2G, ...
            // full bands only go through the banded mapping; a ragged last band is rendered separately
            const uint32_t full_bands = H / band;
            uint32_t my_full = 0;
            for (uint32_t b = g; b < full_bands; b += G) ++my_full;
            // every device writes its bands straight into their rows of the shared frame (RT_OUT_FRAME_ROWS:
            // the library's copies of one band overlap the render of the others); the bands are disjoint rows
            rt_render_opts o;
            rt_render_opts_default(&o, W, H);
            o.max_depth = a.max_depth; o.spp = spp; o.algo = a.algo; o.jitter = a.jitter; o.seed = a.seed;
            o.flags = RT_OUT_BGR_U8 | RT_OUT_FRAME_ROWS; o.bgr_pitch = pitch;
            o.band = band; o.band_stride = G; o.band_phase = g; o.tile_h = my_full * band;
            if (o.tile_h && ((rc[g] = rt_ctx_reserve(ctx, &o, 1, nullptr)) != RT_OK ||
                             (rc[g] = rt_render(ctx, &o, nullptr, frame.data(), &st[g])) != RT_OK)) {
                errs[g] = rt_last_error(ctx); rt_ctx_destroy(ctx); return;
            }
            if (H % band && full_bands % G == static_cast<uint32_t>(g)) {   // the ragged last band
                rt_render_opts t;
                rt_render_opts_default(&t, W, H);
                t.max_depth = a.max_depth; t.spp = spp; t.algo = a.algo; t.jitter = a.jitter; t.seed = a.seed;
                t.flags = RT_OUT_BGR_U8 | RT_OUT_FRAME_ROWS; t.bgr_pitch = pitch;
                t.y0 = full_bands * band; t.tile_h = H % band;
                rt_stats ts{};
                if ((rc[g] = rt_render(ctx, &t, nullptr, frame.data(), &ts)) != RT_OK) {
                    errs[g] = rt_last_error(ctx); rt_ctx_destroy(ctx); return;
                }
                st[g].rays += ts.rays; st[g].shadow_rays += ts.shadow_rays; st[g].kernel_ms += ts.kernel_ms;
            }
            rt_ctx_destroy(ctx);
        });
    }
    for (auto& t : th) t.join();
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t rays = 0;
    double kms = 0;
    for (int g = 0; g < G; ++g) {
        if (rc[g] != RT_OK) { std::printf("error: gpu %d: %s\n", g, errs[g].c_str()); return 1; }
        rays += st[g].rays;
        kms = std::max(kms, st[g].kernel_ms);
    }
    if (rt_write_bmp(a.out.c_str(), W, H, frame.data(), pitch) != RT_OK) {
        std::printf("error: %s\n", rt_last_error(nullptr));
        return 1;
    }
    std::fprintf(stderr, "%ux%u spp=%u depth=%u gpus=%d: %llu rays, max kernel %.3f ms (%.1f Mrays/s), wall %.3f s\n",
                 W, H, spp, a.max_depth, G, static_cast<unsigned long long>(rays), kms,
                 kms > 0 ? rays / (kms * 1e3) : 0.0, sec);
    rt_scene_free(scene);
    return 0;
}
