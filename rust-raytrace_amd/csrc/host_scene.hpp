// Host-side scene model shared by the parser, the C ABI and the device upload.
// Mirrors scene.rs:201-212 (Scene), flattened to the C ABI structs of
// include/raytrace_amd.h.
#pragma once

#include <string>
#include <vector>

#include "raytrace_amd.h"

// texture.rs:22-26: an RGB8 image, rows top-down (image crate order).
struct HostTexture {
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgb;
};

struct rt_scene {
    std::vector<rt_object> objects;     // file order == Scene::intersect order (scene.rs:248)
    std::vector<rt_light> lights;       // file order == shading order (raytrace.rs:39)
    rt_camera camera{};
    int32_t background_kind = RT_BG_SOLID;
    rt_color background{0, 0, 0};
    HostTexture skybox[6];              // SkyboxBackground px, nx, py, ny, pz, nz (scene.rs:174-188)
    uint32_t width = 0, height = 0, antialias = 1;
};

namespace rtamd {

// serialize.rs:427-441.  Returns RT_OK or RT_E_PARSE / RT_E_UNSUPPORTED with a
// "row:col: message" diagnostic in `err`.
int parse_scene_text(const std::string& text, rt_scene& out, std::string& err);

// camera.rs:51-73
void camera_simple_new(const double position[3], const double look[3], const double up[3],
                       double im_dist, rt_camera& out);
void camera_look_at(const double focus[3], const double look[3], const double up[3],
                    double pov, double h, rt_camera& out);

// texture.rs:34-37 Texture::load for the formats this build decodes (BMP
// 24/32-bit uncompressed, binary PPM P6 with maxval 255).  RT_OK or RT_E_IO /
// RT_E_UNSUPPORTED with a message.
int load_texture_file(const std::string& path, HostTexture& out, std::string& err);

// color.rs:75-332 / 335-591, generated (see host_color.cpp)
const double* srgb_average_table();   // 255 entries
const double* srgb_values_table();    // 256 entries
uint8_t to_srgb(double v);

void set_thread_error(const std::string& msg);
const char* thread_error();

}  // namespace rtamd
