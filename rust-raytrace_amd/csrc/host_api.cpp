// C ABI: host-side scene API (parse / build / inspect).  See include/raytrace_amd.h.
#include <cstring>
#include <new>
#include <string>

#include "host_scene.hpp"

extern "C" {

// serialize.rs:427 deserialize
int rt_scene_parse(const char* text, size_t len, rt_scene** out, char* err, size_t err_len) {
    if (!text || !out) return RT_E_INVALID;
    *out = nullptr;
    try {
        std::string src(text, len);
        auto* s = new rt_scene();
        std::string msg;
        int rc = rtamd::parse_scene_text(src, *s, msg);
        if (rc != RT_OK) {
            delete s;
            rtamd::set_thread_error(msg);
            if (err && err_len) {
                std::strncpy(err, msg.c_str(), err_len - 1);
                err[err_len - 1] = '\0';
            }
            return rc;
        }
        *out = s;
        return RT_OK;
    } catch (const std::bad_alloc&) {
        return RT_E_NOMEM;
    } catch (...) {
        return RT_E_INVALID;
    }
}

int rt_scene_from_desc(const rt_scene_desc* d, rt_scene** out) {
    if (!d || !out || (d->n_objects && !d->objects) || (d->n_lights && !d->lights)) return RT_E_INVALID;
    try {
        auto* s = new rt_scene();
        s->objects.assign(d->objects, d->objects + d->n_objects);
        s->lights.assign(d->lights, d->lights + d->n_lights);
        s->camera = d->camera;
        s->background_kind = d->background_kind;
        s->background = d->background;
        s->width = d->width;
        s->height = d->height;
        s->antialias = d->antialias;
        *out = s;
        return RT_OK;
    } catch (...) {
        return RT_E_NOMEM;
    }
}

int rt_scene_get_desc(const rt_scene* s, rt_scene_desc* out) {
    if (!s || !out) return RT_E_INVALID;
    out->objects = s->objects.data();
    out->n_objects = static_cast<uint32_t>(s->objects.size());
    out->lights = s->lights.data();
    out->n_lights = static_cast<uint32_t>(s->lights.size());
    out->camera = s->camera;
    out->background_kind = s->background_kind;
    out->background = s->background;
    out->width = s->width;
    out->height = s->height;
    out->antialias = s->antialias;
    return RT_OK;
}

void rt_scene_free(rt_scene* s) { delete s; }

int rt_abi_version(void) { return RT_ABI_VERSION; }

void rt_render_opts_default(rt_render_opts* o, uint32_t width, uint32_t height) {
    if (!o) return;
    std::memset(o, 0, sizeof *o);
    o->width = width;
    o->height = height;
    o->tile_w = width;
    o->tile_h = height;
    o->band = 1;
    o->band_stride = 1;
    o->max_depth = 4;          // raytrace.rs:18
    o->spp = 0;                // scene's antialias
    o->jitter = RT_JITTER_CENTER;
    o->flags = RT_OUT_RGB_F32 | RT_OUT_BGR_U8;
    o->algo = RT_ALGO_AUTO;
}

}  // extern "C"
