"""ctypes binding of librtamd.so (include/raytrace_amd.h) for tests and bench.

The product is the C ABI + HIP kernels; this module is plumbing that lets the
pytest suite and bench.py drive it.  The names mirror the reference crate
`libraytrace` (Cargo.toml [lib] name): `Scene` (scene.rs:201), `deserialize`
(serialize.rs:427), `Context.render` (the pixel loop of main.rs:45-57),
`to_srgb` (color.rs:593), `bmp_header` (bmp.rs:10).

There is NO CPU fallback: if librtamd.so cannot be loaded the import fails,
and device calls without a GPU raise RtError.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
# RT_LIBRTAMD: an alternative build of the same library (A/B measurement)
LIB_PATH = os.environ.get("RT_LIBRTAMD") or os.path.join(PKG_DIR, "librtamd.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "raytrace_amd.h")

RT_ABI_VERSION = 5               # include/raytrace_amd.h
RT_OK = 0
RT_E_INVALID, RT_E_NODEVICE, RT_E_HIP, RT_E_NOMEM = -1, -2, -3, -4
RT_E_UNSUPPORTED, RT_E_PARSE, RT_E_NOSCENE, RT_E_IO = -5, -6, -7, -8
RT_SHAPE_SPHERE, RT_SHAPE_PLANE = 0, 1
RT_MAT_PHONG, RT_MAT_INDIRECT_PHONG, RT_MAT_FRESNEL, RT_MAT_TRANSPARENT = 0, 1, 2, 3
RT_LIGHT_POINT, RT_LIGHT_DIRECTIONAL, RT_LIGHT_AREA = 0, 1, 2
RT_CAMERA_SIMPLE, RT_CAMERA_DOF = 0, 1
RT_BG_SOLID, RT_BG_SKYBOX = 0, 1
RT_OUT_RGB_F32, RT_OUT_BGR_U8, RT_COUNT_WORK, RT_TIME_KERNELS, RT_OUT_FRAME_ROWS = 1, 2, 4, 8, 16
KERNEL_FAMILIES = ("nearest", "occlusion", "shade", "fold", "tally", "camera", "compose", "tail")   # rt_kernel_family
RT_ALGO_AUTO, RT_ALGO_BRUTE_LDS, RT_ALGO_BRUTE_GLOBAL, RT_ALGO_WAVEFRONT, RT_ALGO_WAVEFRONT_BRUTE = 0, 1, 2, 3, 4
RT_ALGO_PATH = 5
RT_JITTER_CENTER, RT_JITTER_RANDOM = 0, 1
RT_MAX_DEPTH_LIMIT = 30


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


class rt_color(C.Structure):
    _fields_ = [("r", C.c_double), ("g", C.c_double), ("b", C.c_double)]


class rt_object(C.Structure):
    _fields_ = [("shape", C.c_int32), ("material", C.c_int32), ("geom", C.c_double * 6),
                ("diffuse", rt_color), ("specular", rt_color), ("ambient", rt_color),
                ("exponent", C.c_double), ("ior", C.c_double), ("samples", C.c_uint32), ("_pad", C.c_uint32)]


class rt_light(C.Structure):
    _fields_ = [("kind", C.c_int32), ("_pad", C.c_int32), ("v", C.c_double * 9), ("color", rt_color)]


class rt_camera(C.Structure):
    _fields_ = [("kind", C.c_int32), ("samples", C.c_uint32), ("position", C.c_double * 3),
                ("matrix", C.c_double * 9), ("focus", C.c_double), ("aperture", C.c_double)]


class rt_texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgb", C.POINTER(C.c_uint8))]


class rt_scene_desc(C.Structure):
    _fields_ = [("objects", C.POINTER(rt_object)), ("n_objects", C.c_uint32),
                ("lights", C.POINTER(rt_light)), ("n_lights", C.c_uint32),
                ("camera", rt_camera), ("background_kind", C.c_int32), ("background", rt_color),
                ("width", C.c_uint32), ("height", C.c_uint32), ("antialias", C.c_uint32)]


class rt_render_opts(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("x0", C.c_uint32), ("tile_w", C.c_uint32),
                ("y0", C.c_uint32), ("tile_h", C.c_uint32), ("band", C.c_uint32), ("band_stride", C.c_uint32),
                ("band_phase", C.c_uint32), ("max_depth", C.c_uint32), ("spp", C.c_uint32),
                ("jitter", C.c_int32), ("flags", C.c_uint32), ("algo", C.c_int32),
                ("bgr_pitch", C.c_uint32), ("_pad", C.c_uint32), ("seed", C.c_uint64)]


class rt_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("pixels", C.c_uint64),
                ("kernel_ms", C.c_double), ("box_tests", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("shadow_box_tests", C.c_uint64), ("shadow_sphere_tests", C.c_uint64), ("traced_rays", C.c_uint64),
                ("chunks", C.c_uint64)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make -C rust-raytrace_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    sig = {
        "rt_scene_parse": (C.c_int, [C.c_char_p, C.c_size_t, P(C.c_void_p), C.c_char_p, C.c_size_t]),
        "rt_scene_from_desc": (C.c_int, [P(rt_scene_desc), P(C.c_void_p)]),
        "rt_scene_get_desc": (C.c_int, [C.c_void_p, P(rt_scene_desc)]),
        "rt_scene_free": (None, [C.c_void_p]),
        "rt_scene_set_skybox": (C.c_int, [C.c_void_p, P(rt_texture)]),
        "rt_texture_load": (C.c_int, [C.c_char_p, P(C.c_uint32), P(C.c_uint32), P(C.c_uint8), C.c_size_t]),
        "rt_camera_simple_new": (C.c_int, [P(C.c_double), P(C.c_double), P(C.c_double), C.c_double, P(rt_camera)]),
        "rt_camera_look_at": (C.c_int, [P(C.c_double), P(C.c_double), P(C.c_double), C.c_double, C.c_double,
                                        P(rt_camera)]),
        "rt_to_srgb": (C.c_uint8, [C.c_double]),
        "rt_bmp_header": (C.c_int, [P(C.c_uint8), C.c_uint32, C.c_uint32, P(C.c_uint32)]),
        "rt_write_bmp": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, P(C.c_uint8), C.c_uint32]),
        "rt_abi_version": (C.c_int, []),
        "rt_device_count": (C.c_int, [P(C.c_int)]),
        "rt_ctx_create": (C.c_int, [C.c_int, P(C.c_void_p)]),
        "rt_ctx_destroy": (None, [C.c_void_p]),
        "rt_last_error": (C.c_char_p, [C.c_void_p]),
        "rt_scene_upload": (C.c_int, [C.c_void_p, C.c_void_p]),
        "rt_render_opts_default": (None, [P(rt_render_opts), C.c_uint32, C.c_uint32]),
        "rt_render": (C.c_int, [C.c_void_p, P(rt_render_opts), P(C.c_float), P(C.c_uint8), P(rt_stats)]),
        "rt_render_device": (C.c_int, [C.c_void_p, P(rt_render_opts), C.c_void_p, C.c_void_p, C.c_void_p]),
        "rt_ctx_reserve": (C.c_int, [C.c_void_p, P(rt_render_opts), C.c_int, C.c_void_p]),
        "rt_ctx_stats": (C.c_int, [C.c_void_p, P(rt_stats)]),
        "rt_ctx_generation_counts": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_int]),
        "rt_ctx_kernel_times": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_uint32), C.c_int]),
        "rt_light_grid_candidates": (C.c_int, [C.c_void_p, C.c_int, C.c_int, P(C.c_double), C.c_uint32,
                                               P(C.c_int32), P(C.c_int32), C.c_size_t, P(C.c_int64)]),
        "rt_view_grid_candidates": (C.c_int, [C.c_void_p, C.c_int, P(C.c_double), C.c_uint32, P(C.c_int32),
                                              P(C.c_int32), P(C.c_float), C.c_size_t, P(C.c_int64)]),
        "rt_qtree_nodes": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, P(C.c_float), P(C.c_int32), P(C.c_int32),
                                     C.c_size_t, P(C.c_int64)]),
        "rt_div_a2_check": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double), C.c_uint32, P(C.c_double),
                                      P(C.c_double)]),
        "rt_sqrt_check": (C.c_int, [C.c_void_p, P(C.c_double), C.c_uint32, P(C.c_double), P(C.c_double)]),
        "rt_ctx_set_tuning": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64]),
        "rt_ctx_get_tuning": (C.c_int, [C.c_void_p, C.c_char_p, P(C.c_int64)]),
        "rt_tuning_key": (C.c_char_p, [C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.rt_abi_version() != RT_ABI_VERSION:      # the ctypes mirrors below follow this header version
        raise ImportError(f"{LIB_PATH} has ABI {lib.rt_abi_version()}, these bindings expect {RT_ABI_VERSION}: rebuild")
    return lib


lib = _load()


def _err(ctx=None):
    m = lib.rt_last_error(ctx)
    return m.decode(errors="replace") if m else ""


def _check(rc, ctx=None):
    if rc != RT_OK:
        raise RtError(rc, _err(ctx))


def _d3(v):
    return (C.c_double * 3)(*[float(x) for x in v])


def camera_simple_new(position, look, up, im_dist):
    """camera.rs:51-63"""
    cam = rt_camera()
    _check(lib.rt_camera_simple_new(_d3(position), _d3(look), _d3(up), float(im_dist), C.byref(cam)))
    return cam


def camera_look_at(focus, look, up, pov, h):
    """camera.rs:67-73"""
    cam = rt_camera()
    _check(lib.rt_camera_look_at(_d3(focus), _d3(look), _d3(up), float(pov), float(h), C.byref(cam)))
    return cam


def to_srgb(v):
    """color.rs:593-600"""
    return lib.rt_to_srgb(float(v))


def bmp_header(width, height):
    """bmp.rs:10-61 -> (122 header bytes, bytewidth)"""
    buf = (C.c_uint8 * 122)()
    bw = C.c_uint32()
    _check(lib.rt_bmp_header(buf, width, height, C.byref(bw)))
    return bytes(buf), bw.value


def texture_load(path):
    """texture.rs:34-37 Texture::load -> uint8 [height, width, 3], rows top-down (BMP / binary PPM)."""
    w, h = C.c_uint32(), C.c_uint32()
    _check(lib.rt_texture_load(path.encode(), C.byref(w), C.byref(h), None, 0))
    out = np.zeros((h.value, w.value, 3), np.uint8)
    _check(lib.rt_texture_load(path.encode(), C.byref(w), C.byref(h), out.ctypes.data_as(C.POINTER(C.c_uint8)),
                               out.size))
    return out


def write_bmp(path, width, height, bgr, pitch):
    arr = np.ascontiguousarray(bgr, dtype=np.uint8)
    _check(lib.rt_write_bmp(path.encode(), width, height, arr.ctypes.data_as(C.POINTER(C.c_uint8)), pitch))


class Scene:
    """A parsed / built scene (scene.rs:201-212), owned by the C library."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)

    @classmethod
    def deserialize(cls, text):
        """serialize.rs:427: parse scene text, raising RtError(RT_E_PARSE, "row:col: ...")."""
        raw = text.encode() if isinstance(text, str) else bytes(text)
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = lib.rt_scene_parse(raw, len(raw), C.byref(h), err, 512)
        if rc != RT_OK:
            raise RtError(rc, err.value.decode(errors="replace"))
        return cls(h.value)

    @classmethod
    def from_desc(cls, desc):
        h = C.c_void_p()
        _check(lib.rt_scene_from_desc(C.byref(desc), C.byref(h)))
        return cls(h.value)

    def view_grid_candidates(self, dirs, cap=1 << 23, resolution=0):
        """Diagnostic (host only): for each camera-ray direction, (object ids,
        distance bounds) the camera's view grid hands the device (None when it
        tests every sphere), and (R, stored cells, list entries)."""
        d = np.ascontiguousarray(dirs, dtype=np.float64).reshape(-1, 3)
        n = d.shape[0]
        counts = np.zeros(n, np.int32)
        ids = np.zeros(cap, np.int32)
        nears = np.zeros(cap, np.float32)
        info = np.zeros(3, np.int64)
        _check(lib.rt_view_grid_candidates(self._h, int(resolution), d.ctypes.data_as(C.POINTER(C.c_double)), n,
                                           counts.ctypes.data_as(C.POINTER(C.c_int32)),
                                           ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                           nears.ctypes.data_as(C.POINTER(C.c_float)), cap,
                                           info.ctypes.data_as(C.POINTER(C.c_int64))))
        out, at = [], 0
        for c in counts:
            if c < 0:
                out.append(None)
            else:
                out.append((ids[at:at + c].copy(), nears[at:at + c].copy()))
                at += c
        return out, tuple(int(x) for x in info)

    def light_grid_candidates(self, light, points, cap=1 << 22, resolution=0):
        """Diagnostic (host only): for each point p, the object ids the light-view
        grid of point light `light` hands a shadow query from p (None when the
        device tests every sphere), and (R, stored cells, list entries).
        resolution: cells per face side (0 = the upload's automatic choice)."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        n = pts.shape[0]
        counts = np.zeros(n, np.int32)
        ids = np.zeros(cap, np.int32)
        info = np.zeros(3, np.int64)
        _check(lib.rt_light_grid_candidates(self._h, light, int(resolution), pts.ctypes.data_as(C.POINTER(C.c_double)), n,
                                            counts.ctypes.data_as(C.POINTER(C.c_int32)),
                                            ids.ctypes.data_as(C.POINTER(C.c_int32)), cap,
                                            info.ctypes.data_as(C.POINTER(C.c_int64))))
        out, at = [], 0
        for c in counts:
            if c < 0:
                out.append(None)
            else:
                out.append(ids[at:at + c].copy())
                at += c
        return out, tuple(int(x) for x in info)

    def qtree_nodes(self, leaf_max=0, cap=1 << 16):
        """Diagnostic (host only): the quantised 4-wide tree rt_scene_upload builds
        (DevQNode4 records as a structured array, empty when not representable),
        the f32 child boxes [n, 4, 6] (lo xyz, hi xyz; NaN unused), each slot's
        leaf spheres (first, count; -1 / 0 for inner children) and (nodes, stack
        worst case, leaf size)."""
        dt = np.dtype([("frame", "<i4", 3), ("base", "<u4"), ("lo", "<u4", 3), ("hi", "<u4", 3), ("child", "<u2", 4)])
        assert dt.itemsize == 48
        nodes = np.zeros(cap, dt)
        boxes = np.zeros((cap, 4, 6), np.float32)
        first = np.zeros((cap, 4), np.int32)
        count = np.zeros((cap, 4), np.int32)
        info = np.zeros(3, np.int64)
        _check(lib.rt_qtree_nodes(self._h, int(leaf_max), nodes.ctypes.data_as(C.c_void_p),
                                  boxes.ctypes.data_as(C.POINTER(C.c_float)), first.ctypes.data_as(C.POINTER(C.c_int32)),
                                  count.ctypes.data_as(C.POINTER(C.c_int32)), cap, info.ctypes.data_as(C.POINTER(C.c_int64))))
        n = int(info[0])
        return nodes[:n].copy(), boxes[:n].copy(), first[:n].copy(), count[:n].copy(), tuple(int(x) for x in info)

    def set_skybox(self, faces):
        """SkyboxBackground { px, nx, py, ny, pz, nz } from six uint8 [h, w, 3] arrays (copied)."""
        arrs = [np.ascontiguousarray(f, dtype=np.uint8) for f in faces]
        assert len(arrs) == 6 and all(a.ndim == 3 and a.shape[2] == 3 for a in arrs)
        tex = (rt_texture * 6)()
        for t, a in zip(tex, arrs):
            t.width, t.height = a.shape[1], a.shape[0]
            t.rgb = a.ctypes.data_as(C.POINTER(C.c_uint8))
        _check(lib.rt_scene_set_skybox(self._h, tex))

    def desc(self):
        d = rt_scene_desc()
        _check(lib.rt_scene_get_desc(self._h, C.byref(d)))
        d._owner = self          # the desc borrows the scene's arrays: keep the scene alive
        return d

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib.rt_scene_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count():
    n = C.c_int(0)
    lib.rt_device_count(C.byref(n))
    return n.value


def render_opts(width, height, **kw):
    o = rt_render_opts()
    lib.rt_render_opts_default(C.byref(o), width, height)
    for k, v in kw.items():
        if not hasattr(o, k):
            raise TypeError(f"unknown render option {k}")
        setattr(o, k, v)
    return o


def sources_id():
    """16 hex digits identifying the native sources (csrc/ and include/) this
    checkout builds: ties committed profile figures (profiles/pmc_traffic.json)
    to the kernels they were measured on."""
    import hashlib
    h = hashlib.sha256()
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for d in (os.path.join(pkg, "csrc"), os.path.join(os.path.dirname(pkg), "include")):
        for name in sorted(os.listdir(d)):
            h.update(name.encode())
            with open(os.path.join(d, name), "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]


def tuning_keys():
    keys, i = [], 0
    while True:
        k = lib.rt_tuning_key(i)
        if not k:
            return keys
        keys.append(k.decode())
        i += 1


def env_tuning(text=None):
    """Tuning from RT_TUNE="key=value,key=value" (a convenience of this binding
    for A/B tools, read only when asked: Context(tuning="env"); the library
    itself never reads the environment).  Malformed items raise ValueError."""
    text = os.environ.get("RT_TUNE", "") if text is None else text
    out = {}
    for item in filter(None, (x.strip() for x in text.split(","))):
        k, sep, v = item.partition("=")
        if not sep or not k.strip():
            raise ValueError(f"RT_TUNE item {item!r} is not key=value")
        try:
            out[k.strip()] = int(v)
        except ValueError:
            raise ValueError(f"RT_TUNE item {item!r}: value is not an integer") from None
    return out


class Context:
    """One device (rt_ctx).  Mirrors the reference's main.rs render step.
    tuning: {key: value} schedule knobs (rt_ctx_set_tuning); "env" = the RT_TUNE
    environment variable (A/B tools); None = the library's defaults."""

    def __init__(self, device=0, tuning=None):
        h = C.c_void_p()
        _check(lib.rt_ctx_create(device, C.byref(h)))
        self._h = h
        self.device = device
        for k, v in (env_tuning() if tuning == "env" else (tuning or {})).items():
            self.set_tuning(k, v)

    def set_tuning(self, key, value):
        _check(lib.rt_ctx_set_tuning(self._h, key.encode(), int(value)), self._h)

    def get_tuning(self, key):
        v = C.c_int64()
        _check(lib.rt_ctx_get_tuning(self._h, key.encode(), C.byref(v)), self._h)
        return v.value

    def upload(self, scene):
        _check(lib.rt_scene_upload(self._h, scene.handle), self._h)

    def render(self, opts, rgb=True, bgr=True, out=None, stats=True):
        """Synchronous render of opts' tile into host numpy arrays.
        Returns (rgb float32 [tile_h, tile_w, 3] or None, bgr uint8 [tile_h, pitch] or None, stats).
        With RT_OUT_FRAME_ROWS in opts.flags, out= holds whole-frame arrays (height rows) and the tile's
        rows are written into their frame rows.
        out: (rgb, bgr) arrays to reuse (either None to skip that output); stats=False passes
        no rt_stats (the drop-in call of INTEGRATION.md: no counter read-back), returns None."""
        frame = bool(opts.flags & RT_OUT_FRAME_ROWS)
        pitch = opts.bgr_pitch or 3 * (opts.width if frame else opts.tile_w)
        rows, cols = (opts.height, opts.width) if frame else (opts.tile_h, opts.tile_w)
        if out is not None:
            out_rgb, out_bgr = out
            rgb, bgr = out_rgb is not None, out_bgr is not None
            assert not rgb or (out_rgb.dtype == np.float32 and out_rgb.size >= rows * cols * 3
                               and out_rgb.flags.c_contiguous)
            assert not bgr or (out_bgr.dtype == np.uint8 and out_bgr.size >= rows * pitch
                               and out_bgr.flags.c_contiguous)
        else:
            assert not frame, "RT_OUT_FRAME_ROWS renders into caller frames: pass out=(rgb, bgr)"
            out_rgb = np.zeros((opts.tile_h, opts.tile_w, 3), np.float32) if rgb else None
            out_bgr = np.full((opts.tile_h, pitch), 0xCD, np.uint8) if bgr else None
        st = rt_stats() if stats else None
        rc = lib.rt_render(self._h, C.byref(opts),
                           out_rgb.ctypes.data_as(C.POINTER(C.c_float)) if rgb else None,
                           out_bgr.ctypes.data_as(C.POINTER(C.c_uint8)) if bgr else None,
                           C.byref(st) if stats else None)
        _check(rc, self._h)
        return out_rgb, out_bgr, st

    def render_device(self, opts, d_rgb_ptr, d_bgr_ptr, stream_ptr=None):
        """Asynchronous render into device buffers (raw pointers, e.g. torch tensor.data_ptr())."""
        _check(lib.rt_render_device(self._h, C.byref(opts), C.c_void_p(d_rgb_ptr or 0),
                                    C.c_void_p(d_bgr_ptr or 0), C.c_void_p(stream_ptr or 0)), self._h)

    def reserve(self, opts, host=False, stream_ptr=None):
        """rt_ctx_reserve: allocate and warm up everything a render with opts needs (host: rt_render's
        buffers too; stream_ptr: the stream render_device will be called with), so that render runs warm."""
        _check(lib.rt_ctx_reserve(self._h, C.byref(opts), 1 if host else 0, C.c_void_p(stream_ptr or 0)), self._h)

    def stats(self):
        st = rt_stats()
        _check(lib.rt_ctx_stats(self._h, C.byref(st)), self._h)
        return st

    def generation_counts(self, n=34):
        q = (C.c_uint32 * n)()
        s = (C.c_uint32 * n)()
        _check(lib.rt_ctx_generation_counts(self._h, q, s, n), self._h)
        return list(q), list(s)

    def div_a2_check(self, x, a):
        """Diagnostic: (the sphere test's x / (2a) as the device computes it, the
        device's own f64 division) for float64 arrays x, a (rt_div_a2_check)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        a = np.ascontiguousarray(a, dtype=np.float64)
        assert x.shape == a.shape and x.ndim == 1
        fast = np.empty_like(x)
        slow = np.empty_like(x)
        P = C.POINTER(C.c_double)
        _check(lib.rt_div_a2_check(self._h, x.ctypes.data_as(P), a.ctypes.data_as(P), x.size, fast.ctypes.data_as(P),
                                   slow.ctypes.data_as(P)), self._h)
        return fast, slow

    def sqrt_check(self, x):
        """Diagnostic: (the sphere test's sqrt as the device computes it, the device's own
        f64 sqrt) for a float64 array x (rt_sqrt_check)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert x.ndim == 1
        fast = np.empty_like(x)
        slow = np.empty_like(x)
        P = C.POINTER(C.c_double)
        _check(lib.rt_sqrt_check(self._h, x.ctypes.data_as(P), x.size, fast.ctypes.data_as(P), slow.ctypes.data_as(P)),
               self._h)
        return fast, slow

    def kernel_times(self):
        """{family: (summed ms, launches)} over the RT_TIME_KERNELS renders since
        the previous call (then reset); synchronises with the last timed launch."""
        n = len(KERNEL_FAMILIES)
        ms = (C.c_double * n)()
        cnt = (C.c_uint32 * n)()
        _check(lib.rt_ctx_kernel_times(self._h, ms, cnt, n), self._h)
        return {f: (ms[i], cnt[i]) for i, f in enumerate(KERNEL_FAMILIES)}

    def close(self):
        if self._h:
            lib.rt_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def header_functions():
    """Names of every function include/raytrace_amd.h declares (for the export test)."""
    import re
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(rt_[a-z_0-9]+)\s*\(", text, flags=re.M)))
