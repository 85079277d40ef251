"""ctypes wrapper of the CPU ORACLE oracle/libref64.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this, and only as the checker / the timed CPU baseline.  See ref64.h for what it
restates and how it is pinned.
"""
import ctypes as C
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libref64.so")

REF_SPHERE, REF_PLANE = 0, 1
_MAT = {"phong": 0, "indirect_phong": 1, "fresnel": 2, "transparent": 3}
_LIGHT = {"point": 0, "directional": 1, "area": 2}


class ref_object(C.Structure):
    _fields_ = [("shape", C.c_int32), ("material", C.c_int32), ("geom", C.c_double * 6),
                ("diffuse", C.c_double * 3), ("specular", C.c_double * 3), ("ambient", C.c_double * 3),
                ("exponent", C.c_double), ("ior", C.c_double), ("samples", C.c_uint32)]


class ref_light(C.Structure):
    _fields_ = [("kind", C.c_int32), ("v", C.c_double * 9), ("color", C.c_double * 3)]


class ref_camera(C.Structure):
    _fields_ = [("ctor", C.c_int32), ("p0", C.c_double * 3), ("p1", C.c_double * 3), ("p2", C.c_double * 3),
                ("s0", C.c_double), ("s1", C.c_double), ("dof", C.c_int32), ("focus", C.c_double),
                ("aperture", C.c_double), ("dof_samples", C.c_uint32)]


class ref_texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgb", C.POINTER(C.c_uint8))]


class ref_scene(C.Structure):
    _fields_ = [("objects", C.POINTER(ref_object)), ("n_objects", C.c_uint32),
                ("lights", C.POINTER(ref_light)), ("n_lights", C.c_uint32),
                ("camera", ref_camera), ("background", C.c_double * 3),
                ("width", C.c_uint32), ("height", C.c_uint32), ("antialias", C.c_uint32),
                ("skybox", C.POINTER(ref_texture))]


def read_ppm(path):
    """Binary PPM (P6, maxval 255) -> uint8 [h, w, 3], rows top-down (the checker's own decoder)."""
    data = open(path, "rb").read()
    fields, i = [], 2
    while len(fields) < 3:
        while data[i:i + 1].isspace():
            i += 1
        if data[i:i + 1] == b"#":
            while data[i:i + 1] != b"\n":
                i += 1
            continue
        j = i
        while data[j:j + 1].isdigit():
            j += 1
        fields.append(int(data[i:j]))
        i = j
    w, h, mx = fields
    assert data[:2] == b"P6" and mx == 255
    return np.frombuffer(data[i + 1:i + 1 + w * h * 3], np.uint8).reshape(h, w, 3)


class ref_opts(C.Structure):
    _fields_ = [("max_depth", C.c_uint32), ("jitter", C.c_int32), ("seed", C.c_uint64),
                ("x0", C.c_uint32), ("tile_w", C.c_uint32), ("y0", C.c_uint32), ("tile_h", C.c_uint32),
                ("band", C.c_uint32), ("band_stride", C.c_uint32), ("band_phase", C.c_uint32),
                ("threads", C.c_int32), ("rng", C.c_int32)]


class ref_counts(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("plane_tests", C.c_uint64)]


def _load(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(f"{path} missing: run `make -C oracle`")
    lib = C.CDLL(path)
    P = C.POINTER
    lib.ref_render.restype = C.c_int
    lib.ref_render.argtypes = [P(ref_scene), P(ref_opts), P(C.c_double), P(C.c_float), P(C.c_uint8),
                               C.c_uint32, P(ref_counts)]
    lib.ref_sphere_intersect.restype = C.c_int
    lib.ref_sphere_intersect.argtypes = [P(C.c_double), C.c_double, P(C.c_double), P(C.c_double),
                                         P(C.c_double), P(C.c_double)]
    lib.ref_plane_intersect.restype = C.c_int
    lib.ref_plane_intersect.argtypes = [P(C.c_double)] * 4 + [P(C.c_double), P(C.c_double)]
    lib.ref_camera_build.restype = C.c_int
    lib.ref_camera_build.argtypes = [P(ref_camera), P(C.c_double), P(C.c_double)]
    lib.ref_to_srgb.restype = C.c_uint8
    lib.ref_to_srgb.argtypes = [C.c_double]
    lib.ref_srgb_average.restype = C.c_double
    lib.ref_srgb_average.argtypes = [C.c_int]
    lib.ref_srgb_value.restype = C.c_double
    lib.ref_srgb_value.argtypes = [C.c_int]
    lib.ref_bmp_header.restype = C.c_uint32
    lib.ref_bmp_header.argtypes = [P(C.c_uint8), C.c_uint32, C.c_uint32]
    return lib


lib = _load()

# The CPU baseline build (bench.py's cpu_baseline leg): the same ref64.c at
# -O3 -march=native, compiled on the host that runs the benchmark (the GPU
# box's CPU differs from this container's), still without FP contraction or
# fast-math, so it computes the same bits as the checker build above.
NATIVE_FLAGS = ["-O3", "-march=native", "-fPIC", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-pthread",
                "-shared"]


def native_lib():
    """(ctypes lib, compile command) of ref64.c built for this host; raises on failure."""
    import hashlib
    import subprocess
    import tempfile
    src = os.path.join(HERE, "ref64.c")
    tag = hashlib.sha1(open(src, "rb").read() + open(os.path.join(HERE, "ref64.h"), "rb").read()).hexdigest()[:12]
    out = os.path.join(tempfile.gettempdir(), f"ref64_native_{os.getuid()}_{tag}.so")
    cc = os.environ.get("CC", "gcc")
    if not os.path.exists(out):
        tmp = out + f".{os.getpid()}"
        subprocess.run([cc] + NATIVE_FLAGS + ["-o", tmp, src, "-lm"], check=True, capture_output=True)
        os.replace(tmp, out)
    return _load(out), " ".join([cc] + NATIVE_FLAGS) + " ref64.c"


def _d3(v):
    return (C.c_double * 3)(*[float(x) for x in v])


class OracleScene:
    """Keeps the ctypes arrays alive for as long as the ref_scene is used."""

    def __init__(self, spec):
        objs = (ref_object * max(1, len(spec.objects)))()
        for i, o in enumerate(spec.objects):
            r = objs[i]
            if o["shape"] == "sphere":
                r.shape = REF_SPHERE
                g = list(o["center"]) + [o["radius"], 0.0, 0.0]
            else:
                r.shape = REF_PLANE
                g = list(o["point"]) + list(o["normal"])
            r.geom[:] = [float(x) for x in g]
            m = o["material"]
            r.material = _MAT[m["kind"]]
            r.diffuse[:] = [float(x) for x in m.get("diffuse", (0, 0, 0))]
            r.specular[:] = [float(x) for x in m.get("specular", (0, 0, 0))]
            r.ambient[:] = [float(x) for x in m.get("ambient", (0, 0, 0))]
            r.exponent = float(m.get("exponent", 0.0))
            r.ior = float(m.get("ior", 0.0))
            r.samples = int(m.get("samples", 0))
        lights = (ref_light * max(1, len(spec.lights)))()
        for i, L in enumerate(spec.lights):
            r = lights[i]
            r.kind = _LIGHT[L["kind"]]
            if L["kind"] == "point":
                v = list(L["location"]) + [0.0] * 6
            elif L["kind"] == "directional":
                v = list(L["direction"]) + [0.0] * 6
            else:
                v = list(L["origin"]) + list(L["side1"]) + list(L["side2"])
            r.v[:] = [float(x) for x in v]
            r.color[:] = [float(x) for x in L["color"]]
        cam = ref_camera()
        c = spec.camera
        if c.get("ctor", "new") == "new":
            cam.ctor = 0
            cam.p0[:] = [float(x) for x in c["position"]]
            cam.s0 = float(c["im_dist"])
        else:
            cam.ctor = 1
            cam.p0[:] = [float(x) for x in c["focus"]]
            cam.s0 = float(c["pov"])
            cam.s1 = float(c["h"])
        cam.p1[:] = [float(x) for x in c["look"]]
        cam.p2[:] = [float(x) for x in c["up"]]
        if c.get("dof"):
            cam.dof = 1
            cam.focus = float(c["focus_dist"])
            cam.aperture = float(c["aperture"])
            cam.dof_samples = int(c["samples"])
        s = ref_scene()
        s.objects = objs
        s.n_objects = len(spec.objects)
        s.lights = lights
        s.n_lights = len(spec.lights)
        s.camera = cam
        s.background[:] = [float(x) for x in spec.background]
        s.width, s.height, s.antialias = spec.width, spec.height, spec.antialias
        keep = [objs, lights]
        if getattr(spec, "skybox", None):
            tex = (ref_texture * 6)()
            for t, p in zip(tex, spec.skybox):
                a = np.ascontiguousarray(read_ppm(p))
                keep.append(a)
                t.width, t.height = a.shape[1], a.shape[0]
                t.rgb = a.ctypes.data_as(C.POINTER(C.c_uint8))
            keep.append(tex)
            s.skybox = tex
        self._keep = keep
        self.scene = s


def render(spec, *, max_depth=None, x0=0, tile_w=None, y0=0, tile_h=None, band=1, band_stride=1,
           band_phase=0, jitter=0, seed=1, threads=0, want_rgb64=True, rng=0, use_lib=None):
    """Render a tile with the oracle -> dict(rgb64, rgb32, bgr, counts).
    jitter: 0 centre, 1 random; rng: 0 XorShift (the reference's generator,
    sequential), 1 keyed (the device's counter-based specification)."""
    sc = OracleScene(spec)
    tw = spec.width - x0 if tile_w is None else tile_w
    th = spec.height - y0 if tile_h is None else tile_h
    o = ref_opts(max_depth=spec.max_depth if max_depth is None else max_depth, jitter=jitter, seed=seed,
                 x0=x0, tile_w=tw, y0=y0, tile_h=th, band=band, band_stride=band_stride,
                 band_phase=band_phase, threads=threads, rng=rng)
    rgb64 = np.zeros((th, tw, 3), np.float64) if want_rgb64 else None
    rgb32 = np.zeros((th, tw, 3), np.float32)
    pitch = 3 * tw
    bgr = np.zeros((th, pitch), np.uint8)
    cnt = ref_counts()
    P = C.POINTER
    rc = (use_lib or lib).ref_render(C.byref(sc.scene), C.byref(o),
                        rgb64.ctypes.data_as(P(C.c_double)) if want_rgb64 else None,
                        rgb32.ctypes.data_as(P(C.c_float)), bgr.ctypes.data_as(P(C.c_uint8)), pitch, C.byref(cnt))
    if rc != 0:
        raise ValueError("ref_render rejected its arguments")
    return {"rgb64": rgb64, "rgb32": rgb32, "bgr": bgr,
            "counts": {"rays": cnt.rays, "shadow_rays": cnt.shadow_rays,
                       "sphere_tests": cnt.sphere_tests, "plane_tests": cnt.plane_tests}}


def sphere_intersect(center, radius, o, d):
    t = C.c_double()
    n = (C.c_double * 3)()
    h = lib.ref_sphere_intersect(_d3(center), float(radius), _d3(o), _d3(d), C.byref(t), n)
    return (t.value, tuple(n)) if h else None


def plane_intersect(point, normal, o, d):
    t = C.c_double()
    n = (C.c_double * 3)()
    h = lib.ref_plane_intersect(_d3(point), _d3(normal), _d3(o), _d3(d), C.byref(t), n)
    return (t.value, tuple(n)) if h else None


def camera_build(spec_camera):
    sc = OracleScene(type("S", (), {"objects": [], "lights": [], "camera": spec_camera, "background": (0, 0, 0),
                                    "width": 1, "height": 1, "antialias": 1})())
    pos = (C.c_double * 3)()
    m = (C.c_double * 9)()
    lib.ref_camera_build(C.byref(sc.scene.camera), pos, m)
    return tuple(pos), tuple(m)


def to_srgb(v):
    return lib.ref_to_srgb(float(v))


def bmp_header(w, h):
    buf = (C.c_uint8 * 122)()
    bw = lib.ref_bmp_header(buf, w, h)
    return bytes(buf), bw


def srgb_tables():
    return [lib.ref_srgb_value(i) for i in range(256)], [lib.ref_srgb_average(i) for i in range(255)]


__all__ = ["render", "sphere_intersect", "plane_intersect", "camera_build", "to_srgb", "bmp_header",
           "srgb_tables"]
