"""Scene specifications and the seeded synthetic-scene generators.

A SceneSpec is plain Python data.  It can be emitted as text in the reference's
own scene grammar (serialize.rs:606-814) -- that text is what the product path
parses -- and converted to the oracle's structs by oracle/ref64.py, so the two
paths share nothing but these numbers.  Floats are written with repr(), which
round-trips exactly through the reference's f64::from_str (and our parser).

Configs (BASELINE.json "configs"):
  C1 test_scene.txt (IndirectPhong Cornell box; oracle-only, statistical)
  C2 1920x1080, 8 spheres + 1 plane + 2 point lights, depth 4
  C3 4096x4096, 1000 random spheres, 2 point lights, depth 8   <- headline
  C4 8192x8192, 10k spheres, depth 8
  C5 16384x16384, 100k spheres, depth 16
Random numbers come from splitmix64 so the scenes are identical on every
machine and numpy version.
"""
import colorsys
import math
from dataclasses import dataclass, field


def _f(x):
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    return repr(x)


def _t(v):
    return "(" + ", ".join(_f(x) for x in v) + ")"


def _rgb(v):
    return "rgb" + _t(v)


@dataclass
class SceneSpec:
    objects: list = field(default_factory=list)
    lights: list = field(default_factory=list)
    camera: dict = field(default_factory=dict)
    background: tuple = (0.0, 0.0, 0.0)
    width: int = 64
    height: int = 64
    antialias: int = 1
    max_depth: int = 4          # not part of the file format (raytrace.rs:18 is a constant)
    name: str = "scene"
    skybox: list = None         # six texture paths px, nx, py, ny, pz, nz (SkyboxBackground), or None

    # ---- builders ----
    def sphere(self, center, radius, material):
        self.objects.append({"shape": "sphere", "center": tuple(center), "radius": float(radius), "material": material})
        return self

    def plane(self, point, normal, material):
        self.objects.append({"shape": "plane", "point": tuple(point), "normal": tuple(normal), "material": material})
        return self

    def point_light(self, location, color):
        self.lights.append({"kind": "point", "location": tuple(location), "color": tuple(color)})
        return self

    def directional_light(self, direction, color):
        self.lights.append({"kind": "directional", "direction": tuple(direction), "color": tuple(color)})
        return self

    def area_light(self, origin, side1, side2, color):
        """AreaLight (scene.rs:142-155): a parallelogram sampled once per shading point."""
        self.lights.append({"kind": "area", "origin": tuple(origin), "side1": tuple(side1), "side2": tuple(side2),
                            "color": tuple(color)})
        return self

    def depth_of_field(self, focus_dist, aperture, samples):
        """Wrap the camera in a DepthOfFieldCamera (camera.rs:83-123)."""
        self.camera = dict(self.camera, dof=True, focus_dist=float(focus_dist), aperture=float(aperture),
                           samples=int(samples))
        return self

    # ---- reference grammar ----
    def to_text(self):
        out = ["{", "    objects: ["]
        for o in self.objects:
            out.append("        {")
            if o["shape"] == "sphere":
                out.append(f"            bounds: Sphere {{ center: {_t(o['center'])} radius: {_f(o['radius'])} }}")
            else:
                out.append(f"            bounds: Plane {{ point: {_t(o['point'])} normal: {_t(o['normal'])} }}")
            out.append("            material: " + _material_text(o["material"]))
            out.append("        }")
        out.append("    ]")
        out.append("    lights: [")
        for L in self.lights:
            if L["kind"] == "point":
                model = f"PointLight {{ location: {_t(L['location'])} }}"
            elif L["kind"] == "directional":
                model = f"DirectionalLight {{ direction: {_t(L['direction'])} }}"
            else:
                model = (f"AreaLight {{ origin: {_t(L['origin'])} side1: {_t(L['side1'])} "
                         f"side2: {_t(L['side2'])} }}")
            out.append(f"        {{ model: {model} color: {_rgb(L['color'])} }}")
        out.append("    ]")
        cam = self.camera
        if cam.get("ctor", "new") == "new":
            inner = (f"new({_t(cam['position'])}, {_t(cam['look'])}, {_t(cam['up'])}, {_f(cam['im_dist'])})")
        else:
            inner = (f"look_at({_t(cam['focus'])}, {_t(cam['look'])}, {_t(cam['up'])}, "
                     f"{_f(cam['pov'])} rad, {_f(cam['h'])})")
        if cam.get("dof"):
            out.append(f"    camera: DepthOfFieldCamera new({inner}, {_f(cam['focus_dist'])}, "
                       f"{_f(cam['aperture'])}, {int(cam['samples'])})")
        else:
            out.append(f"    camera: SimplePerspectiveCamera {inner}")
        if self.skybox:
            faces = " ".join(f'{k}: load("{p}")' for k, p in zip(("px", "nx", "py", "ny", "pz", "nz"), self.skybox))
            out.append(f"    background: SkyboxBackground {{ {faces} }}")
        else:
            out.append(f"    background: SolidColorBackground {{ color: {_rgb(self.background)} }}")
        out.append(f"    options: {{ width: {self.width} height: {self.height} antialias: {self.antialias} }}")
        out.append("}")
        return "\n".join(out) + "\n"


def phong(diffuse, specular, exponent, ambient):
    return {"kind": "phong", "diffuse": tuple(diffuse), "specular": tuple(specular),
            "exponent": float(exponent), "ambient": tuple(ambient)}


def fresnel(diffuse, specular, exponent, ambient, ior):
    """FresnelMaterial (raytrace.rs:123-167): Phong with a Schlick-weighted specular."""
    return {"kind": "fresnel", "diffuse": tuple(diffuse), "specular": tuple(specular),
            "exponent": float(exponent), "ambient": tuple(ambient), "ior": float(ior)}


def indirect_phong(diffuse, specular, exponent, ambient, samples):
    """IndirectPhongMaterial (raytrace.rs:69-121): Phong plus `samples` random bounce rays per hit."""
    return {"kind": "indirect_phong", "diffuse": tuple(diffuse), "specular": tuple(specular),
            "exponent": float(exponent), "ambient": tuple(ambient), "samples": int(samples)}


def transparent(specular, exponent, ior):
    """TransparentMaterial (raytrace.rs:169-226): Schlick-weighted reflection + refraction."""
    return {"kind": "transparent", "specular": tuple(specular), "exponent": float(exponent), "ior": float(ior)}


def _material_text(m):
    k = m["kind"]
    if k == "phong":
        return (f"PhongMaterial {{ diffuse: {_rgb(m['diffuse'])} specular: {_rgb(m['specular'])} "
                f"exponent: {_f(m['exponent'])} ambient: {_rgb(m['ambient'])} }}")
    if k == "indirect_phong":
        return (f"IndirectPhongMaterial {{ diffuse: {_rgb(m['diffuse'])} specular: {_rgb(m['specular'])} "
                f"exponent: {_f(m['exponent'])} ambient: {_rgb(m['ambient'])} samples: {int(m['samples'])} }}")
    if k == "fresnel":
        return (f"FresnelMaterial {{ diffuse: {_rgb(m['diffuse'])} specular: {_rgb(m['specular'])} "
                f"exponent: {_f(m['exponent'])} ambient: {_rgb(m['ambient'])} ior: {_f(m['ior'])} }}")
    if k == "transparent":
        return (f"TransparentMaterial {{ specular: {_rgb(m['specular'])} exponent: {_f(m['exponent'])} "
                f"ior: {_f(m['ior'])} }}")
    raise ValueError(k)


class SplitMix64:
    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def uniform(self, lo, hi):
        return lo + (hi - lo) * ((self.next() >> 11) * (1.0 / 9007199254740992.0))


DEFAULT_CAMERA = {"ctor": "new", "position": (0.0, 3.0, 10.0), "look": (0.0, -0.2, -1.0),
                  "up": (0.0, 1.0, 0.0), "im_dist": 1.5}
# A view from just in front of the random-sphere box, looking into it: under
# 20% of the camera rays miss every sphere (the default view: 71% at C3).
DENSE_CAMERA = {"ctor": "new", "position": (0.0, 3.15, -0.5), "look": (0.0, 0.0, -1.0),
                "up": (0.0, 1.0, 0.0), "im_dist": 1.5}


def _lights(spec):
    spec.point_light((-10.0, 10.0, 5.0), (0.8, 0.8, 0.8))
    spec.point_light((10.0, 8.0, 0.0), (0.6, 0.6, 0.6))


def config2(width=1920, height=1080):
    """C2: 8 spheres in a ring + ground plane + 2 point lights, depth 4 (= MAX_DEPTH)."""
    s = SceneSpec(width=width, height=height, antialias=1, max_depth=4, name="c2",
                  camera=dict(DEFAULT_CAMERA), background=(0.05, 0.05, 0.05))
    for i in range(8):
        a = 2.0 * math.pi * i / 8.0
        kd = colorsys.hsv_to_rgb(i / 8.0, 0.7, 0.9)
        s.sphere((4.0 * math.cos(a), 1.0, -6.0 + 4.0 * math.sin(a)), 1.0,
                 phong(kd, (0.3, 0.3, 0.3), 32.0, tuple(0.02 * c for c in kd)))
    s.plane((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), phong((0.6, 0.6, 0.6), (0.1, 0.1, 0.1), 16.0, (0.01, 0.01, 0.01)))
    _lights(s)
    return s


def config2_fresnel(width=1920, height=1080, max_depth=6):
    """C2 with FresnelMaterial on every other sphere (ior 1.3 .. 2.0) and on a
    mirror-like ground plane, plus a directional light."""
    s = SceneSpec(width=width, height=height, antialias=1, max_depth=max_depth, name="c2f",
                  camera=dict(DEFAULT_CAMERA), background=(0.05, 0.05, 0.05))
    for i in range(8):
        a = 2.0 * math.pi * i / 8.0
        kd = colorsys.hsv_to_rgb(i / 8.0, 0.7, 0.9)
        amb = tuple(0.02 * c for c in kd)
        if i % 2:
            m = fresnel(kd, (0.9, 0.9, 0.9), 64.0, amb, 1.3 + 0.1 * i)
        else:
            m = phong(kd, (0.3, 0.3, 0.3), 32.0, amb)
        s.sphere((4.0 * math.cos(a), 1.0, -6.0 + 4.0 * math.sin(a)), 1.0, m)
    s.sphere((0.0, 1.5, -6.0), 1.5, fresnel((0.1, 0.1, 0.1), (1.0, 1.0, 1.0), 128.0, (0.0, 0.0, 0.0), 1.5))
    s.plane((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), fresnel((0.6, 0.6, 0.6), (0.8, 0.8, 0.8), 16.0, (0.01, 0.01, 0.01), 1.33))
    _lights(s)
    s.directional_light((0.3, -1.0, -0.2), (0.3, 0.3, 0.35))
    return s


def config1(width=256, height=256, antialias=1024, max_depth=1):
    """C1: the reference's own scene, test_scene.txt (a Cornell box of
    IndirectPhongMaterial walls and spheres lit only by an emissive sphere, no
    lights; camera new((0,3,17), (0,0,-1), (0,1,0), 3.6); 1024 AA samples).
    BASELINE.json configs[0]: 256x256, depth 1."""
    s = SceneSpec(width=width, height=height, antialias=antialias, max_depth=max_depth, name="c1",
                  background=(0.051, 0.051, 0.051),
                  camera={"ctor": "new", "position": (0, 3, 17), "look": (0, 0, -1), "up": (0, 1, 0), "im_dist": 3.6})
    white = indirect_phong((1, 1, 1), (0, 0, 0), 1.0, (0, 0, 0), 1)
    s.plane((0, 0, -3), (0, 0, 1), white)
    s.plane((0, 0, 0), (0, 1.0, 0), white)
    s.plane((0, 6, 0), (0, -1.0, 0), white)
    s.plane((-3, 0, 0), (1, 0, 0), dict(white, diffuse=(1, 0, 0)))
    s.plane((3, 0, 0), (-1, 0, 0), dict(white, diffuse=(0, 1, 0)))
    s.sphere((0, 1.5, 0), 1.5, white)
    s.sphere((0, 10.65, 0), 5, dict(white, ambient=(5, 5, 5)))
    return s


def stochastic(width=96, height=64, antialias=4, max_depth=4, samples=2, dof=False, area=True):
    """Every stochastic / branching class of the reference in one scene (SURVEY.md
    §8(f) rows 3-4): glass (Transparent) and IndirectPhong spheres next to Phong and
    Fresnel ones, a ground plane, a point and an AreaLight, optionally a
    DepthOfFieldCamera.  Rendered with random jitter by the tests."""
    s = SceneSpec(width=width, height=height, antialias=antialias, max_depth=max_depth, name="stoch",
                  camera=dict(DEFAULT_CAMERA), background=(0.1, 0.12, 0.15))
    s.sphere((-2.5, 1.0, -6.0), 1.0, transparent((0.9, 0.9, 0.9), 64.0, 1.5))
    s.sphere((0.0, 1.0, -7.0), 1.0, indirect_phong((0.7, 0.3, 0.2), (0.0, 0.0, 0.0), 1.0, (0.02, 0.01, 0.0), samples))
    s.sphere((2.5, 1.0, -6.0), 1.0, fresnel((0.2, 0.3, 0.7), (0.9, 0.9, 0.9), 64.0, (0.0, 0.01, 0.02), 1.6))
    s.sphere((1.0, 0.5, -4.0), 0.5, phong((0.3, 0.8, 0.3), (0.3, 0.3, 0.3), 32.0, (0.0, 0.02, 0.0)))
    s.sphere((-1.0, 0.4, -3.5), 0.4, transparent((1.0, 1.0, 1.0), 128.0, 1.33))
    s.plane((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), indirect_phong((0.6, 0.6, 0.6), (0.0, 0.0, 0.0), 1.0,
                                                             (0.01, 0.01, 0.01), 1))
    s.point_light((-10.0, 10.0, 5.0), (0.7, 0.7, 0.7))
    if area:
        s.area_light((3.0, 8.0, -2.0), (2.0, 0.0, 0.0), (0.0, 0.0, 2.0), (0.6, 0.55, 0.5))
    if dof:
        s.depth_of_field(7.0, 0.15, 2)
    return s


def write_ppm(path, rgb):
    """Binary PPM (P6) of a uint8 [h, w, 3] array, rows top-down."""
    import numpy as np
    a = np.ascontiguousarray(rgb, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (a.shape[1], a.shape[0]))
        f.write(a.tobytes())


def skybox_faces(size=16, seed=1):
    """Six synthetic sky textures (gradients + noise, a distinct tint per face)."""
    import numpy as np
    rng = SplitMix64(seed)
    faces = []
    for k in range(6):
        yy, xx = np.mgrid[0:size, 0:size]
        base = np.stack([40 + 30 * k + 6 * xx, 200 - 8 * yy, 90 + 20 * ((xx + yy + k) % 5)], axis=-1)
        noise = np.array([rng.next() % 23 for _ in range(size * size * 3)]).reshape(size, size, 3)
        faces.append(np.clip(base + noise, 0, 255).astype(np.uint8))
    return faces


def skybox_scene(paths, width=96, height=64, max_depth=4):
    """Mirror-like Phong and Fresnel spheres reflecting a SkyboxBackground (raytrace.rs:234-256)."""
    s = SceneSpec(width=width, height=height, antialias=1, max_depth=max_depth, name="sky",
                  camera=dict(DEFAULT_CAMERA), skybox=list(paths))
    s.sphere((-1.5, 1.0, -6.0), 1.0, phong((0.1, 0.1, 0.1), (0.8, 0.8, 0.8), 64.0, (0.0, 0.0, 0.0)))
    s.sphere((1.5, 1.0, -6.0), 1.0, fresnel((0.2, 0.2, 0.3), (1.0, 1.0, 1.0), 32.0, (0.0, 0.0, 0.0), 1.5))
    s.sphere((0.0, 2.5, -9.0), 1.5, transparent((0.9, 0.9, 0.9), 64.0, 1.4))
    s.point_light((-10.0, 10.0, 5.0), (0.8, 0.8, 0.8))
    return s


def random_spheres(n, width, height, max_depth, seed, box_scale=1.0, name="rand", plane=False, view="default"):
    """C3/C4/C5 generator: centres U(x in [-8,8], y in [0.3,6], z in [-16,-2]) scaled by
    box_scale about (0, 0.3, -2); r in U[0.1,0.6]; Phong kd in U[0.1,0.9]^3,
    ks = s*(1,1,1) with s in U[0.05,0.4], exponent in U[8,128], ambient = 0.02*kd.
    view: "default" (camera at (0, 3, 10)) or "dense" (DENSE_CAMERA, inside the box's front)."""
    rng = SplitMix64(seed)
    cam = {"default": DEFAULT_CAMERA, "dense": DENSE_CAMERA}[view]
    s = SceneSpec(width=width, height=height, antialias=1, max_depth=max_depth, name=name,
                  camera=dict(cam), background=(0.05, 0.05, 0.05))
    for _ in range(n):
        cx = rng.uniform(-8.0, 8.0) * box_scale
        cy = 0.3 + rng.uniform(0.0, 5.7) * box_scale
        cz = -2.0 - rng.uniform(0.0, 14.0) * box_scale
        r = rng.uniform(0.1, 0.6)
        kd = (rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9))
        ks = rng.uniform(0.05, 0.4)
        ex = rng.uniform(8.0, 128.0)
        s.sphere((cx, cy, cz), r, phong(kd, (ks, ks, ks), ex, tuple(0.02 * c for c in kd)))
    if plane:
        s.plane((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), phong((0.5, 0.5, 0.5), (0.2, 0.2, 0.2), 24.0, (0.01, 0.01, 0.01)))
    _lights(s)
    return s


def config3(width=4096, height=4096, n=1000, view="default"):
    return random_spheres(n, width, height, 8, seed=3, name="c3", view=view)


def config4(width=8192, height=8192, n=10000):
    return random_spheres(n, width, height, 8, seed=4, box_scale=10.0 ** (1.0 / 3.0), name="c4")


def config5(width=16384, height=16384, n=100000):
    return random_spheres(n, width, height, 16, seed=5, box_scale=100.0 ** (1.0 / 3.0), name="c5")
