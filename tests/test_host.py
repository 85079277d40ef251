"""Host-side product code (no GPU): C-ABI exports, the scene parser
(serialize.rs grammar), cameras (camera.rs), sRGB quantiser (color.rs) and BMP
writer (bmp.rs) -- each checked against the oracle / the reference's goldens."""
import ctypes as C
import json
import math
import os
import random

import numpy as np
import pytest

import libraytrace as lr
from libraytrace import scenes
from oracle import ref64

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_library_exports_every_header_symbol():
    names = lr.header_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lr.lib, n), n


def test_abi_struct_sizes_match_header():
    # ctypes mirrors must agree with the C layout (checked through the library's own writers)
    assert C.sizeof(lr.rt_object) == 4 + 4 + 48 + 72 + 8 + 8 + 4 + 4
    assert C.sizeof(lr.rt_render_opts) == 16 * 4 + 8     # ABI 2: + seed
    assert C.sizeof(lr.rt_light) == 8 + 72 + 24
    assert C.sizeof(lr.rt_stats) == 10 * 8                 # `chunks` since ABI 3; unchanged at ABI 4


def test_env_tuning_is_opt_in_and_validated(monkeypatch):
    monkeypatch.setenv("RT_TUNE", "split=0, lanes=2")
    assert lr.env_tuning() == {"split": 0, "lanes": 2}
    for bad in ("split", "=3", "split=x"):
        with pytest.raises(ValueError):
            lr.env_tuning(bad)


def test_parse_reference_test_scene():
    text = open(os.path.join(GOLD, "test_scene.txt")).read()
    sc = lr.Scene.deserialize(text)
    d = sc.desc()
    assert (d.width, d.height, d.antialias) == (800, 800, 1024)
    assert d.n_objects == 7 and d.n_lights == 0
    kinds = [d.objects[i].shape for i in range(7)]
    assert kinds == [lr.RT_SHAPE_PLANE] * 5 + [lr.RT_SHAPE_SPHERE] * 2
    assert all(d.objects[i].material == lr.RT_MAT_INDIRECT_PHONG for i in range(7))
    assert tuple(d.objects[6].geom[:4]) == (0.0, 10.65, 0.0, 5.0)
    assert (d.objects[6].ambient.r, d.objects[6].samples) == (5.0, 1)
    assert tuple(d.objects[3].geom) == (-3.0, 0.0, 0.0, 1.0, 0.0, 0.0)
    assert (d.background.r, d.background.g, d.background.b) == (0.051, 0.051, 0.051)
    pos, m = ref64.camera_build({"ctor": "new", "position": (0, 3, 17), "look": (0, 0, -1),
                                 "up": (0, 1, 0), "im_dist": 3.6})
    assert tuple(d.camera.position) == pos
    assert tuple(d.camera.matrix) == m


def _desc_matches_spec(d, spec):
    assert d.n_objects == len(spec.objects)
    for i, o in enumerate(spec.objects):
        g = d.objects[i]
        if o["shape"] == "sphere":
            assert g.shape == lr.RT_SHAPE_SPHERE
            assert tuple(g.geom[:4]) == tuple(o["center"]) + (o["radius"],)
        else:
            assert g.shape == lr.RT_SHAPE_PLANE
            assert tuple(g.geom) == tuple(o["point"]) + tuple(o["normal"])
        m = o["material"]
        assert (g.diffuse.r, g.diffuse.g, g.diffuse.b) == tuple(m["diffuse"])
        assert (g.specular.r, g.specular.g, g.specular.b) == tuple(m["specular"])
        assert (g.ambient.r, g.ambient.g, g.ambient.b) == tuple(m["ambient"])
        assert g.exponent == m["exponent"]
    assert d.n_lights == len(spec.lights)


def test_generated_scene_text_round_trips_bit_exactly():
    spec = scenes.random_spheres(200, 64, 48, 8, seed=99, plane=True)
    sc = lr.Scene.deserialize(spec.to_text())
    _desc_matches_spec(sc.desc(), spec)
    spec2 = scenes.config2(96, 54)
    _desc_matches_spec(lr.Scene.deserialize(spec2.to_text()).desc(), spec2)


def test_parser_grammar_features():
    text = """
    # hash comment
    {
        // fields in any order, repeated field: last wins
        options: { width: 1 height: 1 antialias: 7 }
        options: { antialias: 2.4 height: 3 width: 4 }
        /* block
           comment */ background: SolidColorBackground { color: rgb(0.1, +2, -3e-1) }
        camera: SimplePerspectiveCamera look_at((0, 1, 2), (0, 0, -1), (0, 1, 0), 90 deg, 2)
        lights: [
            { model: DirectionalLight { direction: (0, -1, 0) } color: rgb(1, 1, 1) }
            { color: rgb(0.5, 0.5, 0.5) model: PointLight { location: (1, 2, 3) } }
        ]
        objects: [
            { bounds: Sphere { radius: 0.5 center: (1, 2, 3) }
              material: FresnelMaterial { diffuse: rgb(1,1,1) specular: rgb(0,0,0) exponent: 1 ambient: rgb(0,0,0) ior: 1.5 } }
            { bounds: Plane { point: (0, 0, 0) normal: (0, 1, 0) }
              material: TransparentMaterial { specular: rgb(1,1,1) exponent: 2 ior: 1.33 } }
        ]
    }
    trailing garbage after the scene is never read @@@
    """
    d = lr.Scene.deserialize(text).desc()
    assert (d.width, d.height, d.antialias) == (4, 3, 2)
    assert (d.background.r, d.background.g, d.background.b) == (0.1, 2.0, -0.3)
    assert d.n_lights == 2 and d.lights[0].kind == lr.RT_LIGHT_DIRECTIONAL and d.lights[1].kind == lr.RT_LIGHT_POINT
    assert d.objects[0].material == lr.RT_MAT_FRESNEL and d.objects[0].ior == 1.5
    assert d.objects[1].material == lr.RT_MAT_TRANSPARENT and d.objects[1].ior == 1.33
    pos, m = ref64.camera_build({"ctor": "look_at", "focus": (0, 1, 2), "look": (0, 0, -1), "up": (0, 1, 0),
                                 "pov": 90 * math.pi / 180.0, "h": 2})
    assert tuple(d.camera.position) == pos and tuple(d.camera.matrix) == m


def test_depth_of_field_camera_parses():
    spec = scenes.config2(8, 8)
    spec.camera = dict(spec.camera, dof=True, focus_dist=7.5, aperture=0.1, samples=16)
    d = lr.Scene.deserialize(spec.to_text()).desc()
    assert d.camera.kind == lr.RT_CAMERA_DOF and d.camera.samples == 16
    assert (d.camera.focus, d.camera.aperture) == (7.5, 0.1)


@pytest.mark.parametrize("text,code,needle", [
    ("{ bogus: 1 }", lr.RT_E_PARSE, "undefined field: bogus"),
    ("{ objects: [] lights: [] }", lr.RT_E_PARSE, "missing"),
    ("{ objects: [ @ ] }", lr.RT_E_PARSE, "invalid token"),
    ("{ objects: [] lights: [] options: { width: 1.2.3", lr.RT_E_PARSE, "invalid number"),
    ("{ objects: [ { bounds: Cube { } } ] }", lr.RT_E_PARSE, "no such class: Cube"),
    ("{ objects: [", lr.RT_E_PARSE, "end of file"),
    ("{ background: SkyboxBackground { } }", lr.RT_E_PARSE, "missing"),
    ('{ background: SkyboxBackground { px: load("/nonexistent/sky.ppm") } }', lr.RT_E_PARSE, "error loading texture"),
    ("{ /* never closed ", lr.RT_E_PARSE, "unterminated"),
    ("{ objects: [ { bounds: Sphere { center: (1 2 3) radius: 1 } } ] }", lr.RT_E_PARSE, "expected Comma"),
])
def test_parser_errors(text, code, needle):
    with pytest.raises(lr.RtError) as e:
        lr.Scene.deserialize(text)
    assert e.value.code == code
    assert needle in str(e.value)
    assert ":" in str(e.value).split(": ", 1)[1]      # "row:col: message"


def test_u32_rounding_rules():
    spec = scenes.config2(4, 4)
    text = spec.to_text().replace("antialias: 1", "antialias: -3")
    assert lr.Scene.deserialize(text).desc().antialias == 0      # negative -> 0 (serialize.rs:463-465)
    text = spec.to_text().replace("antialias: 1", "antialias: 2.5")
    assert lr.Scene.deserialize(text).desc().antialias == 3      # f64::round, half away from zero


def test_camera_builders_match_oracle():
    rnd = random.Random(5)
    for _ in range(50):
        p = [rnd.uniform(-10, 10) for _ in range(3)]
        lk = [rnd.uniform(-1, 1) for _ in range(3)]
        up = [rnd.uniform(-1, 1) for _ in range(3)]
        im = rnd.uniform(0.5, 4)
        cam = lr.camera_simple_new(p, lk, up, im)
        pos, m = ref64.camera_build({"ctor": "new", "position": p, "look": lk, "up": up, "im_dist": im})
        assert tuple(cam.position) == pos and tuple(cam.matrix) == m
        pov, h = rnd.uniform(0.2, 2.5), rnd.uniform(0.5, 5)
        cam = lr.camera_look_at(p, lk, up, pov, h)
        pos, m = ref64.camera_build({"ctor": "look_at", "focus": p, "look": lk, "up": up, "pov": pov, "h": h})
        assert tuple(cam.position) == pos and tuple(cam.matrix) == m


def test_srgb_quantiser_matches_reference_tables():
    t = json.load(open(os.path.join(GOLD, "srgb_tables.json")))
    avg = [float.fromhex(x) for x in t["SRGB_AVERAGE"]]
    for i in range(255):
        assert lr.to_srgb(avg[i]) == i + 1
        assert lr.to_srgb(math.nextafter(avg[i], -math.inf)) == i
    rnd = np.random.default_rng(0)
    vals = np.concatenate([rnd.uniform(-0.1, 1.2, 20000), [float("nan"), float("inf"), -float("inf"), 0.0, -0.0]])
    for v in vals:
        assert lr.to_srgb(v) == ref64.to_srgb(v)


def test_bmp_header_and_file(tmp_path):
    gold = bytes.fromhex(open(os.path.join(GOLD, "out_bmp_header.hex")).read().strip())
    hdr, bw = lr.bmp_header(800, 800)
    assert hdr == gold and bw == 2400
    for w, h in [(1, 1), (2, 3), (801, 5), (1920, 1080)]:
        assert lr.bmp_header(w, h) == ref64.bmp_header(w, h)
    w, h = 5, 3
    pitch = (3 * w + 3) & ~3
    rows = np.arange(h * 3 * w, dtype=np.uint8).reshape(h, 3 * w)
    p = str(tmp_path / "x.bmp")
    lr.write_bmp(p, w, h, rows, 3 * w)
    data = open(p, "rb").read()
    assert data[:122] == lr.bmp_header(w, h)[0]
    assert len(data) == 122 + pitch * h
    for y in range(h):
        assert data[122 + y * pitch:122 + y * pitch + 3 * w] == rows[y].tobytes()
        assert data[122 + y * pitch + 3 * w:122 + (y + 1) * pitch] == b"\0" * (pitch - 3 * w)


def test_device_calls_fail_loudly_without_gpu():
    if lr.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(lr.RtError) as e:
        lr.Context(0)
    assert e.value.code == lr.RT_E_NODEVICE


def test_texture_load_ppm_and_bmp(tmp_path):
    """texture.rs:34-37: RGB8, rows top-down, from binary PPM and from a BMP (bottom-up BGR rows)."""
    img = scenes.skybox_faces(size=5)[3][:, :4]            # 5 rows x 4 columns (odd row pitch in BMP)
    ppm = str(tmp_path / "a.ppm")
    scenes.write_ppm(ppm, img)
    assert np.array_equal(lr.texture_load(ppm), img)
    h, w = img.shape[:2]
    pitch = (3 * w + 3) & ~3
    rows = np.zeros((h, pitch), np.uint8)
    for y in range(h):                                       # BMP row 0 = bottom = image row h-1
        rows[y, :3 * w] = img[h - 1 - y][:, ::-1].reshape(-1)
    bmp = str(tmp_path / "a.bmp")
    lr.write_bmp(bmp, w, h, rows, pitch)
    assert np.array_equal(lr.texture_load(bmp), img)
    bad = tmp_path / "a.png"
    bad.write_bytes(b"\x89PNG\r\n\x1a\n" + bytes(64))
    with pytest.raises(lr.RtError) as e:
        lr.texture_load(str(bad))
    assert e.value.code == lr.RT_E_UNSUPPORTED


def test_texture_load_rejects_crafted_sizes(tmp_path):
    """Headers whose sizes would wrap 64-bit products or overflow int32
    are rejected before any allocation."""
    import struct
    cases = {
        "huge.ppm": b"P6\n40000000000 40000000000\n255\n" + bytes(16),
        "wide.ppm": b"P6\n4000000000 1\n255\n" + bytes(16),
        "short.ppm": b"P6\n4 4\n255\n" + bytes(47),
    }
    hdr = bytearray(54)
    hdr[0:2] = b"BM"
    struct.pack_into("<IIiiHHI", hdr, 10, 54, 40, 4, -2 ** 31, 1, 24, 0)
    cases["intmin.bmp"] = bytes(hdr) + bytes(64)
    struct.pack_into("<IIiiHHI", hdr, 10, 54, 40, 2 ** 31 - 1, 2 ** 31 - 1, 1, 24, 0)
    cases["huge.bmp"] = bytes(hdr) + bytes(64)
    for name, data in cases.items():
        f = tmp_path / name
        f.write_bytes(data)
        with pytest.raises(lr.RtError) as e:
            lr.texture_load(str(f))
        assert e.value.code in (lr.RT_E_IO, lr.RT_E_UNSUPPORTED), name


def test_parse_skybox_background(tmp_path):
    faces = scenes.skybox_faces(size=6)
    paths = [str(tmp_path / f"f{k}.ppm") for k in range(6)]
    for p, f in zip(paths, faces):
        scenes.write_ppm(p, f)
    sc = lr.Scene.deserialize(scenes.skybox_scene(paths).to_text())
    assert sc.desc().background_kind == lr.RT_BG_SKYBOX
    bad = tmp_path / "f.png"
    bad.write_bytes(b"\x89PNG" + bytes(16))
    spec = scenes.skybox_scene(paths[:5] + [str(bad)])
    with pytest.raises(lr.RtError) as e:
        lr.Scene.deserialize(spec.to_text())
    assert e.value.code == lr.RT_E_UNSUPPORTED and "f.png" in str(e.value)
    # the C ABI route: a solid-background scene turned into a skybox scene
    sc2 = lr.Scene.deserialize(scenes.config2(8, 8).to_text())
    sc2.set_skybox(faces)
    assert sc2.desc().background_kind == lr.RT_BG_SKYBOX


def test_parser_survives_mutated_scene_text():
    """Random byte edits of the reference's own scene file (tests/golden/
    test_scene.txt) never crash the parser: every result is RT_OK or RT_E_PARSE /
    RT_E_UNSUPPORTED with a message (serialize.rs:427 returns Result).  Run under
    ASan/UBSan by tools/san_check.sh."""
    import random
    text = open(os.path.join(os.path.dirname(__file__), "golden", "test_scene.txt"), "rb").read()
    rnd = random.Random(1234)
    alphabet = b"{}()[]:,.-+eE0123456789 \n\t/*\"abcxyzPhongSphere\x00\xff"
    ok = bad = 0
    for _ in range(400):
        b = bytearray(text)
        for _ in range(rnd.randint(1, 6)):
            op = rnd.random()
            i = rnd.randrange(len(b)) if b else 0
            if op < 0.4 and b:
                b[i] = rnd.choice(alphabet)
            elif op < 0.7 and b:
                del b[i:i + rnd.randint(1, 40)]
            else:
                b[i:i] = bytes(rnd.choice(alphabet) for _ in range(rnd.randint(1, 8)))
        try:
            lr.Scene.deserialize(bytes(b)).close()
            ok += 1
        except lr.RtError as e:
            assert e.code in (lr.RT_E_PARSE, lr.RT_E_UNSUPPORTED, lr.RT_E_INVALID), e
            bad += 1
    assert ok + bad == 400 and bad > 0


def test_light_grid_builder_extreme_spheres():
    """The light-grid builder on spheres that are huge, tiny, non-finite, at the
    light or enclosing it: builds, and every list query returns (ASan/UBSan run)."""
    s = scenes.SceneSpec(width=8, height=8, max_depth=2, background=(0, 0, 0),
                         camera={"ctor": "new", "position": (0, 0, 0), "look": (0, 0, -1), "up": (0, 1, 0),
                                 "im_dist": 1.0})
    m = scenes.phong((0.5, 0.5, 0.5), (0.2, 0.2, 0.2), 8.0, (0, 0, 0))
    for c, r in [((0, 0, -5), 1.0), ((1e30, 0, 0), 1e29), ((0, 0, 0), 1e-12), ((3, 3, 3), 100.0),
                 ((2, 2, 2), 0.5), ((-1e-300, 0, 1), 1e-300), ((5, 5, 5), 0.0)]:
        s.sphere(c, r, m)
    s.point_light((2, 2, 2), (1, 1, 1))
    s.point_light((1e6, -1e6, 3), (1, 1, 1))
    sc = lr.Scene.deserialize(s.to_text())
    pts = np.array([[0, 0, -4], [2, 2, 2], [1e30, 0, 0], [np.inf, 0, 0], [np.nan, 1, 1], [0, 0, 0]], np.float64)
    for li in range(2):
        cands, info = sc.light_grid_candidates(li, pts)
        assert len(cands) == len(pts) and info[0] > 0


def test_tuning_keys_listed_in_the_header():
    """Every schedule knob the library knows is named in raytrace_amd.h's
    rt_ctx_set_tuning comment, including the round-2 ones (compact_stack,
    half_nodes); no GPU needed to enumerate them."""
    keys = lr.tuning_keys()
    assert {"split", "compact_stack", "half_nodes", "src", "prefix_kb"} <= set(keys)
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "raytrace_amd.h")).read()
    block = hdr[hdr.index("Schedule tuning of a context"):hdr.index("int rt_ctx_set_tuning")]
    for k in keys:
        assert k in block, k


def test_binary16_node_bounds_round_outward():
    """host_bvh.cpp's binary16 conversion for the half-node prefix source
    (DESIGN.md §4 item 5): round_down gives the largest half <= v and round_up
    the smallest half >= v (checked against numpy's float16 neighbours), the
    decode is exact, and values beyond +-65504 or non-finite are refused (the
    tree then keeps f32 nodes).  Internal C++ helpers, reached by their
    mangled names."""
    down = lr.lib._ZN5rtamd15half_round_downEfRt
    up = lr.lib._ZN5rtamd13half_round_upEfRt
    dec = lr.lib._ZN5rtamd13half_to_floatEt
    for f in (down, up):
        f.restype, f.argtypes = C.c_bool, [C.c_float, C.POINTER(C.c_uint16)]
    dec.restype, dec.argtypes = C.c_float, [C.c_uint16]
    rng = np.random.default_rng(16)
    vals = np.concatenate([rng.uniform(-80, 80, 3000), rng.uniform(-1e-3, 1e-3, 500), 10.0 ** rng.uniform(-9, 4.8, 500),
                           [0.0, -0.0, 65504.0, -65504.0, 6.1e-5, -6.1e-5, 1e-8, 2.0 ** -24, 1.0, -1.0]]).astype(np.float32)
    h = C.c_uint16()
    for v in vals:
        v = float(v)
        assert down(v, C.byref(h))
        lo = dec(h.value)
        assert lo <= v and np.float32(lo) == np.float16(np.frombuffer(np.uint16(h.value).tobytes(), np.float16)[0])
        nxt = np.nextafter(np.float16(lo), np.float16(np.inf))
        assert float(nxt) > v or lo == v          # no larger half is <= v
        assert up(v, C.byref(h))
        hi = dec(h.value)
        assert hi >= v
        prv = np.nextafter(np.float16(hi), np.float16(-np.inf))
        assert float(prv) < v or hi == v
    for bad in (70000.0, -70000.0, float("inf"), float("nan")):
        assert not down(bad, C.byref(h)) and not up(bad, C.byref(h))
