"""Parity of the HIP path (through the C ABI) with the CPU oracle.

Bar (north_star): u8 BGR bit-exact; f32 colour within 1e-5 relative of the
oracle's f64 value (RTOL below); Scene::intersect call counts identical.
The device computes in f64 with the reference's operation order, so in
practice the f32 output is bit-identical too except where OCML pow and glibc
pow differ in the last f64 ulp; that rate is reported, not asserted.
"""
import json
import os

import numpy as np
import pytest

import libraytrace as lr
from libraytrace import scenes
from oracle import ref64

pytestmark = pytest.mark.gpu

RTOL = 1e-5
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ALGOS = [lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE, lr.RT_ALGO_BRUTE_LDS, lr.RT_ALGO_BRUTE_GLOBAL]


def gpu_render(ctx, spec, algo=lr.RT_ALGO_AUTO, **kw):
    sc = lr.Scene.deserialize(spec.to_text())
    ctx.upload(sc)
    o = lr.render_opts(spec.width, spec.height, max_depth=spec.max_depth, spp=spec.antialias, algo=algo)
    for k, v in kw.items():
        setattr(o, k, v)
    rgb, bgr, st = ctx.render(o)
    return rgb, bgr, st


def check_close(rgb_gpu, rgb64):
    ref = rgb64.astype(np.float64)
    g = rgb_gpu.astype(np.float64)
    both_nan = np.isnan(ref) & np.isnan(g)
    # an f64 colour beyond the f32 range rounds to +-infinity in the f32 output (IEEE)
    with np.errstate(over="ignore"):
        ref32 = ref.astype(np.float32).astype(np.float64)
    same_inf = np.isinf(ref32) & (ref32 == g)
    ok = both_nan | same_inf | (np.abs(g - ref) <= RTOL * np.abs(ref) + 1e-300)
    assert ok.all(), f"{(~ok).sum()} colour components beyond rtol {RTOL}"
    return float(np.mean(rgb_gpu.view(np.uint32) == rgb64.astype(np.float32).view(np.uint32)))


def check_parity(ctx, spec, algo=lr.RT_ALGO_AUTO, **kw):
    rgb, bgr, st = gpu_render(ctx, spec, algo)
    ref = ref64.render(spec, **kw)
    assert np.array_equal(bgr, ref["bgr"]), f"{(bgr != ref['bgr']).sum()} BGR bytes differ"
    frac = check_close(rgb, ref["rgb64"])
    assert st.rays == ref["counts"]["rays"]
    assert st.shadow_rays == ref["counts"]["shadow_rays"]
    return frac, st


@pytest.mark.parametrize("algo", ALGOS)
def test_config2_full_size(gpu_ctx, algo):
    frac, st = check_parity(gpu_ctx, scenes.config2(), algo)
    assert st.pixels == 1920 * 1080
    print(f"C2 1920x1080 algo={algo}: f32 bit-identical fraction {frac:.6f}, rays {st.rays}")


@pytest.mark.parametrize("algo", ALGOS)
def test_config3_downscaled(gpu_ctx, algo):
    frac, st = check_parity(gpu_ctx, scenes.config3(256, 256), algo)
    print(f"C3 256x256 algo={algo}: f32 bit-identical fraction {frac:.6f}, rays {st.rays}")


@pytest.mark.parametrize("algo", ALGOS)
def test_fresnel_material(gpu_ctx, algo):
    """FresnelMaterial (raytrace.rs:123-167) on spheres and the ground plane,
    with point and directional lights: Schlick factor from the unflipped n.d,
    Fresnel-weighted specular, fresnel*sig*ks.sig significance and the
    (ks * child) * fresnel fold."""
    frac, st = check_parity(gpu_ctx, scenes.config2_fresnel(320, 180), algo)
    print(f"C2-Fresnel 320x180 algo={algo}: f32 bit-identical fraction {frac:.6f}, rays {st.rays}")


def test_fresnel_random_spheres_deep(gpu_ctx):
    """A third of C3's spheres turned Fresnel, depth 16: mixed Phong / Fresnel
    chains through the BVH paths."""
    spec = scenes.config3(192, 128)
    spec.max_depth = 16
    for i, o in enumerate(spec.objects):
        if i % 3 == 0:
            m = o["material"]
            o["material"] = scenes.fresnel(m["diffuse"], (0.95, 0.95, 0.95), m["exponent"], m["ambient"],
                                           1.2 + 0.05 * (i % 16))
    check_parity(gpu_ctx, spec)


def test_config3_full_size_sampled_rows(gpu_ctx):
    """The headline config at full size: every 256th row (16 rows x 4096 px)
    checked against the oracle, plus frame-level properties."""
    spec = scenes.config3()
    rgb, bgr, st = gpu_render(gpu_ctx, spec)
    assert st.pixels == 4096 * 4096
    ref = ref64.render(spec, y0=0, tile_h=16, band=1, band_stride=256, band_phase=0)
    rows = np.arange(16) * 256
    assert np.array_equal(bgr[rows], ref["bgr"])
    check_close(rgb[rows], ref["rgb64"])
    # every ray issued either hits or escapes; a frame issues >= 1 query per pixel
    assert st.rays >= st.pixels and st.shadow_rays <= 2 * (st.rays - st.shadow_rays)
    assert np.isfinite(rgb).all()


@pytest.mark.parametrize("name", ["c2_96x54", "c3_64x64", "mirror16_48x40", "c2fresnel_80x45"])
def test_golden_fixtures(gpu_ctx, name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    sc = lr.Scene.deserialize(str(z["scene_text"]))
    gpu_ctx.upload(sc)
    d = sc.desc()
    o = lr.render_opts(d.width, d.height, max_depth=int(z["max_depth"]), spp=d.antialias)
    rgb, bgr, st = gpu_ctx.render(o)
    assert np.array_equal(bgr.reshape(z["bgr"].shape), z["bgr"])
    assert np.allclose(rgb, z["rgb32"], rtol=RTOL, atol=0)
    assert st.rays == int(z["rays"]) and st.shadow_rays == int(z["shadow_rays"])


def _tiny(**kw):
    s = scenes.SceneSpec(width=kw.pop("width", 8), height=kw.pop("height", 8), max_depth=kw.pop("max_depth", 4),
                         background=(0.2, 0.3, 0.4),
                         camera={"ctor": "new", "position": (0, 0, 0), "look": (0, 0, -1), "up": (0, 1, 0),
                                 "im_dist": 1.0})
    return s


def test_nan_plane_wins(gpu_ctx):
    # camera ray inside a plane: t = 0/0 = NaN wins over a nearer sphere (scene.rs:223-249)
    s = _tiny(width=9, height=9)
    s.sphere((0, 0, -5), 1.0, scenes.phong((0.5, 0.5, 0.5), (0.3, 0.3, 0.3), 8.0, (0, 1, 0)))
    s.plane((0, 0, 0), (0, 1, 0), scenes.phong((0.1, 0.2, 0.3), (0.2, 0.2, 0.2), 4.0, (0, 0, 1)))
    s.point_light((3, 3, 3), (1, 1, 1))
    s.directional_light((0, -1, 0.2), (0.5, 0.5, 0.5))
    check_parity(gpu_ctx, s)


def test_directional_lights_and_parallel_planes(gpu_ctx):
    s = scenes.config2(64, 48)
    s.directional_light((0.3, -1.0, -0.2), (0.4, 0.4, 0.4))
    s.directional_light((0.0, 0.0, 1.0), (0.3, 0.1, 0.1))        # parallel to the ground plane
    s.plane((0, 5, 0), (0, -1, 0), scenes.phong((0.3, 0.3, 0.3), (0.0, 0.0, 0.0), 2.0, (0.0, 0.0, 0.0)))
    check_parity(gpu_ctx, s)


@pytest.mark.parametrize("algo", [lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE, lr.RT_ALGO_BRUTE_LDS])
def test_extreme_light_and_plane_magnitudes(gpu_ctx, algo):
    """Operands outside the window of the sphere test's hoisted division
    (trace_common.hpp div_a2: 2a in [2^-100, 2^101)): a directional light of
    magnitude 1e-35 (its shadow rays keep the unnormalised -direction, a = 1e-70),
    one of magnitude 1e34, and mirror planes with normals of length 1e25 and 1e-20
    (reflection directions d - 2n(d.n) far from unit length), over random spheres:
    the image and ray counts stay the oracle's bit for bit."""
    s = scenes.random_spheres(60, 64, 48, 6, seed=33, plane=False)
    s.lights = []
    s.directional_light((3e-36, -1e-35, -2e-36), (0.5, 0.5, 0.4))
    s.directional_light((2e33, -1e34, 1e33), (0.0, 0.0, 0.0))       # (black: its shadow rays still run)
    s.point_light((0.0, 8.0, 2.0), (0.6, 0.6, 0.6))
    s.plane((0.0, -0.5, 0.0), (0.0, 1e25, 0.0), scenes.phong((0.2, 0.2, 0.2), (0.6, 0.6, 0.6), 10.0, (0.01, 0.01, 0.01)))
    s.plane((0.0, 0.0, -40.0), (0.0, 3e-21, 1e-20), scenes.phong((0.3, 0.2, 0.1), (0.5, 0.5, 0.5), 10.0, (0.0, 0.0, 0.0)))
    check_parity(gpu_ctx, s, algo)


def test_coincident_objects_first_wins(gpu_ctx):
    s = _tiny(width=16, height=16)
    a = scenes.phong((0.9, 0.1, 0.1), (0.2, 0.2, 0.2), 10.0, (0.1, 0, 0))
    b = scenes.phong((0.1, 0.9, 0.1), (0.2, 0.2, 0.2), 10.0, (0, 0.1, 0))
    s.sphere((0.3, 0, -4), 1.0, a)
    s.sphere((0.3, 0, -4), 1.0, b)
    s.plane((0, -1, 0), (0, 1, 0), a)
    s.plane((0, -1, 0), (0, 1, 0), b)
    s.point_light((2, 3, 0), (1, 1, 1))
    check_parity(gpu_ctx, s)


@pytest.mark.parametrize("depth", [0, 1, 16, lr.RT_MAX_DEPTH_LIMIT])
def test_depths(gpu_ctx, depth):
    s = scenes.random_spheres(30, 40, 32, depth, seed=21, plane=True)
    for o in s.objects:
        o["material"] = dict(o["material"], specular=(0.95, 0.9, 0.85))   # ks.sig > 1: never insignificant
    check_parity(gpu_ctx, s)


def test_antialias_samples_average(gpu_ctx):
    s = scenes.config2(40, 24)
    s.antialias = 3
    check_parity(gpu_ctx, s)


def test_empty_scene_and_single_pixel(gpu_ctx):
    s = _tiny(width=1, height=1)
    check_parity(gpu_ctx, s)
    s = _tiny(width=13, height=7)
    s.point_light((0, 1, 0), (1, 1, 1))
    check_parity(gpu_ctx, s)


def test_tiles_offsets_and_bands_match_oracle(gpu_ctx):
    spec = scenes.config2(67, 41)
    sc = lr.Scene.deserialize(spec.to_text())
    gpu_ctx.upload(sc)
    for (x0, tw, y0, th, band, stride, phase) in [(0, 67, 0, 41, 1, 1, 0), (5, 17, 3, 13, 1, 1, 0),
                                                   (0, 67, 0, 12, 4, 3, 1), (10, 50, 1, 15, 5, 2, 1)]:
        o = lr.render_opts(67, 41, x0=x0, tile_w=tw, y0=y0, tile_h=th, band=band, band_stride=stride,
                           band_phase=phase, max_depth=4, spp=1, bgr_pitch=3 * tw + 5)
        rgb, bgr, st = gpu_ctx.render(o)
        ref = ref64.render(spec, x0=x0, tile_w=tw, y0=y0, tile_h=th, band=band, band_stride=stride,
                           band_phase=phase)
        assert np.array_equal(bgr[:, :3 * tw], ref["bgr"])
        assert (bgr[:, 3 * tw:] == 0).all()           # BMP row padding (main.rs:42)
        check_close(rgb, ref["rgb64"])
        assert st.rays == ref["counts"]["rays"]


def test_sharded_frame_is_bit_identical(gpu_ctx):
    """Multi-GPU decomposition (row bands dealt round-robin over N devices) is a
    pure function of the rows: the reassembled frame equals the untiled one."""
    spec = scenes.config3(128, 96)
    sc = lr.Scene.deserialize(spec.to_text())
    gpu_ctx.upload(sc)
    full = gpu_ctx.render(lr.render_opts(128, 96, max_depth=8, spp=1))
    for n in (2, 3, 8):
        band = 4
        frame_bgr = np.zeros_like(full[1])
        frame_rgb = np.zeros_like(full[0])
        rays = 0
        nb = 96 // band
        for r in range(n):
            mine = len(range(r, nb, n))
            if mine == 0:
                continue
            o = lr.render_opts(128, 96, tile_h=mine * band, band=band, band_stride=n, band_phase=r,
                               max_depth=8, spp=1)
            rgb, bgr, st = gpu_ctx.render(o)
            rays += st.rays
            for j in range(mine * band):
                y = ((j // band) * n + r) * band + j % band
                frame_bgr[y] = bgr[j]
                frame_rgb[y] = rgb[j]
        assert np.array_equal(frame_bgr, full[1])
        assert np.array_equal(frame_rgb.view(np.uint32), full[0].view(np.uint32))
        assert rays == full[2].rays


def test_stochastic_classes_need_the_path_kernel(gpu_ctx):
    """test_scene.txt (IndirectPhongMaterial) and a DepthOfFieldCamera upload, but
    only the path kernel renders them: the chain algorithms fail loudly."""
    text = open(os.path.join(GOLD, "test_scene.txt")).read()
    gpu_ctx.upload(lr.Scene.deserialize(text))
    o = lr.render_opts(16, 16, spp=1, max_depth=1)
    for algo in (lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE, lr.RT_ALGO_BRUTE_GLOBAL):
        o.algo = algo
        with pytest.raises(lr.RtError) as e:
            gpu_ctx.render(o)
        assert e.value.code == lr.RT_E_UNSUPPORTED
    o.algo = lr.RT_ALGO_AUTO
    _, _, st = gpu_ctx.render(o)
    assert st.rays > 0
    s = scenes.config2(8, 8)
    s.camera = dict(s.camera, dof=True, focus_dist=5.0, aperture=0.1, samples=4)
    gpu_ctx.upload(lr.Scene.deserialize(s.to_text()))
    with pytest.raises(lr.RtError) as e:
        gpu_ctx.render(lr.render_opts(8, 8, spp=1, algo=lr.RT_ALGO_WAVEFRONT))
    assert e.value.code == lr.RT_E_UNSUPPORTED


def test_render_without_scene_and_bad_opts():
    with lr.Context(0) as ctx:
        with pytest.raises(lr.RtError) as e:
            ctx.render(lr.render_opts(8, 8, spp=1))
        assert e.value.code == lr.RT_E_NOSCENE
        ctx.upload(lr.Scene.deserialize(scenes.config2(8, 8).to_text()))
        for bad in (dict(max_depth=lr.RT_MAX_DEPTH_LIMIT + 1, spp=1), dict(spp=1, x0=5),
                    dict(spp=1, band_stride=2, band_phase=2), dict(spp=1, bgr_pitch=3)):
            with pytest.raises(lr.RtError) as e:
                ctx.render(lr.render_opts(8, 8, **bad))
            assert e.value.code == lr.RT_E_INVALID


# ---- BVH culling must be conservative: adversarial scenes ------------------

def _nan_plane_scene():
    """test_nan_plane_wins's camera-in-a-plane scene (NaN plane hits) with 60
    more spheres, so that the wave query has several clusters to cull."""
    s = _tiny(width=17, height=13)
    s.max_depth = 5
    s.sphere((0, 0, -5), 1.0, scenes.phong((0.5, 0.5, 0.5), (0.3, 0.3, 0.3), 8.0, (0, 1, 0)))
    rng = scenes.SplitMix64(21)
    for k in range(60):
        c = (rng.uniform(-4, 4), rng.uniform(-3, 3), rng.uniform(-12, -3))
        s.sphere(c, rng.uniform(0.1, 0.8), scenes.phong((0.4, 0.5, 0.6), (0.5, 0.5, 0.5), 20.0, (0, 0, 0)))
    s.plane((0, 0, 0), (0, 1, 0), scenes.phong((0.1, 0.2, 0.3), (0.2, 0.2, 0.2), 4.0, (0, 0, 1)))
    s.point_light((3, 3, 3), (1, 1, 1))
    s.directional_light((0, -1, 0.2), (0.5, 0.5, 0.5))
    return s


def _axis_tie_scene():
    s = scenes.SceneSpec(width=33, height=31, max_depth=6, background=(0.1, 0.1, 0.2),
                         camera={"ctor": "new", "position": (0, 0, 0), "look": (0, 0, -1), "up": (0, 1, 0),
                                 "im_dist": 1.0})
    rng = scenes.SplitMix64(77)
    for k in range(24):
        kd = (rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(0, 1))
        s.sphere((0.0, 0.0, -6.0), 1.5, scenes.phong(kd, (0.3, 0.3, 0.3), 20.0, (0.01, 0.01, 0.01)))
    for k in range(300):     # clutter so the duplicates spread over the tree
        c = (rng.uniform(-6, 6), rng.uniform(-6, 6), rng.uniform(-20, -3))
        s.sphere(c, rng.uniform(0.05, 0.5), scenes.phong((0.5, 0.5, 0.5), (0.4, 0.4, 0.4), 30.0, (0, 0, 0)))
    # spheres exactly tangent to the axis rays and to each other
    s.sphere((1.0, 0.0, -10.0), 1.0, scenes.phong((0.9, 0.2, 0.2), (0.5, 0.5, 0.5), 8.0, (0, 0, 0)))
    s.sphere((-1.0, 0.0, -10.0), 1.0, scenes.phong((0.2, 0.9, 0.2), (0.5, 0.5, 0.5), 8.0, (0, 0, 0)))
    s.point_light((0.0, 5.0, 0.0), (1, 1, 1))
    s.directional_light((0.0, -1.0, 0.0), (0.3, 0.3, 0.3))
    return s


@pytest.mark.parametrize("algo", [lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE])
def test_axis_aligned_rays_and_ties_across_leaves(gpu_ctx, algo):
    """Odd image sizes put pixel centres exactly on the camera axes (direction
    components exactly 0); 24 coincident spheres with different colours land in
    different BVH leaves and must still resolve to the FIRST in file order."""
    check_parity(gpu_ctx, _axis_tie_scene(), algo)


@pytest.mark.parametrize("scene", ["axis_ties", "sphere_chain", "config3", "planes_nan", "fresnel"])
def test_fused_tail_matches_oracle(gpu_ctx, scene):
    """The fused tail (tuning tail_fuse = T, trace_kernel.hip wf_tail): every
    chain still running at generation T-1 goes from its shade record through
    all its remaining bounces -- light-view grid shadows, Phong sum,
    reflection, nearest hit -- in one launch, one chain per work-item, and
    folds it there, the chains that ended earlier being folded on a B stream
    meanwhile.  From generation 1 (nearly the whole recursion) to 4, on ties
    across leaves, the deepest small tree, NaN planes, Fresnel levels and a C3
    workload: bit for bit the oracle's image, and the same ray and shadow-ray
    counts (the tail publishes every generation's queue and record counts).
    The timed render checks that the tail really ran: one tail launch,
    nearest-hit launches for generations 1 .. T-1 only, shadow and shading
    launches for 0 .. T-2, and the fold of the chains that ended by T-1."""
    def fresnel():
        s = scenes.config3(96, 72)
        s.max_depth = 10
        for i in range(0, len(s.objects), 3):
            s.objects[i]["material"] = scenes.fresnel((0.3, 0.4, 0.5), (0.7, 0.7, 0.7), 30.0, (0.01, 0.01, 0.01), 1.5)
        return s
    s = {"axis_ties": _axis_tie_scene, "sphere_chain": _sphere_chain_scene, "config3": lambda: scenes.config3(160, 128),
         "planes_nan": _nan_plane_scene, "fresnel": fresnel}[scene]()
    # (the tail answers shadows through light-view grids only: directional lights become point lights far away)
    s.lights = [l if l["kind"] == "point" else
                {"kind": "point", "location": tuple(-40.0 * x for x in l["direction"]), "color": l["color"]} for l in s.lights]
    for T in (1, 2, 3, 4):
        with _with_tuning(gpu_ctx, tail_fuse=T):
            check_parity(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)
            gpu_ctx.kernel_times()
            gpu_ctx.render(lr.render_opts(s.width, s.height, max_depth=s.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT,
                                          flags=lr.RT_OUT_BGR_U8 | lr.RT_TIME_KERNELS))
            kt = gpu_ctx.kernel_times()
        if T <= s.max_depth + 1:
            assert kt["nearest"][1] == T - 1 and kt["tail"][1] == 1, (T, kt)     # generations 1 .. T-1, the tail
            assert kt["occlusion"][1] == T - 1 and kt["shade"][1] == T - 1, (T, kt)   # generations 0 .. T-2
            assert kt["fold"][1] == 1, (T, kt)     # the chains that ended by T-1


@pytest.mark.parametrize("scene", ["axis_ties", "config3", "dense", "planes_nan", "config4", "camera_inside"])
def test_camera_view_grid_matches_oracle(gpu_ctx, scene):
    """Generation 0 through the camera's view grid (tuning cam 3, trace_common.hpp
    nearest_cgrid; spheres in LDS, or through L2 for 10k spheres): camera rays
    on the axes, coincident spheres, NaN planes, the camera inside spheres and
    the C3 / C4 workloads match the oracle bit for bit."""
    def camera_inside():
        s = scenes.SceneSpec(width=41, height=29, max_depth=3, background=(0.1, 0.2, 0.3),
                             camera={"ctor": "new", "position": (0.0, 0.0, 0.0), "look": (0.0, 0.0, -1.0),
                                     "up": (0.0, 1.0, 0.0), "im_dist": 1.0})
        rng = scenes.SplitMix64(31)
        for k in range(200):
            c = (rng.uniform(-6, 6), rng.uniform(-4, 4), rng.uniform(-15, 3))
            s.sphere(c, rng.uniform(0.05, 1.0), scenes.phong((0.4, 0.5, 0.6), (0.5, 0.5, 0.5), 20.0, (0.01, 0, 0)))
        s.sphere((0.2, 0.0, 0.0), 0.5, scenes.phong((0.9, 0.1, 0.1), (0.3, 0.3, 0.3), 8.0, (0.1, 0, 0)))
        s.point_light((2, 3, 1), (1, 1, 1))
        return s
    s = {"axis_ties": _axis_tie_scene, "config3": lambda: scenes.config3(160, 128),
         "dense": lambda: scenes.config3(128, 96, view="dense"), "planes_nan": _nan_plane_scene,
         "config4": lambda: scenes.config4(96, 80), "camera_inside": camera_inside}[scene]()
    with _with_tuning(gpu_ctx, cam=3):                       # (check_parity uploads: the grid is built then)
        check_parity(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)
    with _with_tuning(gpu_ctx, cam=3, cam_grid_res=7):       # a coarse grid: long lists, same bits
        check_parity(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)


@pytest.mark.parametrize("algo", [lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE])
def test_extreme_sphere_sizes_and_far_plane_origins(gpu_ctx, algo):
    s = scenes.config2(97, 61)
    s.max_depth = 8
    rng = scenes.SplitMix64(5)
    for k in range(200):
        c = (rng.uniform(-30, 30), rng.uniform(0.001, 4), rng.uniform(-60, 0))
        s.sphere(c, 10 ** rng.uniform(-4, 0.3), scenes.phong((0.3, 0.6, 0.9), (0.6, 0.6, 0.6), 50.0, (0, 0, 0)))
    s.sphere((0.0, -1e4 + 0.0, -5.0), 1e4, scenes.phong((0.2, 0.2, 0.2), (0.5, 0.5, 0.5), 5.0, (0, 0, 0)))
    s.sphere((1e5, 3.0, -1e5), 2e3, scenes.phong((0.9, 0.9, 0.2), (0.2, 0.2, 0.2), 5.0, (0, 0, 0)))
    check_parity(gpu_ctx, s, algo)


def _sphere_chain_scene():
    s = scenes.config2(80, 60)
    s.max_depth = 6
    for i in range(46):
        r = 0.9 * 2.0 ** -i            # sphere i at x = -2 + 4 (1 - 2^-i): each level of the SAH peels one
        s.sphere((-2.0 + 4.0 * (1.0 - 2.0 ** -i), 1.5, -6.0), r,
                 scenes.phong((0.5, 0.4, 0.3), (0.5, 0.5, 0.5), 20.0, (0.01, 0.01, 0.01)))
    rng = scenes.SplitMix64(9)
    for _ in range(150):
        s.sphere((rng.uniform(-6, 6), rng.uniform(0.2, 4), rng.uniform(-14, -3)), rng.uniform(0.05, 0.4),
                 scenes.phong((0.3, 0.6, 0.9), (0.4, 0.4, 0.4), 30.0, (0, 0, 0)))
    return s


def test_chain_of_shrinking_spheres_both_stacks(gpu_ctx):
    """A chain of spheres halving in size and spacing toward x = 2 inside a
    random cloud: the binned SAH peels a few spheres per level, giving the
    deepest tree a scene this small reaches (still within the compact stack's
    32 entries: tools/schedule_probe.py prints short_stack 1; a binned SAH
    re-bins every node over its own extent, so depth > 32 needs far more
    spheres than the compact source's 4096).  Compact 32-bit entries (src 9)
    and the 64-bit stack (compact_stack=0, src 7) both match the oracle bit
    for bit."""
    s = _sphere_chain_scene()
    check_parity(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)
    base = gpu_render(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)
    with _with_tuning(gpu_ctx, compact_stack=0):
        wide = gpu_render(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)
    assert np.array_equal(base[1], wide[1]) and base[2].rays == wide[2].rays


@pytest.mark.parametrize("algo", [lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE])
def test_light_view_grids_adversarial_lights(gpu_ctx, algo):
    """Point-light shadows through the light-view grids (host_lightgrid.cpp):
    lights inside the sphere cloud (boxes straddling the light's axis planes,
    every cube face populated), a light inside a sphere and one on a sphere's
    surface (the always list), shade points close to a light, spheres from
    1e-3 to 1e3, a plane through a light.  Every shadow answer must be the
    linear scan's (the oracle)."""
    s = scenes.SceneSpec(width=81, height=67, max_depth=6, background=(0.05, 0.05, 0.1),
                         camera={"ctor": "new", "position": (0, 2, 12), "look": (0, -0.1, -1), "up": (0, 1, 0),
                                 "im_dist": 1.2})
    rng = scenes.SplitMix64(4242)
    for k in range(400):
        c = (rng.uniform(-6, 6), rng.uniform(-2, 6), rng.uniform(-10, 2))
        kd = (rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9))
        s.sphere(c, 10 ** rng.uniform(-3, -0.2), scenes.phong(kd, (0.3, 0.3, 0.3), 20.0, (0.01, 0.01, 0.01)))
    s.sphere((3.0, 1.0, -4.0), 0.8, scenes.phong((0.8, 0.8, 0.2), (0.4, 0.4, 0.4), 10.0, (0, 0, 0)))
    s.sphere((0.0, -1e3 - 2.5, -4.0), 1e3, scenes.phong((0.5, 0.5, 0.5), (0.2, 0.2, 0.2), 5.0, (0, 0, 0)))
    s.plane((0.0, 0.0, -30.0), (0.0, 0.0, 1.0), scenes.phong((0.3, 0.3, 0.3), (0.0, 0.0, 0.0), 1.0, (0, 0, 0)))
    s.point_light((0.0, 2.0, -4.0), (0.6, 0.6, 0.6))          # inside the cloud
    s.point_light((3.0, 1.0, -4.0), (0.5, 0.2, 0.2))          # at the centre of a sphere
    s.point_light((3.0, 1.8, -4.0), (0.2, 0.5, 0.2))          # on that sphere's surface
    s.point_light((-5.0, 0.5, -30.0), (0.2, 0.2, 0.5))        # on the plane
    s.directional_light((0.2, -1.0, -0.1), (0.2, 0.2, 0.2))   # no grid: the tree
    check_parity(gpu_ctx, s, algo)


def test_light_view_grids_off_is_bit_identical(gpu_ctx):
    """Tuning light_grids=0 (shadow queries through the 4-wide tree) and the default
    grids give the same bytes, colours and ray counts on the 10k-sphere scene."""
    spec = scenes.config4(160, 120)
    a = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    gpu_ctx.set_tuning("light_grids", 0)
    try:
        b = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    finally:
        gpu_ctx.set_tuning("light_grids", 1)
    assert np.array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert a[2].rays == b[2].rays and a[2].shadow_rays == b[2].shadow_rays


def test_bvh_ten_thousand_spheres(gpu_ctx):
    s = scenes.config4(96, 96)
    check_parity(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)


def test_half_node_prefix_source_is_bit_identical(gpu_ctx):
    """C4's workload (10k spheres: the f32 tree exceeds LDS): the nearest-hit walk
    over binary16 nodes (bounds rounded outward, twice the nodes in the LDS
    prefix; the default), over f32 nodes and over the quantised 4-wide tree
    (whole in LDS, or mostly through L2) give the same bytes, colours and rays,
    equal to the oracle's; also with a 1 KB prefix, so most nodes come from HBM/L2."""
    spec = scenes.config4(128, 96)
    ref = ref64.render(spec, threads=min(16, os.cpu_count() or 1))
    base = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    assert np.array_equal(base[1], ref["bgr"])
    assert base[2].rays == ref["counts"]["rays"]
    for kv in [dict(qtree=1), dict(half_nodes=0), dict(prefix_kb=1), dict(half_nodes=0, prefix_kb=1), dict(split=1),
               dict(qtree=1, split=0), dict(prefix_kb=1, src=26, src_occ=11), dict(cam=0)]:
        with _with_tuning(gpu_ctx, **kv):
            got = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
        assert np.array_equal(got[1], base[1]), kv
        assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32)), kv
        assert got[2].rays == base[2].rays and got[2].shadow_rays == base[2].shadow_rays, kv


@pytest.mark.parametrize("scene", ["axis_ties", "sphere_chain", "config3", "planes_nan", "extreme", "config4"])
def test_quantised_tree_matches_oracle(gpu_ctx, scene):
    """The quantised 4-wide tree (trace_common.hpp nearest_q4; host_bvh.cpp
    quantize_bvh4) forced onto every nearest-hit generation: whole in LDS (src
    25) and with a 1 KB LDS prefix, every other node read through L2 (src 26).
    Ties across leaves, axis-aligned rays, the deepest small tree, NaN planes,
    spheres from 1e-4 to 1e4 (coarse frames), C3 and C4 workloads: bit for bit
    the oracle's image and ray counts."""
    def extreme():
        s = scenes.config2(57, 41)
        s.max_depth = 8
        rng = scenes.SplitMix64(9)
        for k in range(150):
            c = (rng.uniform(-30, 30), rng.uniform(0.001, 4), rng.uniform(-60, 0))
            s.sphere(c, 10 ** rng.uniform(-4, 0.3), scenes.phong((0.3, 0.6, 0.9), (0.6, 0.6, 0.6), 50.0, (0, 0, 0)))
        s.sphere((0.0, -1e4 + 0.0, -5.0), 1e4, scenes.phong((0.2, 0.2, 0.2), (0.5, 0.5, 0.5), 5.0, (0, 0, 0)))
        s.sphere((1e5, 3.0, -1e5), 2e3, scenes.phong((0.9, 0.9, 0.2), (0.2, 0.2, 0.2), 5.0, (0, 0, 0)))
        return s
    s = {"axis_ties": _axis_tie_scene, "sphere_chain": _sphere_chain_scene, "config3": lambda: scenes.config3(160, 128),
         "planes_nan": _nan_plane_scene, "extreme": extreme, "config4": lambda: scenes.config4(96, 80)}[scene]()
    for kv in (dict(src=25, src_occ=11), dict(src=26, src_occ=11, prefix_kb=1)):
        with _with_tuning(gpu_ctx, verbose=1, **kv):
            check_parity(gpu_ctx, s, lr.RT_ALGO_WAVEFRONT)


def test_bvh_matches_brute_force_bit_for_bit_full_frame(gpu_ctx):
    """Headline scene, full 4096x4096: BVH and linear scan agree on every byte
    and every ray (a size-independent property of conservative culling)."""
    spec = scenes.config3()
    a = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    b = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT_BRUTE)
    assert np.array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert a[2].rays == b[2].rays and a[2].shadow_rays == b[2].shadow_rays


def test_work_counters(gpu_ctx):
    """RT_COUNT_WORK: identical image; brute force tests every sphere for every
    nearest query; the BVH tests a subset."""
    spec = scenes.config3(64, 48)
    sc = lr.Scene.deserialize(spec.to_text())
    gpu_ctx.upload(sc)
    base = dict(max_depth=8, spp=1)
    plain = gpu_ctx.render(lr.render_opts(64, 48, algo=lr.RT_ALGO_WAVEFRONT, **base))
    counted = gpu_ctx.render(lr.render_opts(64, 48, algo=lr.RT_ALGO_WAVEFRONT, flags=7, **base))
    assert np.array_equal(plain[1], counted[1]) and plain[2].rays == counted[2].rays
    brute = gpu_ctx.render(lr.render_opts(64, 48, algo=lr.RT_ALGO_WAVEFRONT_BRUTE, flags=7, **base))[2]
    nearest = brute.rays - brute.shadow_rays
    assert brute.sphere_tests - brute.shadow_sphere_tests == nearest * 1000
    assert brute.box_tests == 0
    bvh = counted[2]
    assert 0 < bvh.sphere_tests < brute.sphere_tests
    assert bvh.box_tests > 0
    q, s = gpu_ctx.generation_counts()
    assert sum(q[1:]) + 64 * 48 == nearest


def test_kernel_times(gpu_ctx):
    """RT_TIME_KERNELS: identical image; one interval per launch, accumulated
    over renders until harvested."""
    spec = scenes.config3(64, 48)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    base = dict(max_depth=8, spp=1, algo=lr.RT_ALGO_WAVEFRONT)
    with _with_tuning(gpu_ctx, tail_fuse=0):               # one launch set per generation (no fused tail)
        _kernel_times_per_generation(gpu_ctx, base)


def _kernel_times_per_generation(gpu_ctx, base):
    plain = gpu_ctx.render(lr.render_opts(64, 48, **base))
    gpu_ctx.kernel_times()
    timed = [gpu_ctx.render(lr.render_opts(64, 48, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_TIME_KERNELS,
                                           **base)) for _ in range(2)]
    for t in timed:
        assert np.array_equal(plain[1], t[1])
    kt = gpu_ctx.kernel_times()
    gens = 8 + 2
    assert kt["camera"][1] == 2 and kt["nearest"][1] == 2 * (gens - 1)
    # shadow queries and shading of the lit generations 0..max_depth (none past the cut-off)
    assert kt["occlusion"][1] == 2 * (gens - 1) and kt["shade"][1] == 2 * (gens - 1)   # config3 has lights
    assert kt["tail"][1] == 0
    assert kt["compose"][1] == 2 * gpu_ctx.get_tuning("compose")      # one row-ordered frame pass per render
    # frame-end fold: one launch per chunk, in chain order; the tally of a one-chunk render runs
    # only when its statistics are read (rt_render's stats, after the render: not a frame launch)
    assert kt["fold"][1] == 2 and kt["tally"][1] == 0
    assert all(ms > 0 for ms, n in kt.values() if n)
    assert all(n == 0 for ms, n in gpu_ctx.kernel_times().values())   # harvested


def _with_tuning(ctx, **kv):
    """Context manager: set tuning keys, restore the previous values after."""
    import contextlib

    @contextlib.contextmanager
    def cm():
        old = {k: ctx.get_tuning(k) for k in kv}
        try:
            for k, v in kv.items():
                ctx.set_tuning(k, v)
            yield
        finally:
            for k, v in old.items():
                ctx.set_tuning(k, v)
    return cm()


def test_config5_workload_downscaled(gpu_ctx):
    """BASELINE config 5's workload (100k spheres, depth 16, 2 point lights) at
    128x96: a tree far larger than LDS (the LDS-prefix sources), the linear-scan
    semantics of scene.rs:247-249 over 100k objects, and the raytrace.rs:33
    cut-off after 17 levels.  Rendered as one chunk and as three chunks of 32
    rows (tuning chunk_pixels), both against the oracle bit for bit."""
    spec = scenes.config5(128, 96)
    ref = ref64.render(spec, threads=min(16, os.cpu_count() or 1))
    rgb, bgr, st = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    assert np.array_equal(bgr, ref["bgr"]), f"{(bgr != ref['bgr']).sum()} BGR bytes differ"
    check_close(rgb, ref["rgb64"])
    assert st.rays == ref["counts"]["rays"] and st.shadow_rays == ref["counts"]["shadow_rays"]
    with _with_tuning(gpu_ctx, chunk_pixels=128 * 32):
        rgb2, bgr2, st2 = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    assert np.array_equal(bgr2, bgr) and np.array_equal(rgb2.view(np.uint32), rgb.view(np.uint32))
    assert st2.rays == st.rays and st2.shadow_rays == st.shadow_rays


@pytest.mark.parametrize("lanes", [1, 2])
def test_multi_chunk_schedule_matches_oracle(gpu_ctx, lanes):
    """The wavefront schedule over many chunks (row0 > 0), on one or two chunk
    lanes, for a plain tile and for a banded tile (band_stride > 1, band_phase
    > 0): bit-identical to the one-chunk render and to the oracle."""
    spec = scenes.config3(256, 256)
    sc = lr.Scene.deserialize(spec.to_text())
    gpu_ctx.upload(sc)
    layouts = [dict(tile_h=256), dict(y0=0, tile_h=80, band=8, band_stride=3, band_phase=1)]
    for lay in layouts:
        o = lr.render_opts(256, 256, max_depth=spec.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT, **lay)
        one = gpu_ctx.render(o)
        with _with_tuning(gpu_ctx, chunk_pixels=256 * 16, lanes=lanes):
            many = gpu_ctx.render(o)
        with _with_tuning(gpu_ctx, chunk_pixels=256 * 8, lanes=lanes):      # > 16 chunks: copied after the render
            many8 = gpu_ctx.render(o)
        assert np.array_equal(many8[1], one[1]) and np.array_equal(many8[0].view(np.uint32), one[0].view(np.uint32))
        assert np.array_equal(many[1], one[1])
        assert np.array_equal(many[0].view(np.uint32), one[0].view(np.uint32))
        assert many[2].rays == one[2].rays and many[2].shadow_rays == one[2].shadow_rays
        kw = {k: v for k, v in lay.items()}
        ref = ref64.render(spec, **kw)
        assert np.array_equal(many[1], ref["bgr"])
        check_close(many[0], ref["rgb64"])
        assert many[2].rays == ref["counts"]["rays"]


def test_working_set_budget_splits_chunks_bit_identically(gpu_ctx):
    """The wavefront working set is sized from a budget (tuning wf_budget_mb;
    default: the device's free memory): a C4-workload tile (10k spheres, depth
    8) under a small budget runs as several row chunks, bit-identical to the
    one-chunk render."""
    spec = scenes.config4(1024, 768)
    base = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    assert base[2].chunks == 1
    with _with_tuning(gpu_ctx, wf_budget_mb=100):
        got = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    assert got[2].chunks > 2, got[2].chunks
    assert np.array_equal(got[1], base[1])
    assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32))
    assert got[2].rays == base[2].rays and got[2].shadow_rays == base[2].shadow_rays


def test_oversized_budget_falls_back_to_smaller_chunks():
    """A budget beyond the device's 288 GB (the whole 16384^2 depth-16 tile in
    one chunk needs ~0.5 TB): the working set does not fit the free device
    memory (checked before hipMalloc, which has crashed inside the runtime on
    requests that size), the render halves its chunks until it fits, and the
    image equals the default schedule's.
    Own context, closed at the end (its working set is large)."""
    spec = scenes.random_spheres(40, 16384, 16384, 16, seed=11, name="sparse")
    o = lr.render_opts(16384, 16384, max_depth=16, spp=1, algo=lr.RT_ALGO_WAVEFRONT)
    with lr.Context(0) as ctx:
        ctx.upload(lr.Scene.deserialize(spec.to_text()))
        _, ref, st0 = ctx.render(o, rgb=False)
    with lr.Context(0, tuning={"wf_budget_mb": 600_000}) as ctx:
        ctx.upload(lr.Scene.deserialize(spec.to_text()))
        _, got, st = ctx.render(o, rgb=False)
    assert st.chunks >= 2
    assert np.array_equal(got, ref) and st.rays == st0.rays


def test_tuning_knobs_do_not_change_results(gpu_ctx):
    """Schedule knobs (one stream, per-ray camera rays, workgroup-first dealing,
    other region counts and stream counts, other sphere sources, the fused tail
    from several generations and widths) leave every bit of a C3-workload frame
    unchanged."""
    spec = scenes.config3(192, 160)
    base = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    for kv in [dict(split=0), dict(cam=0), dict(deal=0), dict(regions=96), dict(bstreams=1), dict(bstreams=3),
               dict(src=2, src_occ=11), dict(compact_stack=0), dict(src=7, src_occ=10), dict(src=7, src_occ=7),
               dict(src=25, src_occ=11), dict(prio=0), dict(grid_occ=0), dict(spread_below=1 << 20),
               dict(tail_fuse=1), dict(tail_fuse=3, regions=96), dict(tail_fuse=5, bstreams=1), dict(tail_fuse=2, deal=0),
               dict(tail_fuse=4, tail_width=64), dict(tail_fuse=6, tail_width=7), dict(tail_fuse=3, split=0),
               dict(compose=0), dict(compose=0, tail_fuse=3), dict(compose=0, cam=0), dict(compose=1),
               dict(dev_join=0), dict(dev_join=0, tail_fuse=0), dict(dev_join=1, tail_fuse=0, bstreams=3),
               dict(chain_on_caller=0), dict(chain_on_caller=0, dev_join=0), dict(copy_engine=0), dict(copy_engine=1)]:
        with _with_tuning(gpu_ctx, **kv):
            got = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
        assert np.array_equal(got[1], base[1]), kv
        assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32)), kv
        assert got[2].rays == base[2].rays, kv


@pytest.mark.parametrize("compose", [1, 0])
def test_row_ordered_compose_matches_oracle(gpu_ctx, compose):
    """The row-ordered frame pass (tuning compose, trace_kernel.hip wf_compose):
    widths around the 64-pixel segment (1, 63, 64, 65, 130, 197), tight BGR rows
    (3 w bytes: byte stores) and dword-padded rows with extra slack (dword
    stores, the padding zeroed), misses, ambient ends and chains in one frame:
    the oracle's BGR bytes and f32 colours either way, with and without the
    fused tail."""
    for w, h in [(1, 5), (63, 9), (64, 7), (65, 11), (130, 6), (197, 13)]:
        spec = scenes.config3(w, h)
        spec.max_depth = 3
        ref = ref64.render(spec)
        for tail in (0, 2):
            with _with_tuning(gpu_ctx, compose=compose, tail_fuse=tail):
                gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
                for pitch in (0, ((3 * w + 3) & ~3) + 8):
                    o = lr.render_opts(w, h, max_depth=spec.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT, bgr_pitch=pitch)
                    rgb, bgr, st = gpu_ctx.render(o)
                    assert np.array_equal(bgr[:, :3 * w], ref["bgr"]), (w, h, tail, pitch)
                    assert (bgr[:, 3 * w:] == 0).all(), (w, h, tail, pitch)
                    check_close(rgb, ref["rgb64"])
                    assert st.rays == ref["counts"]["rays"]


def test_host_chunks_overlap_copies_bit_identically(gpu_ctx):
    """rt_render into host memory in several chunks (tuning host_chunks,
    host_first: each chunk's rows copied while the next one renders): the same
    bytes and colours as one chunk, rows split unevenly, on one and two lanes."""
    spec = scenes.config3(200, 147)
    base = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
    for kv in [dict(host_chunks=2), dict(host_chunks=3), dict(host_chunks=2, host_first=30),
               dict(host_chunks=2, host_first=70, lanes=2), dict(host_chunks=5, lanes=2)]:
        with _with_tuning(gpu_ctx, **kv):
            got = gpu_render(gpu_ctx, spec, lr.RT_ALGO_WAVEFRONT)
        assert np.array_equal(got[1], base[1]), kv
        assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32)), kv
        assert got[2].rays == base[2].rays, kv
        assert got[2].chunks == kv["host_chunks"] and base[2].chunks == 1, kv


@pytest.mark.parametrize("scene", ["config3", "config2", "fresnel"])
def test_sparse_host_copies_bit_identical(gpu_ctx, scene):
    """rt_render into host memory with tuning sparse_out (rt_device.cpp
    copy_sparse: the frame copied after the camera pass, then the packed
    segments of the chain pixels scattered into it): every byte and colour as
    the plain copy, into buffers holding garbage, for widths around the
    16-pixel segment, padded rows, BGR only, RGB only, with and without the
    fused tail.  (sparse_out is the default: every other rt_render parity test
    runs it against the oracle too.)"""
    for w, h in [(197, 64), (64, 40), (33, 17), (1, 9)]:
        spec = {"config3": scenes.config3, "config2": scenes.config2, "fresnel": scenes.config2_fresnel}[scene](w, h)
        gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
        for pitch in (0, ((3 * w + 3) & ~3) + 8):
            o = lr.render_opts(w, h, max_depth=spec.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT, bgr_pitch=pitch)
            with _with_tuning(gpu_ctx, sparse_out=0):
                base = gpu_ctx.render(o)
            for kv in [dict(sparse_out=1), dict(sparse_out=1, tail_fuse=0)]:
                for outs in [(True, True), (False, True), (True, False)]:
                    rgb = np.full_like(base[0], np.nan) if outs[0] else None
                    bgr = np.full_like(base[1], 0xAB) if outs[1] else None
                    with _with_tuning(gpu_ctx, **kv):
                        got = gpu_ctx.render(o, out=(rgb, bgr))
                    if outs[1]:
                        assert np.array_equal(got[1], base[1]), (w, h, pitch, kv, outs)
                    if outs[0]:
                        assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32)), (w, h, pitch, kv, outs)


def _hip():
    import ctypes as C
    return C.CDLL("libamdhip64.so.7")      # the HIP runtime librtamd.so runs on (already loaded: by soname)


class _Pinned:
    """A page-locked host array (hipHostMalloc of the HIP runtime librtamd.so uses): rt_render DMAs
    into it directly instead of through its staging slices."""

    def __init__(self, shape, dtype, fill):
        import ctypes as C
        self.hip = _hip()
        self.p = C.c_void_p()
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        assert self.hip.hipHostMalloc(C.byref(self.p), C.c_size_t(nbytes), 0) == 0
        self.arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.p.value)).view(dtype).reshape(shape)
        self.arr[...] = fill

    def free(self):
        self.arr = None
        self.hip.hipHostFree(self.p)


@pytest.mark.parametrize("scene", ["config3", "fresnel"])
def test_sparse_host_copies_banded_tiles(gpu_ctx, scene):
    """Sparse copies for row-band tiles (a rank's share of a multi-GPU frame:
    band_stride > 1, band_phase > 0, a ragged band count), into pageable and
    page-locked buffers holding garbage: every byte and colour as the plain
    copy (sparse_out 0)."""
    w, h = 197, 160
    spec = {"config3": scenes.config3, "fresnel": scenes.config2_fresnel}[scene](w, h)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    for band, stride, phase, pitch in [(16, 2, 1, 0), (16, 3, 0, 604), (8, 8, 7, 0), (5, 4, 2, 0)]:
        rows = sum(min(band, h - b * band) for b in range(phase, (h + band - 1) // band, stride)
                   if (b + 1) * band <= h)           # whole bands only (check_opts: the tile stays in the frame)
        o = lr.render_opts(w, h, max_depth=spec.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT, band=band,
                           band_stride=stride, band_phase=phase, tile_h=rows, bgr_pitch=pitch)
        with _with_tuning(gpu_ctx, sparse_out=0):
            base = gpu_ctx.render(o)
        for pinned in (False, True):
            for outs in [(True, True), (False, True), (True, False)]:
                mk = (lambda s, d, f: _Pinned(s, d, f)) if pinned else (lambda s, d, f: type("A", (), {
                    "arr": np.full(s, f, d), "free": lambda self: None})())
                rgb = mk(base[0].shape, np.float32, np.nan) if outs[0] else None
                bgr = mk(base[1].shape, np.uint8, 0xAB) if outs[1] else None
                try:
                    with _with_tuning(gpu_ctx, sparse_out=1):
                        got = gpu_ctx.render(o, out=(rgb.arr if rgb else None, bgr.arr if bgr else None))
                    if outs[1]:
                        assert np.array_equal(got[1], base[1]), (band, stride, phase, pitch, pinned, outs)
                    if outs[0]:
                        assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32)), (band, stride, phase,
                                                                                                  pinned, outs)
                finally:
                    for a in (rgb, bgr):
                        if a:
                            a.free()


@pytest.mark.parametrize("engine", [0, -1, 1])
def test_sparse_host_copies_large_tile_pinned(gpu_ctx, engine):
    """A tile large enough that the frame copy and the 16 packed row ranges
    really overlap the generations (1024 x 512, depth 8), into a page-locked
    and a pageable buffer: bit for bit the plain copy; the copies
    through hipMemcpyAsync (engine 0) or an SDMA engine (tuning copy_engine)."""
    spec = scenes.config3(1024, 512)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    o = lr.render_opts(1024, 512, max_depth=8, spp=1)
    with _with_tuning(gpu_ctx, sparse_out=0, copy_engine=0):
        base = gpu_ctx.render(o)
    rgb, bgr = _Pinned(base[0].shape, np.float32, np.nan), _Pinned(base[1].shape, np.uint8, 0x5A)
    try:
        with _with_tuning(gpu_ctx, copy_engine=engine):
            for _ in range(2):
                got = gpu_ctx.render(o, out=(rgb.arr, bgr.arr))
                assert np.array_equal(got[1], base[1])
                assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32))
                rgb.arr[...] = np.nan
                bgr.arr[...] = 0x5A
    finally:
        rgb.free()
        bgr.free()
    for sparse in (1, 0):
        with _with_tuning(gpu_ctx, copy_engine=engine, sparse_out=sparse):
            got = gpu_ctx.render(o, out=(np.full_like(base[0], np.nan), np.full_like(base[1], 0x5A)))
        assert np.array_equal(got[1], base[1]), sparse
        assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32)), sparse


@pytest.mark.parametrize("sparse,engine", [(1, 0), (0, 0), (1, -1), (0, -1), (1, 1)])
def test_frame_rows_gather_matches_whole_frame(gpu_ctx, sparse, engine):
    """RT_OUT_FRAME_ROWS (the multi-GPU host gather, main.rs:45-58 split over
    devices): N "ranks" render their 16-row bands straight into one shared
    frame (page-locked, like bench.py's shared frame, and pageable), each
    writing only its rows; with a ragged last band rendered as its own tile,
    a padded BMP pitch, and a partial-width tile (columns x0.. of the frame):
    the frame equals the whole-frame render bit for bit, and the oracle's.
    engine: the copies through hipMemcpyAsync (0) or an SDMA engine driven
    directly (tuning copy_engine: -1 engines 0-3 in turn, 1 engine 0 alone).
    Each layout is rendered three times (ordering races between the copies and
    the host scatter show up on first use, tools/copy_stress.py)."""
    W, H, band = 150, 100, 16
    spec = scenes.config3(W, H)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    pitch = (3 * W + 3) & ~3
    whole = gpu_ctx.render(lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, bgr_pitch=pitch))
    ref = ref64.render(spec)
    assert np.array_equal(whole[1][:, :3 * W], ref["bgr"])
    full = H // band
    for n, pinned in [(3, True), (2, False), (1, True), (2, True)]:
        mk = (lambda s, d, f: _Pinned(s, d, f)) if pinned else (lambda s, d, f: type("A", (), {
            "arr": np.full(s, f, d), "free": lambda self: None})())
        rgb, bgr = mk((H, W, 3), np.float32, np.nan), mk((H, pitch), np.uint8, 0xAB)
        try:
            with _with_tuning(gpu_ctx, sparse_out=sparse, copy_engine=engine):
                for r in range(n):
                    nb = len(range(r, full, n))
                    o = lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, band=band, band_stride=n, band_phase=r,
                                       tile_h=nb * band, bgr_pitch=pitch,
                                       flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS)
                    gpu_ctx.render(o, out=(rgb.arr, bgr.arr))
                # the ragged last band (rows full*band .. H-1) as one more tile
                o = lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, y0=full * band, tile_h=H - full * band,
                                   bgr_pitch=pitch, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS)
                gpu_ctx.render(o, out=(rgb.arr, bgr.arr))
            assert np.array_equal(bgr.arr, whole[1]), (n, pinned)
            assert np.array_equal(rgb.arr.view(np.uint32), whole[0].view(np.uint32)), (n, pinned)
            for rep in range(3):
                # a partial-width tile (columns 40..139 of rows 20..59) lands in its columns; the rest is untouched
                bgr.arr[...] = 0xAB
                rgb.arr[...] = np.nan
                with _with_tuning(gpu_ctx, sparse_out=sparse, copy_engine=engine):
                    o = lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, x0=40, tile_w=100, y0=20, tile_h=40,
                                       bgr_pitch=pitch, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS)
                    gpu_ctx.render(o, out=(rgb.arr, bgr.arr))
                assert np.array_equal(bgr.arr[20:60, 120:420], whole[1][20:60, 120:420]), (n, pinned, rep)
                assert (bgr.arr[20:60, :120] == 0xAB).all() and (bgr.arr[20:60, 420:] == 0xAB).all()
                assert (bgr.arr[:20] == 0xAB).all() and (bgr.arr[60:] == 0xAB).all()
                assert np.array_equal(rgb.arr[20:60, 40:140].view(np.uint32), whole[0][20:60, 40:140].view(np.uint32))
                assert np.isnan(rgb.arr[20:60, :40]).all() and np.isnan(rgb.arr[20:60, 140:]).all()
                # ... and the tile at the right edge writes the BMP row padding (zero)
                bgr.arr[...] = 0xAB
                with _with_tuning(gpu_ctx, sparse_out=sparse, copy_engine=engine):
                    o = lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, x0=50, tile_w=W - 50, y0=0, tile_h=8,
                                       bgr_pitch=pitch, flags=lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS)
                    gpu_ctx.render(o, out=(None, bgr.arr))
                assert np.array_equal(bgr.arr[:8, 150:], whole[1][:8, 150:]), (n, pinned, rep)
                assert (bgr.arr[:8, 3 * W:] == 0).all() and (bgr.arr[:8, :150] == 0xAB).all()
        finally:
            rgb.free()
            bgr.free()


def test_frame_rows_rejects_bad_layouts(gpu_ctx):
    spec = scenes.config3(64, 32)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    fr = lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS
    bgr = np.zeros((32, 64 * 3), np.uint8)
    with pytest.raises(lr.RtError) as e:          # a frame pitch below 3 * width
        gpu_ctx.render(lr.render_opts(64, 32, tile_w=32, bgr_pitch=100, flags=fr, max_depth=2), out=(None, bgr))
    assert e.value.code == lr.RT_E_INVALID
    with pytest.raises(lr.RtError) as e:          # device buffers have no frame rows
        gpu_ctx.render_device(lr.render_opts(64, 32, flags=fr, max_depth=2), 0, 1 << 40)
    assert e.value.code == lr.RT_E_INVALID


def test_reserve_then_render_is_unchanged(gpu_ctx):
    """rt_ctx_reserve allocates and warms up without rendering: the render after
    it gives the same bytes and counts as without it, the statistics of the
    render before it are untouched, and reserving for a render already
    prepared is cheap (no allocation)."""
    import time
    spec = scenes.config3(256, 192)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    o = lr.render_opts(256, 192, max_depth=8, spp=1)
    rgb0, bgr0, st0 = gpu_ctx.render(o)
    gpu_ctx.reserve(o, host=True)
    gpu_ctx.reserve(o, host=False)
    assert gpu_ctx.stats().rays == st0.rays
    t0 = time.perf_counter()
    gpu_ctx.reserve(o, host=True)
    assert time.perf_counter() - t0 < 0.5
    rgb1, bgr1, st1 = gpu_ctx.render(o)
    assert np.array_equal(bgr1, bgr0) and np.array_equal(rgb1.view(np.uint32), rgb0.view(np.uint32))
    assert st1.rays == st0.rays
    with lr.Context(0) as fresh:                    # a fresh context: reserve before its first render
        with pytest.raises(lr.RtError) as e:
            fresh.reserve(o)
        assert e.value.code == lr.RT_E_NOSCENE
        fresh.upload(lr.Scene.deserialize(spec.to_text()))
        fresh.reserve(o, host=True)
        rgb2, bgr2, st2 = fresh.render(o)
    assert np.array_equal(bgr2, bgr0) and np.array_equal(rgb2.view(np.uint32), rgb0.view(np.uint32))


def test_default_spp_is_the_scenes_antialias(gpu_ctx):
    """rt_render_opts.spp = 0 (the default options) renders with the uploaded
    scene's Options.antialias (scene.rs:191-198)."""
    spec = scenes.config2(40, 24)
    spec.antialias = 3
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    o = lr.render_opts(40, 24, max_depth=spec.max_depth)
    assert o.spp == 0
    rgb, bgr, st = gpu_ctx.render(o)
    ref = ref64.render(spec)
    assert np.array_equal(bgr, ref["bgr"])
    assert st.rays == ref["counts"]["rays"]
    assert st.traced_rays * 3 == st.rays        # centre jitter: one traced sample counted 3 times


_TWO_STREAMS = r"""
import sys
sys.path[:0] = sys.argv[1:3]
import numpy as np
import torch                      # first: the process then uses torch's HIP runtime for both
import libraytrace as lr
from libraytrace import scenes
from oracle import ref64
spec = scenes.config3(128, 128)
dev = torch.device("cuda", 0)
outs = [(torch.empty((128, 128, 3), dtype=torch.float32, device=dev),
         torch.empty((128, 384), dtype=torch.uint8, device=dev)) for _ in range(2)]
streams = [torch.cuda.Stream(dev) for _ in range(2)]
with lr.Context(0) as ctx:
    ctx.upload(lr.Scene.deserialize(spec.to_text()))
    o = lr.render_opts(128, 128, max_depth=spec.max_depth, spp=1)
    ref = ref64.render(spec)
    for join in (1, 0):                       # b streams joined on the device / through events
        ctx.set_tuning("dev_join", join)
        for t in outs:
            t[1].fill_(0)
        for _ in range(3):
            for (a, b), s in zip(outs, streams):
                ctx.render_device(o, a.data_ptr(), b.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        for a, b in outs:
            assert np.array_equal(b.cpu().numpy(), ref["bgr"]), join
    # a plain rt_render_device records no start event: kernel_ms 0; with RT_TIME_KERNELS it is timed
    assert ctx.stats().kernel_ms == 0.0
    ot = lr.render_opts(128, 128, max_depth=spec.max_depth, spp=1,
                        flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_TIME_KERNELS)
    ctx.render_device(ot, outs[0][0].data_ptr(), outs[0][1].data_ptr(), streams[0].cuda_stream)
    torch.cuda.synchronize(dev)
    assert ctx.stats().kernel_ms > 0.0
    ctx.kernel_times()
print("ordered ok")
"""


def test_renders_on_two_streams_are_ordered():
    """Two asynchronous renders of one context on different (torch) streams share
    its working set; the second waits for the first on the device.
    In a child process: torch must initialise HIP before the library does."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _TWO_STREAMS, root, os.path.join(root, "rust-raytrace_amd")],
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and "ordered ok" in out.stdout, out.stderr[-3000:]


_SERIALISED = r"""
import sys
sys.path[:0] = sys.argv[1:3]
import numpy as np
import libraytrace as lr
from libraytrace import scenes
from oracle import ref64
spec = scenes.config3(96, 64)
with lr.Context(0) as ctx:
    assert ctx.get_tuning("dev_join") == 0
    ctx.upload(lr.Scene.deserialize(spec.to_text()))
    rgb, bgr, st = ctx.render(lr.render_opts(96, 64, max_depth=spec.max_depth, spp=1))
assert np.array_equal(bgr, ref64.render(spec)["bgr"])
print("serialised ok")
"""


def test_device_join_off_under_kernel_serialisation():
    """Under rocprofv3 counter collection (ROCPROF_COUNTER_COLLECTION) the b
    streams cannot run beside a spinning join kernel: a context created there
    defaults dev_join to 0 (events), and renders stay exact."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ROCPROF_COUNTER_COLLECTION="1")
    out = subprocess.run([sys.executable, "-c", _SERIALISED, root, os.path.join(root, "rust-raytrace_amd")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0 and "serialised ok" in out.stdout, out.stderr[-3000:]


@pytest.mark.parametrize("engine", [-2, -1, 0])
def test_frame_rows_into_registered_frame(gpu_ctx, engine):
    """bench.py's multi-GPU frame: ordinary host memory page-locked with
    hipHostRegister, every "rank" of 4 writing its full-width 16-row bands (a
    ragged last band included) through the SDMA engines (copy_engine -2, the
    default for banded tiles, and -1) or hipMemcpyAsync (0): the whole-frame
    render bit for bit, with and without the sparse copies."""
    import ctypes as C
    W, H, band, n = 128, 136, 16, 4
    spec = scenes.config3(W, H)
    gpu_ctx.upload(lr.Scene.deserialize(spec.to_text()))
    whole = gpu_ctx.render(lr.render_opts(W, H, max_depth=spec.max_depth, spp=1))
    hip = _hip()
    rgb = np.full((H, W, 3), np.nan, np.float32)
    bgr = np.full((H, 3 * W), 0xAB, np.uint8)
    for a in (rgb, bgr):
        assert hip.hipHostRegister(C.c_void_p(a.ctypes.data), C.c_size_t(a.nbytes), 0) == 0
    try:
        for sparse in (1, 0):
            rgb[...] = np.nan
            bgr[...] = 0xAB
            with _with_tuning(gpu_ctx, sparse_out=sparse, copy_engine=engine):
                nbands = (H + band - 1) // band
                for r in range(n):
                    idx = list(range(r, nbands, n))
                    rows = sum(min(band, H - q * band) for q in idx)
                    o = lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, band=band, band_stride=n, band_phase=r,
                                       tile_h=rows, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS)
                    gpu_ctx.render(o, out=(rgb, bgr))
            assert np.array_equal(bgr, whole[1]), sparse
            assert np.array_equal(rgb.view(np.uint32), whole[0].view(np.uint32)), sparse
    finally:
        for a in (rgb, bgr):
            hip.hipHostUnregister(C.c_void_p(a.ctypes.data))
