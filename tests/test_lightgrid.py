"""Light-view grids (host_lightgrid.cpp) on the CPU: for every
point light and many shade points, each sphere whose exact f64 test blocks
the shadow ray (raytrace.rs:39-49: ray from p + 1e-5*l toward the light,
Some(t) with t*t < |L - p|^2; shapes.rs:50-89 quadratic in the device's
operation order) must be on the candidate list the grid hands the device for
that point (rt_light_grid_candidates mirrors the device lookup, f32 face
coordinates and early stop included).  Checked against the linear scan of
every sphere, the reference's own shadow query (scene.rs:247-249)."""
import numpy as np
import pytest

import libraytrace as lr
from libraytrace import scenes


def _spheres(spec):
    c, r, ids = [], [], []
    for i, o in enumerate(spec.objects):
        if o["shape"] == "sphere":
            c.append(o["center"]); r.append(o["radius"]); ids.append(i)
    return np.array(c, np.float64), np.array(r, np.float64), np.array(ids)


def _blockers(c, r, ids, L, p):
    """Object ids whose exact test shadows p from point light L (every sphere tested)."""
    v = L - p
    r2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2]          # location.sqdist(pt)
    ln = np.sqrt(r2)
    d = v / ln                                           # normalize
    o = p + d * 1e-5
    oc = o - c
    a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2]
    b = 2.0 * (d[0] * oc[:, 0] + d[1] * oc[:, 1] + d[2] * oc[:, 2])
    cc = (oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1] + oc[:, 2] * oc[:, 2]) - r * r
    disc = b * b - (4.0 * a) * cc
    with np.errstate(invalid="ignore"):
        s = np.sqrt(np.where(disc > 0.0, disc, 0.0))
        t1 = (-b - s) / (2.0 * a)
        t2 = (-b + s) / (2.0 * a)
    t = np.where(t1 > 0.0, t1, t2)
    hit = (disc > 0.0) & (t > 0.0) & (t * t < r2)
    return set(ids[hit].tolist())


def _shade_points(c, r, rng, n):
    """Points on sphere surfaces (where shadow queries start) and in the open."""
    k = rng.integers(0, len(c), n)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    on = c[k] + u * r[k][:, None]
    lo, hi = c.min(0) - 1.0, c.max(0) + 1.0
    free = lo + (hi - lo) * rng.random((n // 4, 3))
    return np.vstack([on, free])


def _check(spec, n_points=1500, seed=0, resolution=0):
    sc = lr.Scene.deserialize(spec.to_text())
    c, r, ids = _spheres(spec)
    rng = np.random.default_rng(seed)
    pts = _shade_points(c, r, rng, n_points)
    checked = 0
    for li, L in enumerate(spec.lights):
        if L["kind"] != "point":
            continue
        Lp = np.array(L["location"], np.float64)
        # also points right next to the light
        near = Lp + rng.normal(size=(50, 3)) * 1e-3
        allp = np.vstack([pts, near])
        cands, info = sc.light_grid_candidates(li, allp, resolution=resolution)
        assert info[0] > 0
        for p, cand in zip(allp, cands):
            if cand is None:            # the device tests every sphere
                continue
            missing = _blockers(c, r, ids, Lp, p) - set(cand.tolist())
            assert not missing, f"light {li} point {p.tolist()}: blockers {sorted(missing)} not listed"
            checked += 1
    return checked


def test_grid_lists_every_blocker_config3():
    assert _check(scenes.config3(64, 64)) > 2000


def test_grid_lists_every_blocker_adversarial_lights():
    """Lights inside the cloud, at a sphere's centre, on its surface, on a plane;
    spheres from 1e-3 to 1e3 (the scene of test_gpu_parity's grid test)."""
    s = scenes.SceneSpec(width=8, height=8, max_depth=2,
                         camera={"ctor": "new", "position": (0, 2, 12), "look": (0, -0.1, -1), "up": (0, 1, 0),
                                 "im_dist": 1.2})
    rng = scenes.SplitMix64(4242)
    for k in range(400):
        cen = (rng.uniform(-6, 6), rng.uniform(-2, 6), rng.uniform(-10, 2))
        kd = (rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9))
        s.sphere(cen, 10 ** rng.uniform(-3, -0.2), scenes.phong(kd, (0.3, 0.3, 0.3), 20.0, (0.01, 0.01, 0.01)))
    s.sphere((3.0, 1.0, -4.0), 0.8, scenes.phong((0.8, 0.8, 0.2), (0.4, 0.4, 0.4), 10.0, (0, 0, 0)))
    s.sphere((0.0, -1e3 - 2.5, -4.0), 1e3, scenes.phong((0.5, 0.5, 0.5), (0.2, 0.2, 0.2), 5.0, (0, 0, 0)))
    s.point_light((0.0, 2.0, -4.0), (0.6, 0.6, 0.6))
    s.point_light((3.0, 1.0, -4.0), (0.5, 0.2, 0.2))
    s.point_light((3.0, 1.8, -4.0), (0.2, 0.5, 0.2))
    s.point_light((-5.0, 0.5, -30.0), (0.2, 0.2, 0.5))
    assert _check(s, n_points=1200, seed=1) > 4000


def test_grid_lists_every_blocker_ten_thousand_spheres():
    assert _check(scenes.config4(32, 32), n_points=800, seed=2) > 1000


@pytest.mark.parametrize("R", [16, 40, 512])
def test_grid_resolution_does_not_matter(R):
    """Any forced resolution (tuning "light_grid_res") keeps every blocker listed."""
    assert _check(scenes.config3(32, 32), n_points=600, seed=3, resolution=R) > 500


def test_grid_sizes_config3():
    sc = lr.Scene.deserialize(scenes.config3(32, 32).to_text())
    _, info0 = sc.light_grid_candidates(0, np.zeros((0, 3)))
    _, info1 = sc.light_grid_candidates(1, np.zeros((0, 3)))
    print(f"C3 grids: light 0 R={info0[0]} cells={info0[1]}; light 1 R={info1[0]} cells={info1[1]}; "
          f"entries (both) {info0[2]}")
    assert 16 <= info0[0] <= 512 and 16 <= info1[0] <= 512


# ---- the camera's view grid (host_lightgrid.cpp build_view_grid) ----

def _camera_dirs(sc, W, H, rng, n):
    """Camera-ray directions exactly as camera_ray builds them (main.rs:50-53,
    camera.rs:78): random pixels with centre jitter, plus the frame's corners."""
    d = sc.desc()
    M = np.array(d.camera.matrix[:], np.float64).reshape(3, 3)
    hw, hh = W / 2.0, H / 2.0
    scale = max(1.0 / hw, 1.0 / hh)
    xs = np.concatenate([rng.integers(0, W, n), [0, W - 1, 0, W - 1]])
    ys = np.concatenate([rng.integers(0, H, n), [0, 0, H - 1, H - 1]])
    px = ((xs + 0.5) - hw) * scale
    py = ((ys + 0.5) - hh) * scale
    dx = M[0, 0] * px + M[0, 1] * py + M[0, 2] * 1.0
    dy = M[1, 0] * px + M[1, 1] * py + M[1, 2] * 1.0
    dz = M[2, 0] * px + M[2, 1] * py + M[2, 2] * 1.0
    l = np.sqrt(dx * dx + dy * dy + dz * dz)
    return np.stack([dx / l, dy / l, dz / l], 1), np.array(d.camera.position[:], np.float64)


def _hits(c, r, o, d):
    """Exact t of every sphere for one ray (shapes.rs:60-89 in the device's order), inf = miss."""
    oc = o - c
    a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2]
    b = 2.0 * (d[0] * oc[:, 0] + d[1] * oc[:, 1] + d[2] * oc[:, 2])
    cc = (oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1] + oc[:, 2] * oc[:, 2]) - r * r
    disc = b * b - (4.0 * a) * cc
    with np.errstate(invalid="ignore"):
        s = np.sqrt(np.where(disc > 0.0, disc, 0.0))
        t1 = (-b - s) / (2.0 * a)
        t2 = (-b + s) / (2.0 * a)
    t = np.where(t1 > 0.0, t1, t2)
    return np.where((disc > 0.0) & (t > 0.0), t, np.inf)


def _check_view(spec, n_rays=3000, seed=0, resolution=0):
    """Every sphere whose exact hit t is <= the ray's nearest t (the winner and any
    tie) is on the ray's list with a distance bound <= t, so the device's early
    stop (bound > t_limit(best t) >= best t) cannot skip it."""
    sc = lr.Scene.deserialize(spec.to_text())
    c, r, ids = _spheres(spec)
    rng = np.random.default_rng(seed)
    dirs, pos = _camera_dirs(sc, spec.width, spec.height, rng, n_rays)
    cands, info = sc.view_grid_candidates(dirs, resolution=resolution)
    assert info[0] > 0
    hits = 0
    for d, cand in zip(dirs, cands):
        if cand is None:                 # the device tests every sphere
            continue
        t = _hits(c, r, pos, d)
        best = t.min()
        if not np.isfinite(best):
            continue
        listed = dict(zip(cand[0].tolist(), cand[1].tolist()))
        for k in np.nonzero(t <= best)[0]:
            oid = int(ids[k])
            assert oid in listed, f"dir {d.tolist()}: sphere {oid} (t={t[k]}) not listed"
            assert listed[oid] <= t[k], (oid, listed[oid], t[k])
        hits += 1
    return hits, info


def test_view_grid_lists_every_winner_config3():
    n, info = _check_view(scenes.config3(4096, 4096))
    assert n > 500 and info[2] > 0
    print(f"C3 view grid: R={info[0]} cells={info[1]} entries={info[2]}")


def test_view_grid_dense_view_and_ten_thousand_spheres():
    assert _check_view(scenes.config3(512, 512, view="dense"), seed=1)[0] > 1000
    assert _check_view(scenes.config4(1024, 1024), n_rays=1500, seed=2)[0] > 300


@pytest.mark.parametrize("R", [1, 16, 333, 2048])
def test_view_grid_resolution_does_not_matter(R):
    assert _check_view(scenes.config3(256, 256), n_rays=1500, seed=3, resolution=R)[0] > 300


def test_view_grid_camera_inside_spheres():
    """The camera inside two nested spheres and on a third one's surface (always
    list), spheres from 1e-3 to 1e3, rays along the axes."""
    s = scenes.SceneSpec(width=33, height=33, max_depth=2,
                         camera={"ctor": "new", "position": (0.0, 0.0, 0.0), "look": (0.0, 0.0, -1.0),
                                 "up": (0.0, 1.0, 0.0), "im_dist": 1.0})
    m = scenes.phong((0.5, 0.5, 0.5), (0.2, 0.2, 0.2), 10.0, (0, 0, 0))
    s.sphere((0.0, 0.0, 0.0), 50.0, m)
    s.sphere((0.1, 0.0, 0.0), 2.0, m)
    s.sphere((0.0, 0.0, -3.0), 3.0, m)
    rng = scenes.SplitMix64(77)
    for k in range(300):
        s.sphere((rng.uniform(-20, 20), rng.uniform(-20, 20), rng.uniform(-40, 5)), 10 ** rng.uniform(-3, 0.5), m)
    s.sphere((0.0, -1e3 - 5.0, 0.0), 1e3, m)
    assert _check_view(s, n_rays=2000, seed=4)[0] > 1000
