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
