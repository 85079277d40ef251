"""Diagnostic for test_extreme_light_and_plane_magnitudes: which pixels differ
from the oracle, by how much, per algorithm and per tuning."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]
import numpy as np

import libraytrace as lr
from libraytrace import scenes
from oracle import ref64


def scene(variant):
    s = scenes.random_spheres(60, 64, 48, 6, seed=33, plane=False)
    s.lights = []
    if "dirsmall" in variant:
        s.directional_light((3e-36, -1e-35, -2e-36), (0.5, 0.5, 0.4))
    if "dirbig" in variant:
        s.directional_light((2e33, -1e34, 1e33), (0.0, 0.0, 0.0))
    s.point_light((0.0, 8.0, 2.0), (0.6, 0.6, 0.6))
    if "planebig" in variant:
        s.plane((0.0, -0.5, 0.0), (0.0, 1e25, 0.0), scenes.phong((0.2, 0.2, 0.2), (0.6, 0.6, 0.6), 10.0, (0.01, 0.01, 0.01)))
    if "planesmall" in variant:
        s.plane((0.0, 0.0, -40.0), (0.0, 3e-21, 1e-20), scenes.phong((0.3, 0.2, 0.1), (0.5, 0.5, 0.5), 10.0, (0.0, 0.0, 0.0)))
    return s


with lr.Context(0) as ctx:
    for variant in ["dirsmall", "dirbig", "planebig", "planesmall", "dirsmall+dirbig+planebig+planesmall"]:
        s = scene(variant)
        ref = ref64.render(s)
        ctx.upload(lr.Scene.deserialize(s.to_text()))
        for algo in (lr.RT_ALGO_WAVEFRONT, lr.RT_ALGO_WAVEFRONT_BRUTE, lr.RT_ALGO_BRUTE_LDS):
            rgb, bgr, st = ctx.render(lr.render_opts(s.width, s.height, max_depth=s.max_depth, spp=1, algo=algo))
            r64 = ref["rgb64"]
            g = rgb.astype(np.float64)
            bad = ~((np.isnan(r64) & np.isnan(g)) | (np.abs(g - r64) <= 1e-5 * np.abs(r64)))
            nb = int((bgr != ref["bgr"]).sum())
            print(f"{variant:40s} algo {algo}: bgr diff {nb}, rgb bad {int(bad.sum())}, rays {st.rays} vs {ref['counts']['rays']}, "
                  f"shadow {st.shadow_rays} vs {ref['counts']['shadow_rays']}")
            if bad.any():
                idx = np.argwhere(bad)[:4]
                for i in idx:
                    y, x, c = i
                    print(f"    px ({x},{y}) c{c}: gpu {g[y, x, c]!r} ref {r64[y, x, c]!r}")
