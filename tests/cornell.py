"""test_scene.txt's Cornell box (the reference's only rendered scene, out.bmp)
and the statistical check against out.bmp shared by the oracle and device tests."""
import json
import os

import numpy as np

from libraytrace import scenes

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def cornell_spec(width=200, height=200, antialias=1024, max_depth=4):
    """test_scene.txt (IndirectPhong walls, spheres and a lamp, no lights) at 200x200:
    each pixel spans a 4x4 block of out.bmp's 800x800."""
    return scenes.config1(width, height, antialias, max_depth)


def check_out_bmp_statistics(bgr):
    """8x8 block means of a 200x200 render's sRGB bytes against out.bmp's."""
    st = json.load(open(os.path.join(GOLD, "out_bmp_stats.json")))
    img = np.asarray(bgr).reshape(200, 200, 3).astype(np.float64)
    grid = img.reshape(8, 25, 8, 25, 3).mean(axis=(1, 3))
    gold = np.array(st["grid"])
    err = grid - gold
    assert np.abs(err).max() < 4.5, np.abs(err).max()
    assert np.sqrt((err ** 2).mean()) < 1.2, np.sqrt((err ** 2).mean())
    assert np.abs(grid.mean(axis=(0, 1)) - np.array(st["mean_bgr"])).max() < 1.0
    # red wall on the left, green on the right (camera handedness, camera.rs:52)
    assert grid[:, 0, 2].mean() > grid[:, 0, 1].mean() + 20
    assert grid[:, 7, 1].mean() > grid[:, 7, 2].mean() + 20
    return float(np.sqrt((err ** 2).mean())), float(np.abs(err).max())
