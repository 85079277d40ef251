"""BASELINE configs C3/C4/C5 at their FULL sizes on the production schedule,
checked against the oracle on sampled rows (the oracle's linear scan over 10k /
100k spheres cannot render whole frames in test time).

Per config:
  * one full-frame render through the C ABI with the default schedule (C4: one
    67 M-pixel chunk; C5: the default multi-chunk schedule, chunks starting at
    row0 > 0, 268 M pixels, so the large-offset indexing of queues, levels and
    the BGR pitch x 16384 rows is exercised);
  * sampled rows of that frame: BGR bit-exact, f32 within 1e-5 relative;
  * the same rows rendered alone on the device: identical bytes (schedule
    independence) and Scene::intersect counts equal to the oracle's.
C3 is additionally rendered as one rank's share of an 8-GPU frame (16-row
bands, band_stride 8, band_phase 7 -- bench.py's layout): the whole shard
against the oracle.  References: main.rs:45-57 (pixels independent),
scene.rs:247-249, raytrace.rs:30-67.
"""
import os

import numpy as np
import pytest

import libraytrace as lr
from libraytrace import scenes
from oracle import ref64
from test_gpu_parity import check_close

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def _upload(ctx, spec):
    ctx.upload(lr.Scene.deserialize(spec.to_text()))


def _opts(spec, **kw):
    return lr.render_opts(spec.width, spec.height, max_depth=spec.max_depth, spp=1, **kw)


def _check_rows(ctx, spec, rgb, bgr, rows, x0, tw):
    """rows of the full frame (rgb/bgr indexed by frame row) against the oracle,
    and against the same rows rendered alone on the device (counts too)."""
    for y in rows:
        ref = ref64.render(spec, x0=x0, tile_w=tw, y0=y, tile_h=1, threads=THREADS)
        got_b = bgr[y, 3 * x0:3 * (x0 + tw)]
        assert np.array_equal(got_b, ref["bgr"][0]), f"row {y}: {(got_b != ref['bgr'][0]).sum()} BGR bytes differ"
        check_close(rgb[y, x0:x0 + tw][None], ref["rgb64"])
        r1, b1, st = ctx.render(_opts(spec, x0=x0, tile_w=tw, y0=y, tile_h=1))
        assert np.array_equal(b1[0], got_b), f"row {y} rendered alone differs from the full frame"
        assert np.array_equal(r1[0].view(np.uint32), rgb[y, x0:x0 + tw].view(np.uint32))
        assert st.rays == ref["counts"]["rays"] and st.shadow_rays == ref["counts"]["shadow_rays"], (y, st.rays)


def test_config4_full_size(gpu_ctx):
    """C4: 8192^2, 10k spheres, depth 8, one 67 M-pixel chunk.  Every 512th row,
    full width (16 x 8192 px)."""
    spec = scenes.config4()
    _upload(gpu_ctx, spec)
    rgb, bgr, st = gpu_ctx.render(_opts(spec))
    assert st.pixels == 8192 * 8192
    rows = np.arange(16) * 512
    ref = ref64.render(spec, y0=0, tile_h=16, band=1, band_stride=512, band_phase=0, threads=THREADS)
    assert np.array_equal(bgr[rows], ref["bgr"]), f"{(bgr[rows] != ref['bgr']).sum()} BGR bytes differ"
    check_close(rgb[rows], ref["rgb64"])
    # the same 16 rows as one banded tile on the device: bytes and counts
    r2, b2, st2 = gpu_ctx.render(_opts(spec, tile_h=16, band=1, band_stride=512))
    assert np.array_equal(b2, bgr[rows])
    assert st2.rays == ref["counts"]["rays"] and st2.shadow_rays == ref["counts"]["shadow_rays"]
    assert np.isfinite(rgb).all() and st.rays >= st.pixels


def test_config5_full_size(gpu_ctx):
    """C5: 16384^2, 100k spheres, depth 16, the default multi-chunk schedule.
    Two rows in different chunks over a 2048-column window, and the top row
    (largest offsets) over 256 columns."""
    spec = scenes.config5()
    _upload(gpu_ctx, spec)
    rgb, bgr, st = gpu_ctx.render(_opts(spec))
    assert st.pixels == 16384 * 16384
    assert bgr.shape == (16384, 3 * 16384)
    _check_rows(gpu_ctx, spec, rgb, bgr, [3001, 9999], 7168, 2048)
    _check_rows(gpu_ctx, spec, rgb, bgr, [16383], 8064, 256)
    assert np.isfinite(rgb).all() and st.rays >= st.pixels


def test_config3_eight_rank_shard(gpu_ctx):
    """C3 as rank 7 of an 8-GPU frame (bench.py's 16-row bands dealt round-robin):
    the whole 512-row shard against the oracle, bytes, colours and counts."""
    spec = scenes.config3()
    _upload(gpu_ctx, spec)
    lay = dict(y0=0, tile_h=512, band=16, band_stride=8, band_phase=7)
    rgb, bgr, st = gpu_ctx.render(_opts(spec, **lay))
    ref = ref64.render(spec, threads=THREADS, **lay)
    assert np.array_equal(bgr, ref["bgr"]), f"{(bgr != ref['bgr']).sum()} BGR bytes differ"
    check_close(rgb, ref["rgb64"])
    assert st.rays == ref["counts"]["rays"] and st.shadow_rays == ref["counts"]["shadow_rays"]
