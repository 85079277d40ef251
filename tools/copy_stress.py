"""Repeat rt_render into host frames many times and report every byte that
differs from a reference render: the page-locked and pageable destinations,
plain / sparse copies, hipMemcpyAsync and the SDMA engines,
row-band tiles and partial-width tiles (tests/test_gpu_parity.py's frame-row
cases, looped).  Diagnostic for ordering races between the frame copy, the
packed segments and the host scatter.

    python3 tools/copy_stress.py [repeats]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]

import numpy as np  # noqa: E402

import libraytrace as lr  # noqa: E402
from libraytrace import scenes  # noqa: E402


def pinned(shape, dtype, hip):
    p = C.c_void_p()
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    assert hip.hipHostMalloc(C.byref(p), C.c_size_t(n), 0) == 0
    return np.ctypeslib.as_array((C.c_uint8 * n).from_address(p.value)).view(dtype).reshape(shape), p


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    hip = C.CDLL("libamdhip64.so.7")
    W, H = 150, 100
    pitch = (3 * W + 3) & ~3
    spec = scenes.config3(W, H)
    ctx = lr.Context(0)
    ctx.upload(lr.Scene.deserialize(spec.to_text()))
    whole = ctx.render(lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, bgr_pitch=pitch))
    fr = lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS
    cases = {
        "right_edge_bgr": dict(x0=50, tile_w=W - 50, y0=0, tile_h=8, flags=lr.RT_OUT_BGR_U8 | lr.RT_OUT_FRAME_ROWS),
        "partial": dict(x0=40, tile_w=100, y0=20, tile_h=40, flags=fr),
        "bands3": dict(band=16, band_stride=3, band_phase=1, tile_h=32, flags=fr),
        "full": dict(flags=fr),
    }
    bad = 0
    for tune in [dict(sparse_out=1, copy_engine=0), dict(sparse_out=1, copy_engine=-1), dict(sparse_out=0, copy_engine=0),
                 dict(sparse_out=0, copy_engine=-1)]:
        for k, v in tune.items():
            ctx.set_tuning(k, v)
        for pin in (True, False):
            if pin:
                rgb, prgb = pinned((H, W, 3), np.float32, hip)
                bgr, pbgr = pinned((H, pitch), np.uint8, hip)
            else:
                rgb, bgr = np.zeros((H, W, 3), np.float32), np.zeros((H, pitch), np.uint8)
            for name, kw in cases.items():
                o = lr.render_opts(W, H, max_depth=spec.max_depth, spp=1, bgr_pitch=pitch, **kw)
                rows = [o.y0 + ((j // o.band) * o.band_stride + o.band_phase) * o.band + j % o.band for j in range(o.tile_h)]
                xs = slice(3 * o.x0, 3 * (o.x0 + o.tile_w) + (pitch - 3 * W if o.x0 + o.tile_w == W else 0))
                for i in range(reps):
                    bgr[...] = 0xAB
                    rgb[...] = np.nan
                    ctx.render(o, out=(rgb if o.flags & lr.RT_OUT_RGB_F32 else None, bgr), stats=False)
                    got, want = bgr[rows, xs], whole[1][rows, xs]
                    if not np.array_equal(got, want):
                        bad += 1
                        d = np.argwhere(got != want)
                        print(f"BGR {tune} pinned={pin} {name} rep {i}: {len(d)} bytes differ, first at row/col "
                              f"{d[:4].tolist()}, got {got[tuple(d[0])]} want {want[tuple(d[0])]}", flush=True)
                    if o.flags & lr.RT_OUT_RGB_F32:
                        g = rgb[rows, o.x0:o.x0 + o.tile_w].view(np.uint32)
                        w_ = whole[0][rows, o.x0:o.x0 + o.tile_w].view(np.uint32)
                        if not np.array_equal(g, w_):
                            bad += 1
                            d = np.argwhere(g != w_)
                            print(f"RGB {tune} pinned={pin} {name} rep {i}: {len(d)} words differ, first {d[:4].tolist()}",
                                  flush=True)
            if pin:
                del rgb, bgr
                hip.hipHostFree(prgb)
                hip.hipHostFree(pbgr)
        print(f"done {tune}: {bad} bad so far", flush=True)
    ctx.close()
    print(f"total bad renders: {bad}")


if __name__ == "__main__":
    main()
