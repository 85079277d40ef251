"""Where wf_nearest's time goes: in-kernel s_memtime stamps of an RT_STAMP=1
build (diagnostic only; make BUILD=build_st LIB=librtamd_st.so EXTRA=-DRT_STAMP=1).

    RT_LIBRTAMD=rust-raytrace_amd/librtamd_st.so python tools/stamp_probe.py [--config c3|c4] [--tune k=v,...]

Per generation: wave-cycles per 64-ray chunk by phase (ray load + region entry,
traversal, finish) and per wave for the setup (region scan + LDS staging),
then from a counting render the slowest lane's node visits per chunk against
the mean lane's (the divergence factor of the traversal loop).
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c3", "c4"])
    ap.add_argument("--tune", default="")
    ap.add_argument("--shard-of", type=int, default=1, help="render the last rank's 16-row bands of an N-way shard")
    a = ap.parse_args()
    import torch
    import libraytrace as lr
    from libraytrace import scenes
    lib = lr.lib
    lib.rt_debug_stamps.restype = C.c_int
    lib.rt_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    G, F = 34, 16
    buf = (C.c_ulonglong * (G * F))()

    def read(reset):
        assert lib.rt_debug_stamps(buf, G * F, 1 if reset else 0) == 0
        return [[buf[g * F + f] for f in range(F)] for g in range(G)]

    n, side, seed, scale = (1000, 4096, 3, 1.0) if a.config == "c3" else (10000, 8192, 4, 10.0 ** (1 / 3))
    spec = scenes.random_spheres(n, side, side, 8, seed=seed, box_scale=scale, name=a.config)
    tune = {k: int(v) for k, v in (x.split("=") for x in a.tune.split(",") if x)}
    ctx = lr.Context(0, tuning=tune)
    ctx.upload(lr.Scene.deserialize(spec.to_text()))
    dev = torch.device("cuda", 0)
    rgb = torch.empty((side, side, 3), dtype=torch.float32, device=dev)
    bgr = torch.empty((side, 3 * side), dtype=torch.uint8, device=dev)
    N = a.shard_of
    shard = dict(tile_h=side // N, band=16, band_stride=N, band_phase=N - 1) if N > 1 else {}
    opts = lr.render_opts(side, side, max_depth=8, spp=1, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8, **shard)
    cnt = lr.render_opts(side, side, max_depth=8, spp=1, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_COUNT_WORK,
                         **shard)
    s = torch.cuda.Stream(dev)
    for _ in range(2):
        ctx.render_device(opts, rgb.data_ptr(), bgr.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    read(True)
    ctx.render_device(opts, rgb.data_ptr(), bgr.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    plain = read(True)
    ctx.render_device(cnt, rgb.data_ptr(), bgr.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    counted = read(True)
    print(f"{a.config} {tune or ''}: cycles per chunk (64 rays) by phase; setup per wave; node visits per chunk")
    print(" gen  chunks   waves  setup/wave  load/chunk  trav/chunk  fin/chunk   maxlane  meanlane  div   desc/ch   leaf/ch    pop/ch"
          "  slowest-wave  wave-iters/ch desc leaf pop  cycles/iter desc leaf pop")
    for g in range(G):
        st, ld, tr, fi, ch, wv, _, _, de, le, po, _, slow, nd, nl, np_ = plain[g]
        mx, sm = counted[g][6], counted[g][7]
        if ch == 0:
            continue
        cc = counted[g][4] or 1
        print(f"{g:4d} {ch:7d} {wv:7d} {st / max(wv, 1):11.0f} {ld / ch:11.0f} {tr / ch:11.0f} {fi / ch:10.0f} "
              f"{mx / cc:9.1f} {sm / cc / 64:9.1f} {mx / max(sm / 64, 1):5.2f} {de / ch:9.0f} {le / ch:9.0f} {po / ch:9.0f}"
              f" {slow:13d}  {nd / ch:6.1f} {nl / ch:5.1f} {np_ / ch:5.1f}  {de / max(nd, 1):6.0f} {le / max(nl, 1):5.0f} {po / max(np_, 1):5.0f}")
    ctx.close()


if __name__ == "__main__":
    main()
