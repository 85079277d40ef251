"""Where the first render of a process goes (DESIGN.md §6 first_frame_ms): the C3
frame rendered by a fresh context, phase by phase, each synchronised and timed
on the host: rt_ctx_create, rt_scene_upload, rt_ctx_reserve, then three renders.
Run under rocprofv3 --kernel-trace --hip-runtime-trace to see which launches or
API calls the first render pays for.

    python3 tools/cold_probe.py [--no-reserve] [--config c3|c4] [--host]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-reserve", action="store_true")
    ap.add_argument("--host", action="store_true", help="rt_render into pageable host buffers instead of device ones")
    ap.add_argument("--config", default="c3", choices=["c3", "c4"])
    ap.add_argument("--tiny", action="store_true", help="render an 8-row tile first (every kernel launched once)")
    ap.add_argument("--api", action="store_true", help="host cost per render: enqueue time against wall time")
    a = ap.parse_args()
    import numpy as np
    import torch
    import libraytrace as lr
    from libraytrace import scenes
    side, n, box = (4096, 1000, 1.0) if a.config == "c3" else (8192, 10000, 10.0 ** (1 / 3))
    spec = scenes.random_spheres(n, side, side, 8, seed=3 if a.config == "c3" else 4, box_scale=box, name=a.config)
    text = spec.to_text()
    dev = torch.device("cuda", 0)
    torch.cuda.synchronize(dev)
    out = {}
    t = time.perf_counter()
    ctx = lr.Context(0)
    out["ctx_create"] = time.perf_counter() - t
    scene = lr.Scene.deserialize(text)
    t = time.perf_counter()
    ctx.upload(scene)
    out["upload"] = time.perf_counter() - t
    o = lr.render_opts(side, side, max_depth=8, spp=1)
    rgb = torch.empty((side, side, 3), dtype=torch.float32, device=dev)
    bgr = torch.empty((side, 3 * side), dtype=torch.uint8, device=dev)
    hr = np.zeros((side, side, 3), np.float32)
    hb = np.zeros((side, 3 * side), np.uint8)
    s = torch.cuda.Stream(dev)
    if not a.no_reserve:
        t = time.perf_counter()
        ctx.reserve(o, host=a.host, stream_ptr=s.cuda_stream)
        out["reserve"] = time.perf_counter() - t
    if a.tiny:                 # every kernel's first launch, on a one-row tile, before the timed renders
        t = time.perf_counter()
        ctx.render_device(lr.render_opts(side, side, max_depth=8, spp=1, y0=side // 2, tile_h=8), rgb.data_ptr(),
                          bgr.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        out["tiny"] = time.perf_counter() - t
    for i in range(3):
        t = time.perf_counter()
        if a.host:
            ctx.render(o, out=(hr, hb), stats=False)
        else:
            ctx.render_device(o, rgb.data_ptr(), bgr.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
        out[f"render{i}"] = time.perf_counter() - t
    print(" ".join(f"{k} {v * 1e3:.3f} ms" for k, v in out.items()), flush=True)
    if a.api:
        # host cost per frame: enqueueing K renders back to back (no wait) against their GPU time,
        # and the HIP calls a render makes that may reach the kernel driver
        import ctypes as C
        hip = C.CDLL("libamdhip64.so.7")
        fr, tot = C.c_size_t(), C.c_size_t()
        t = time.perf_counter()
        for _ in range(1000):
            hip.hipMemGetInfo(C.byref(fr), C.byref(tot))
        print(f"hipMemGetInfo {(time.perf_counter() - t) * 1e3:.3f} us per call", flush=True)
        for shard in (1, 8):
            ob = lr.render_opts(side, side, max_depth=8, spp=1, band=16, band_stride=shard, band_phase=0,
                                tile_h=side // shard)
            for _ in range(3):
                ctx.render_device(ob, rgb.data_ptr(), bgr.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
            K = 50
            t = time.perf_counter()
            for _ in range(K):
                ctx.render_device(ob, rgb.data_ptr(), bgr.data_ptr(), s.cuda_stream)
            te = time.perf_counter() - t
            torch.cuda.synchronize(dev)
            tt = time.perf_counter() - t
            print(f"share 1/{shard}: enqueue {te / K * 1e3:.3f} ms per render, wall {tt / K * 1e3:.3f} ms per render",
                  flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
