"""Where rt_render's device -> host time goes at C3 (BGR only, 50 MB): the raw
DMA rate into page-locked memory, host memcpy rates, and rt_render end to end
against the same frame rendered into device buffers.

    python tools/pcie_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]


def best(f, n=5):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t0) * 1e3)
    return min(ts)


def main():
    import numpy as np
    import torch
    import libraytrace as lr
    from libraytrace import scenes
    dev = torch.device("cuda", 0)
    nbytes = 4096 * 4096 * 3
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    pin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    page = np.zeros(nbytes, np.uint8)
    torch.cuda.synchronize()

    def dma():
        pin.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
    ms = best(dma)
    print(f"DMA device -> pinned, 50 MB: {ms:.3f} ms = {nbytes / ms / 1e6:.1f} GB/s")
    pn = pin.numpy()
    ms = best(lambda: np.copyto(page, pn))
    print(f"host memcpy pinned -> pageable, one thread: {ms:.3f} ms = {nbytes / ms / 1e6:.1f} GB/s")

    spec = scenes.config3()
    ctx = lr.Context(0, tuning="env")
    ctx.upload(lr.Scene.deserialize(spec.to_text()))
    o = lr.render_opts(4096, 4096, max_depth=8, spp=1)
    hb = np.zeros((4096, 3 * 4096), np.uint8)
    out_rgb = torch.empty((4096, 4096, 3), dtype=torch.float32, device=dev)
    out_bgr = torch.empty((4096, 3 * 4096), dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)

    def dev_only():
        ctx.render_device(o, out_rgb.data_ptr(), out_bgr.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
    for _ in range(3):
        dev_only()
    print(f"render into device buffers (+ sync): {best(dev_only):.3f} ms")
    ctx.render(o, rgb=False, out=(None, hb))
    print(f"rt_render, BGR to pageable host memory: {best(lambda: ctx.render(o, out=(None, hb), stats=False)):.3f} ms")
    print(f"  ... with rt_stats read back: {best(lambda: ctx.render(o, out=(None, hb))):.3f} ms")
    hp = torch.empty((4096, 3 * 4096), dtype=torch.uint8, pin_memory=True)
    hpn = hp.numpy()
    ctx.render(o, out=(None, hpn))
    print(f"rt_render, BGR to page-locked host memory: {best(lambda: ctx.render(o, out=(None, hpn), stats=False)):.3f} ms")
    # the bench's context history before its PCIe-inclusive measurement
    pg = lambda oo: best(lambda: ctx.render(oo, out=(None, hb), stats=False), 3)
    ob = lr.render_opts(4096, 4096, max_depth=8, spp=1, tile_h=4096, band=16, band_stride=1, band_phase=0)
    print(f"  band=16 opts: {pg(ob):.3f} ms")
    ot = lr.render_opts(4096, 4096, max_depth=8, spp=1, flags=o.flags | lr.RT_TIME_KERNELS)
    for _ in range(3):
        ctx.render_device(ot, out_rgb.data_ptr(), out_bgr.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    ctx.kernel_times()
    print(f"  after RT_TIME_KERNELS renders: {pg(o):.3f} ms")
    oc = lr.render_opts(4096, 4096, max_depth=8, spp=1, flags=o.flags | lr.RT_COUNT_WORK)
    ctx.render_device(oc, out_rgb.data_ptr(), out_bgr.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    ctx.stats()
    print(f"  after an RT_COUNT_WORK render: {pg(o):.3f} ms")
    hb2 = np.zeros((4096, 3 * 4096), np.uint8)
    print(f"  fresh pageable buffer (first touch inside): {pg(o):.3f} ms")
    ctx.close()


if __name__ == "__main__":
    main()
