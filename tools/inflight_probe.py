"""Do two contexts' renders overlap on the device?  Issues N renders of one
rank's share of an 8-way C3 frame alternately on F contexts (own streams) and
prints, per call, the host time spent inside rt_render_device (a call that
blocks the host serialises the frames whatever the streams) and, afterwards,
each render's device start / end from HIP events on its stream.
    python3 tools/inflight_probe.py [--contexts F] [--renders N] [--tune k=v,...]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contexts", type=int, default=2)
    ap.add_argument("--renders", type=int, default=8)
    ap.add_argument("--shard-of", type=int, default=8)
    ap.add_argument("--tune", default="")
    a = ap.parse_args()
    import torch
    import libraytrace as lr
    from libraytrace import scenes, shard
    tune = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.tune.split(",") if kv)
    spec = scenes.config3()
    sc = lr.Scene.deserialize(spec.to_text())
    W, H = spec.width, spec.height
    rows = shard.local_rows(H, 16, a.shard_of, 0)
    o = lr.render_opts(W, H, tile_h=len(rows), band=16, band_stride=a.shard_of, band_phase=0, max_depth=8, spp=1,
                       flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8)
    dev = torch.device("cuda", 0)
    ctxs = [lr.Context(0, tuning=tune) for _ in range(a.contexts)]
    for c in ctxs:
        c.upload(sc)
    outs = [(torch.empty((len(rows), W, 3), dtype=torch.float32, device=dev),
             torch.empty((len(rows), 3 * W), dtype=torch.uint8, device=dev)) for _ in ctxs]
    streams = [torch.cuda.Stream(dev) for _ in ctxs]
    for i in range(2 * a.contexts):                       # warm-up: working sets, streams
        f = i % a.contexts
        ctxs[f].render_device(o, outs[f][0].data_ptr(), outs[f][1].data_ptr(), streams[f].cuda_stream)
    torch.cuda.synchronize(dev)
    evs, host = [], []
    t_all = time.perf_counter()
    for i in range(a.renders):
        f = i % a.contexts
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[f])
        t0 = time.perf_counter()
        ctxs[f].render_device(o, outs[f][0].data_ptr(), outs[f][1].data_ptr(), streams[f].cuda_stream)
        host.append((time.perf_counter() - t0) * 1e3)
        e1.record(streams[f])
        evs.append((f, e0, e1))
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t_all) * 1e3
    base = evs[0][1]
    for i, ((f, e0, e1), h) in enumerate(zip(evs, host)):
        print(f"render {i} ctx {f}: host call {h:7.3f} ms   device start {base.elapsed_time(e0):8.3f}  "
              f"end {base.elapsed_time(e1):8.3f} ms")
    print(f"wall {wall:.3f} ms for {a.renders} renders = {wall / a.renders:.3f} ms each")
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
