"""Headline benchmark: Mrays/s at 4096x4096, 1000 spheres, depth 8 (BASELINE.json).

One step = one full pass of the hot path over one frame of the headline
workload (config C3): every pixel's camera ray, its Phong
shading with shadow rays to 2 point lights, and mirror bounces to depth 8,
f64 arithmetic, f32 RGB + sRGB BGR written to HBM.  The scene is uploaded once
(inputs resident in HBM before timing); output stays in HBM (the PCIe copy is
reported separately in DESIGN.md, never in `value`).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

Multi-GPU: the frame's rows are dealt in 16-row bands round-robin over ranks
(libraytrace/shard.py); no collective touches the data path (RCCL carries the
barrier and the max-over-ranks timing only).  Default "scaling": "weak": at N
GPUs the same scene and view are rendered at sqrt(N) x the resolution (frame
side 4096*sqrt(N), rounded to whole bands), so every GPU renders the N=1
frame's 16.7 M pixels; --scaling strong splits the 4096^2 frame instead.
value = rays of the whole frame x K / max-over-ranks wall time of the K timed
steps.  --config c4 / c5 select the larger configs of BASELINE.json; --config
c1 the reference's own scene (test_scene.txt: IndirectPhong Cornell box, 1024
random AA samples, 256x256, depth 1) on the path kernel.

Rays = every Scene::intersect query the reference would issue (camera +
reflection + shadow), counted by the kernel; identical to the oracle's count
(tests/test_gpu_parity.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VALU_PEAK_TFLOPS = 78.6   # spec, FMA counted; the kernel issues no FMA (parity), so ~39.3 is its ceiling
BAND = 16


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="c3", choices=["c1", "c3", "c4", "c5"],
                   help="c3 4096^2/1000 spheres/depth 8 (headline); c4 8192^2/10k/8; c5 16384^2/100k/16; "
                        "c1 test_scene.txt 256^2, 1024 random AA samples, depth 1 (path kernel)")
    p.add_argument("--spp", type=int, default=0, help="c1: AA samples (default: the scene's 1024)")
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--spheres", type=int, default=0)
    p.add_argument("--depth", type=int, default=-1)
    p.add_argument("--algo", default="auto", choices=["auto", "wavefront", "lds", "global"])
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU time of the cpu_baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="N > 1: weak = the frame side grows by sqrt(N) (same scene and view, every GPU "
                        "renders the N=1 pixel count); strong = the N=1 frame split N ways")
    p.add_argument("--shard-of", type=int, default=0,
                   help="(diagnostic, one process) render only rank 0's row bands of an N-rank frame; "
                        "its time is what each rank of an N-GPU run spends")
    p.add_argument("--no-kernel-times", action="store_true",
                   help="skip the instrumented frames that time every launch with HIP events")
    p.add_argument("--inflight", type=int, default=1,
                   help="frames in flight: F contexts (each its own working set and streams) render successive "
                        "steps into F output buffers, so frame i+1's first generations overlap frame i's tail")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="N > 1: process-group backend for the barrier and the max-over-ranks timing (nccl = RCCL; "
                        "gloo rehearses N ranks on fewer GPUs, ranks sharing a device round-robin)")
    return p.parse_args()


def pmc_traffic(config_key):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        e = d.get(config_key)
        return float(e["hbm_bytes_per_launch"]) if e else None
    except Exception:
        return None


def cpu_baseline(spec, args, **draws):
    """Oracle (algorithmically the reference: same recursion, same linear scan,
    f64) on the host, on a deterministic row sample of the same frame.
    draws: jitter / seed / rng of a stochastic workload (the device's keyed draws)."""
    from oracle import ref64
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    rows, stride = 8, max(1, spec.height // 8)
    for _ in range(5):
        # every stride-th row of the frame (a deterministic sample of the same workload),
        # grown until the sample takes about cpu_seconds or covers the whole frame
        rows = spec.height // stride
        t0 = time.time()
        r = ref64.render(spec, tile_h=rows, band=1, band_stride=stride, band_phase=0, threads=threads,
                         want_rgb64=False, **draws)
        dt = time.time() - t0
        if dt >= 0.6 * args.cpu_seconds or stride == 1:
            break
        want = rows * args.cpu_seconds / max(dt, 1e-3)
        stride = max(1, min(stride - 1, int(spec.height / want)))
    return {"value": r["counts"]["rays"] / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{rows} rows (every {stride}th) x {spec.width} px of the same frame; "
                      f"{r['counts']['rays']} rays in {dt:.2f} s; oracle/ref64.c, f64, {threads} threads"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import libraytrace as lr
    from libraytrace import scenes, shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    band_world = args.shard_of if (args.shard_of > 1 and world == 1) else world
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":
        local %= max(1, torch.cuda.device_count())      # rehearsal: several ranks per device
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)

    cfg = {"c1": (256, 0, 1, 1, 1.0), "c3": (4096, 1000, 8, 3, 1.0), "c4": (8192, 10000, 8, 4, 10.0 ** (1 / 3)),
           "c5": (16384, 100000, 16, 5, 100.0 ** (1 / 3))}[args.config]       # scenes.config1/3/4/5
    path_cfg = args.config == "c1"
    args.width = args.width or cfg[0]
    args.height = args.height or cfg[0]
    n_split = args.shard_of if (args.shard_of > 1 and world == 1) else world
    if n_split > 1 and args.scaling == "weak":
        # weak scaling: the same view at sqrt(N) x the resolution, so each of the N ranks renders
        # (up to rounding to whole bands) the N=1 frame's pixel count
        f = n_split ** 0.5
        args.width = max(BAND, int(round(args.width * f / BAND)) * BAND)
        args.height = max(BAND, int(round(args.height * f / BAND)) * BAND)
    args.spheres = args.spheres or cfg[1]
    args.depth = cfg[2] if args.depth < 0 else args.depth
    if path_cfg:
        spec = scenes.config1(args.width, args.height, max_depth=args.depth)
        if args.spp:
            spec.antialias = args.spp
    else:
        spec = scenes.random_spheres(args.spheres, args.width, args.height, args.depth, seed=cfg[3],
                                     box_scale=cfg[4], name=args.config)
    spp = spec.antialias
    jitter = lr.RT_JITTER_RANDOM if path_cfg else lr.RT_JITTER_CENTER
    W, H = spec.width, spec.height
    scene = lr.Scene.deserialize(spec.to_text())
    F = max(1, args.inflight)
    ctxs = [lr.Context(local) for _ in range(F)]
    for c in ctxs:
        c.upload(scene)
    ctx = ctxs[0]
    rows = shard.local_rows(H, BAND, band_world, rank)
    tail = shard.tail_rows(H, BAND) if shard.tail_owner(H, BAND, band_world) == rank else None
    assert tail is None or len(tail) == 0, "bench frames are whole bands"
    algo = {"auto": lr.RT_ALGO_AUTO, "wavefront": lr.RT_ALGO_WAVEFRONT, "lds": lr.RT_ALGO_BRUTE_LDS,
            "global": lr.RT_ALGO_BRUTE_GLOBAL}[args.algo]
    common = dict(tile_h=len(rows), band=BAND, band_stride=band_world, band_phase=rank, max_depth=args.depth,
                  spp=spp, algo=algo, jitter=jitter, seed=cfg[3])
    opts = lr.render_opts(W, H, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8, **common)
    pitch = 3 * W
    outs = [(torch.empty((len(rows), W, 3), dtype=torch.float32, device=dev),
             torch.empty((len(rows), pitch), dtype=torch.uint8, device=dev)) for _ in range(F)]
    out_rgb, out_bgr = outs[0]
    # a real (non-null) stream: the library launches on exactly this stream, so the
    # torch events below bracket the kernel (handle 0 would select the context's own stream)
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    stream = streams[0]

    # per-kernel-family launch durations come from K more frames that record HIP
    # events around every launch (RT_TIME_KERNELS), after the timed region: the
    # events sit between launches on both streams and would perturb the timing
    timed_flags = opts.flags | lr.RT_TIME_KERNELS
    opts_timed = lr.render_opts(W, H, flags=timed_flags, **common)

    def step(o=opts, i=0):
        f = i % F
        ctxs[f].render_device(o, outs[f][0].data_ptr(), outs[f][1].data_ptr(), streams[f].cuda_stream)

    for i in range(max(args.warmup, F)):
        step(i=i)
    torch.cuda.synchronize(dev)
    st = ctx.stats()                       # rays of one frame-slice (deterministic: same every step)
    local_rays = st.rays
    ctx.kernel_times()                     # discard anything recorded before the timed region

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(streams[i % F])
        step(i=i)
        evs[i][1].record(streams[i % F])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    ktimes = {}
    if not args.no_kernel_times:
        for _ in range(args.steps):
            step(opts_timed)
        torch.cuda.synchronize(dev)
        ktimes = ctx.kernel_times()        # {family: (ms summed over K instrumented frames, launches)}

    # one more, untimed frame with the instrumented kernels: exact box / sphere test counts
    work = lr.render_opts(W, H, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8 | lr.RT_COUNT_WORK, **common)
    ctx.render_device(work, out_rgb.data_ptr(), out_bgr.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    wst = ctx.stats()
    try:
        gen_q, gen_s = ctx.generation_counts()
    except lr.RtError:
        gen_q, gen_s = [], []

    # PCIe-inclusive rate: rt_render into host buffers, D2H of f32 RGB + BGR included.
    # Reported beside `value`, never as it.
    host_ms = []
    for _ in range(2):
        t0h = time.perf_counter()
        ctx.render(opts)
        host_ms.append((time.perf_counter() - t0h) * 1e3)
    host_ms = min(host_ms)

    t = torch.tensor([elapsed, float(local_rays), avg_kernel_ms, float(wst.sphere_tests), float(wst.box_tests)],
                     dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, avg_kernel_ms = mx[0].item(), mx[2].item()
        total_rays = int(sm[1].item())
        sphere_tests, box_tests = int(sm[3].item()), int(sm[4].item())
    else:
        total_rays = local_rays
        sphere_tests, box_tests = wst.sphere_tests, wst.box_tests

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = total_rays * args.steps / elapsed / 1e6
        pixels_local = len(rows) * W
        scene_bytes = args.spheres * (32 + 4) + args.spheres * 128 + 2 * 56
        algo_bytes = pixels_local * (12 + 3) + scene_bytes          # f32 RGB + u8 BGR writes + scene read once
        achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9
        key = f"{args.config}_{W}x{H}_n{args.spheres}_d{args.depth}"
        traffic = pmc_traffic(key)
        kernels = {}
        for fam, (ms, n) in ktimes.items():
            if n:
                kernels["wf_" + fam] = {"avg_launch_us": round(ms / n * 1e3, 2),
                                        "launches_per_frame": round(n / args.steps, 2),
                                        "ms_per_frame": round(ms / args.steps, 4)}
        if path_cfg:        # one launch of path_kernel per frame: its duration is the render's
            kernels = {"path_kernel": {"avg_launch_us": round(avg_kernel_ms * 1e3, 2), "launches_per_frame": 1.0,
                                       "ms_per_frame": round(avg_kernel_ms, 4)}}
        dominant = max(kernels, key=lambda k: kernels[k]["ms_per_frame"]) if kernels else None
        if path_cfg:
            workload = (f"C1: test_scene.txt (IndirectPhong Cornell box, no lights) at {W}x{H}, {spp} random AA "
                        f"samples per pixel (keyed draws, seed {cfg[3]}), depth {args.depth}")
        else:
            workload = (f"{args.config.upper()}: {W}x{H}, {args.spheres} random Phong spheres, 2 point lights, "
                        f"depth {args.depth}, 1 spp centre jitter (seed {cfg[3]})")
        line = {
            "metric": "Mrays/sec at 4096x4096, 1000 spheres, depth 8; fraction of HBM roofline",
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload,
                       "width": W, "height": H, "spheres": args.spheres, "max_depth": args.depth, "spp": spp,
                       "rays_per_frame": total_rays, "band_rows": BAND, "parallelism": f"row-bands x{world}", "frames_in_flight": F,
                       "algo": args.algo},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": "path_kernel" if path_cfg else
                                   "whole render (wavefront launches)" if args.algo in ("auto", "wavefront") else
                                   "trace_frame_kernel", "avg_kernel_ms": round(avg_kernel_ms, 4),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "kernels": kernels or None, "dominant_kernel": dominant,
                         "note": "VALU-bound path (f64 exact tests, f32 BVH boxes); HBM fraction reported "
                                 "because the metric asks for it; see 'compute'"},
            "compute": {"bound": "valu", "sphere_tests_per_frame": sphere_tests, "box_tests_per_frame": box_tests,
                        "f64_flops_per_sphere_test": 19, "f32_flops_per_box_test": 20,
                        "achieved_f64_tflops": round(sphere_tests * 19 / (avg_kernel_ms * 1e-3) / 1e12, 3),
                        "achieved_f32_box_tflops": round(box_tests * 20 / (avg_kernel_ms * 1e-3) / 1e12, 3),
                        "peak_f64_tflops": FP64_VALU_PEAK_TFLOPS,
                        "tests_per_ray": round((sphere_tests + box_tests) / max(1, total_rays), 2),
                        "generation_queue_sizes": gen_q[:args.depth + 3] if world == 1 else None,
                        "generation_shaded": gen_s[:args.depth + 3] if world == 1 else None},
        }
        if world == 1:
            line["pcie_inclusive"] = {"ms_per_frame": round(host_ms, 3),
                                      "value": round(total_rays / (host_ms * 1e-3) / 1e6, 3), "unit": "Mrays/s",
                                      "note": f"rt_render to pageable host buffers: kernels + D2H of "
                                              f"{W * H * 12 / 1e6:.0f} MB f32 RGB + {W * H * 3 / 1e6:.0f} MB BGR "
                                              f"(+ host allocation)"}
        if world == 1 and not args.no_cpu:
            try:
                draws = dict(jitter=1, seed=cfg[3], rng=1) if path_cfg else {}
                line["cpu_baseline"] = cpu_baseline(spec, args, **draws)
            except Exception as e:  # the oracle is optional on a box where it was not built
                line["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
