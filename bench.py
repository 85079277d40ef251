"""Headline benchmark: Mrays/s at 4096x4096, 1000 spheres, depth 8 (BASELINE.json).

One step = one full pass of the hot path over one frame of the headline
workload (config C3): every pixel's camera ray, its Phong
shading with shadow rays to 2 point lights, and mirror bounces to depth 8,
f64 arithmetic, f32 RGB + sRGB BGR written to HBM.  The scene is uploaded once
(inputs resident in HBM before timing); output stays in HBM (the PCIe copy and
the host gather are reported beside `value`, never in it).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

Every N measures the headline config C3: the N = 1 line is the headline
number, and N > 1 deals that same 4096² frame over the N GPUs (strong
scaling, below); --config c4 --gpus N gives BASELINE config 4's curve
(8192², 10k spheres, depth 8, one image tiled across the N GPUs).  --inflight F renders
successive steps through F contexts into F output buffers (every step still
one whole frame, all K finished inside the timed region); the roofline's
per-render duration then comes from K further renders issued one at a time.

Multi-GPU: run as plain `python bench.py --gpus N` the script starts N rank
processes itself (before anything touches a GPU), one device each; under
torchrun it uses the launcher's ranks.  Pixels are independent (main.rs:45-57),
so the frame's rows are dealt in 16-row bands round-robin over the ranks
(libraytrace/shard.py) and no collective touches the data path (RCCL carries
the barrier and the max-over-ranks timing only).  Default "scaling": "strong":
the N = 1 frame itself dealt over the N ranks (the metric's own 4096² config,
BASELINE config 4's "image tiled across GPUs"; per-rank projection on one GPU:
--shard-of N), value = the frame's rays x K / max-over-ranks time.  --scaling
weak (opt-in) renders the same scene and view at sqrt(N) x the resolution,
every rank a 4096^2-pixel share; its line names that larger frame in
`metric`, never the headline's.
After the timed region every rank renders its bands again, K frames, with
rt_render straight into ONE shared page-locked host frame (the host gather of
SURVEY §8(e), RT_OUT_FRAME_ROWS: the copies overlap the render), reported as
`host_frame` beside the device-only value.  --config c4 / c5 select the larger configs of BASELINE.json;
--config c1 the reference's own scene (test_scene.txt: IndirectPhong Cornell
box, 1024 random AA samples, 256x256, depth 1) on the path kernel.

Rays = every Scene::intersect query the reference would issue (camera +
reflection + shadow), counted by the kernel; identical to the oracle's count
(tests/test_gpu_parity.py).  The value uses the rays the device actually
traced (rt_stats.traced_rays), which differ only for centre jitter with spp > 1.
"""
import argparse
import json
import mmap
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VALU_PEAK_TFLOPS = 78.6   # spec, FMA counted; the kernel issues no FMA (parity), so ~39.3 is its ceiling
BAND = 16
# Frames in flight (--inflight F) are opt-in: measured at the driver's K = 20 / W = 5 on one MI355X
# (tools/gpu_s5.sh), F = 4 with 16 hardware queues gave 3.23-3.28 vs 3.19-3.28 ms per C3 frame and
# 0.87-1.04 vs 0.91-0.93 ms for one rank's share of N = 8; an earlier sweep's 3.17 / 0.75 did not repeat.


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # K = 20 / W = 5 by default (the driver's own choice): C3 2.809 vs 2.865 ms per frame at K = 5 / W = 2
    # on one box (the first frames after a short warmup run before the clocks settle)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c3", choices=["c1", "c3", "c4", "c5"],
                   help="c3 4096^2/1000 spheres/depth 8 (headline); c4 8192^2/10k/8; c5 16384^2/100k/16; "
                        "c1 test_scene.txt 256^2, 1024 random AA samples, depth 1 (path kernel)")
    p.add_argument("--spp", type=int, default=0, help="c1: AA samples (default: the scene's 1024)")
    p.add_argument("--view", default="default", choices=["default", "dense"],
                   help="c3/c4/c5 camera: default (0, 3, 10), 71%% of C3's camera rays miss every sphere; dense: "
                        "just in front of the sphere box looking in (context line, never the headline)")
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--spheres", type=int, default=0)
    p.add_argument("--depth", type=int, default=-1)
    p.add_argument("--algo", default="auto", choices=["auto", "wavefront", "lds", "global", "path"])
    p.add_argument("--cpu-seconds", type=float, default=20.0,
                   help="target CPU time of the cpu_baseline samples (split between 1 thread and all threads)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                   help="N > 1: strong (default) = the N=1 frame dealt over N ranks in row bands; weak = the frame "
                        "side grows by sqrt(N) (same scene and view, every rank renders the N=1 pixel count; the "
                        "line's metric then names the larger frame)")
    p.add_argument("--shard-of", type=int, default=0,
                   help="(diagnostic, one process) render only rank 0's row bands of an N-rank frame; "
                        "its time is what each rank of an N-GPU run spends")
    p.add_argument("--no-kernel-times", action="store_true",
                   help="skip the instrumented frames that time every launch with HIP events")
    p.add_argument("--no-gather", action="store_true", help="skip the host-gather measurement")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive rt_render measurement")
    p.add_argument("--inflight", type=int, default=1,
                   help="frames in flight: F contexts (each its own working set and streams) render successive "
                        "steps into F output buffers, so frame i+1's first generations overlap frame i's tail "
                        "(c4/c5: each context's working set is sized to an 80 GB budget, so keep F = 1 there)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="N > 1: process-group backend for the barrier and the max-over-ranks timing (nccl = RCCL; "
                        "gloo rehearses N ranks on fewer GPUs, ranks sharing a device round-robin)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: start the ranks, form the process group, report the "
                        "world and the devices seen, render nothing")
    return p.parse_args()


# ---------------------------------------------------------------- launcher

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`python bench.py --gpus N`: start N rank processes of this script (one per
    device) and wait for them.  The parent never touches a GPU."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:                 # one rank failed: stop the others (their exact PIDs)
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


# ---------------------------------------------------------------- CPU baseline

def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """Host threads this process may use: the affinity mask, capped by a cgroup
    CPU quota when one is set (a GPU box shares its host between jobs)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_sample(spec, threads, budget_s, draws, use_lib=None):
    """The oracle (algorithmically the reference: same recursion, same linear
    scan, f64) on a deterministic sample of the same frame: every stride-th row,
    a centred window of columns, grown until it takes about budget_s."""
    from oracle import ref64
    if use_lib is not None:
        draws = dict(draws, use_lib=use_lib)
    W, H = spec.width, spec.height
    stride, tw = max(1, H // 4), min(W, 64)
    for _ in range(8):
        rows = H // stride
        x0 = (W - tw) // 2
        t0 = time.time()
        r = ref64.render(spec, x0=x0, tile_w=tw, tile_h=rows, band=1, band_stride=stride, band_phase=0,
                         threads=threads, want_rgb64=False, **draws)
        dt = time.time() - t0
        if dt >= 0.5 * budget_s or (stride == 1 and tw == W):
            break
        f = budget_s / max(dt, 1e-3)
        if tw < W:
            ntw = min(W, int(tw * f))
            f = f * tw / ntw
            tw = ntw
        if f > 1.2 and stride > 1:
            stride = max(1, int(stride / f))
    rays = r["counts"]["rays"]
    return {"value": rays / dt / 1e6, "threads": threads, "seconds": round(dt, 2), "rays": rays,
            "sample": f"{rows} rows (every {stride}th) x {tw} px (columns {x0}..{x0 + tw - 1}) of the same frame"}


def cpu_baseline(spec, args, **draws):
    """the oracle built -O3 -march=native for this host (no FP
    contraction: the same bits as the checker build, verified on a small tile
    first) on every host thread this job may use, and on one thread."""
    from oracle import ref64
    import numpy as np
    share = cpu_share()
    try:
        nlib, build = ref64.native_lib()
        probe = dict(x0=spec.width // 2 - 8, tile_w=16, y0=spec.height // 2 - 4, tile_h=8, threads=1, **draws)
        a, b = ref64.render(spec, **probe), ref64.render(spec, use_lib=nlib, **probe)
        if not (np.array_equal(a["bgr"], b["bgr"]) and np.array_equal(a["rgb32"], b["rgb32"])):
            raise RuntimeError("the -march=native build differs from the checker build")
    except Exception as e:                  # no compiler on this host: the checker build (-O2), said so
        nlib, build = None, f"oracle/Makefile (-O2; native build failed: {e})"
    one = cpu_sample(spec, 1, args.cpu_seconds / 2, draws, nlib)
    allc = cpu_sample(spec, share, args.cpu_seconds / 2, draws, nlib) if share > 1 else one
    return {"value": allc["value"], "unit": "Mrays/s", "cores": allc["threads"], "kind": "port",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(), "build": build,
            "sample": f"{allc['sample']}; {allc['rays']} rays in {allc['seconds']} s; oracle/ref64.c "
                      f"(linear scan, f64), {allc['threads']} threads",
            "one_thread": {"value": one["value"], "unit": "Mrays/s",
                           "sample": f"{one['sample']}; {one['rays']} rays in {one['seconds']} s",
                           "note": "the reference's own execution model: one thread (main.rs:45-59)"}}


# ---------------------------------------------------------------- helpers

def pmc_traffic(config_key, sources_id):
    """HBM bytes per render from the committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), and where the
    figure comes from.  Reported only when that entry was measured on these
    native sources (sources_id) with the default tuning; otherwise None and
    the reason (a stale figure is never passed off as this run's)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        e = json.load(open(path)).get(config_key)
    except Exception:
        e = None
    if not e:
        return None, "no committed PMC measurement for this config"
    if e.get("sources_id") != sources_id:
        return None, (f"stale: profiles/pmc_traffic.json[{config_key}] was measured on sources "
                      f"{e.get('sources_id')}, this build is {sources_id}")
    if e.get("tuning") or os.environ.get("RT_TUNE"):
        return None, "tuning differs from the measured default schedule"
    return float(e["hbm_bytes_per_launch"]), (f"profiles/pmc_traffic.json[{config_key}]: rocprofv3 --pmc FETCH_SIZE x2 "
                                              f"+ WRITE_SIZE, one render, same sources ({sources_id})")


class SharedFrame:
    """One host frame shared by every rank (a /dev/shm file mapped by each),
    page-locked in each process, that the ranks copy their row bands into."""

    def __init__(self, name, nbytes, create):
        import numpy as np
        self.path = "/dev/shm/" + name
        if create:
            with open(self.path, "wb") as f:
                f.truncate(nbytes)
        self.f = open(self.path, "r+b")
        self.mm = mmap.mmap(self.f.fileno(), nbytes)
        self.arr = np.frombuffer(self.mm, dtype=np.uint8, count=nbytes)
        self.pinned = False
        try:
            import torch
            ok = torch.cuda.cudart().cudaHostRegister(self.arr.ctypes.data, nbytes, 0)
            self.pinned = int(ok[0] if isinstance(ok, tuple) else ok) == 0
        except Exception:
            self.pinned = False

    def close(self, unlink):
        try:
            if self.pinned:
                import torch
                torch.cuda.cudart().cudaHostUnregister(self.arr.ctypes.data)
        except Exception:
            pass
        del self.arr
        self.mm.close()
        self.f.close()
        if unlink:
            try:
                os.unlink(self.path)
            except OSError:
                pass


def frame_gather(dist, world, rank, ctx, lr, W, H, pitch, common, steps, red_dev):
    """The multi-GPU frame end to end: every rank rt_render's its row bands
    straight into ONE shared page-locked host frame (RT_OUT_FRAME_ROWS: the library copies
    each part of its tile as the render finishes it, so the gather overlaps the render).
    Per output set: rt_ctx_reserve, two untimed frames, then K frames back to back on every
    rank between barriers; ms per frame = the slowest rank's time / K."""
    import numpy as np
    rgb_bytes, bgr_bytes = H * W * 12, H * pitch
    name = [f"rtframe_{os.environ.get('MASTER_PORT', '0')}_{os.getpid()}"]
    if world > 1:
        dist.broadcast_object_list(name, src=0)
    fr = SharedFrame(name[0], rgb_bytes + bgr_bytes, create=True) if rank == 0 else None
    if world > 1:
        dist.barrier()
    if fr is None:
        fr = SharedFrame(name[0], rgb_bytes + bgr_bytes, create=False)
    out = {"pinned": bool(fr.pinned)}
    try:
        rgb = fr.arr[:rgb_bytes].view(np.float32).reshape(H, W, 3)
        bgr = fr.arr[rgb_bytes:].reshape(H, pitch)
        for key, flags, outs in (("bgr_only", lr.RT_OUT_BGR_U8, (None, bgr)),
                                 ("rgb_and_bgr", lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8, (rgb, bgr))):
            o = lr.render_opts(W, H, flags=flags | lr.RT_OUT_FRAME_ROWS, bgr_pitch=pitch, **common)
            ctx.reserve(o, host=True)
            for _ in range(2):
                ctx.render(o, out=outs, stats=False)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                ctx.render(o, out=outs, stats=False)
            ms = (time.perf_counter() - t0) * 1e3 / steps
            if world > 1:
                import torch
                t = torch.tensor([ms], dtype=torch.float64, device=red_dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                ms = t.item()
            out[key] = ms
        del rgb, bgr, outs               # every view of the shared frame, before its mapping closes
    finally:
        if world > 1:
            dist.barrier()
        fr.close(unlink=(rank == 0))
    return out


CONFIGS = {"c1":(256, 0, 1, 1, 1.0), "c3": (4096, 1000, 8, 3, 1.0), "c4": (8192, 10000, 8, 4, 10.0 ** (1 / 3)),
           "c5": (16384, 100000, 16, 5, 100.0 ** (1 / 3))}       # side, spheres, depth, seed, box scale (scenes.config*)
HEADLINE_METRIC = "Mrays/sec at 4096x4096, 1000 spheres, depth 8; fraction of HBM roofline"   # BASELINE.json


def frame_of(args, band_world):
    """(W, H, base (W, H)) of the job's frame: the config's side (or --width/--height);
    weak scaling over band_world > 1 ranks grows it by sqrt(band_world)."""
    side = CONFIGS[args.config][0]
    base = (args.width or side, args.height or side)
    if band_world > 1 and args.scaling == "weak":
        return weak_frame(base[0], base[1], band_world) + (base,)
    return base + (base,)


def metric_name(config, spheres, depth, view, W, H, scaling="strong", ranks=1):
    """BASELINE.json's metric string only for the headline workload itself (the
    4096^2 / 1000-sphere / depth-8 frame, default view); any other frame -- a
    weak-scaled N-GPU frame included -- names its own size."""
    if config == "c3" and (W, H) == (4096, 4096) and spheres == 1000 and depth == 8 and view == "default":
        return HEADLINE_METRIC
    return (f"Mrays/sec at {W}x{H}, {spheres} spheres, depth {depth}" + (" (dense view)" if view == "dense" else "") +
            (f" (weak scaling: {ranks} ranks, each a {W * H // max(1, ranks)}-pixel share)"
             if scaling == "weak" and ranks > 1 else ""))


def weak_frame(w, h, n):
    """Weak scaling over n ranks: the same view at sqrt(n) x the resolution,
    sides rounded to whole 16-row bands, so each rank renders (up to that
    rounding) the N = 1 frame's pixel count."""
    f = n ** 0.5
    return max(BAND, int(round(w * f / BAND)) * BAND), max(BAND, int(round(h * f / BAND)) * BAND)


# ---------------------------------------------------------------- main

def main():
    args = parse()
    args.inflight = max(1, args.inflight)
    if args.inflight > 1:
        # F contexts x 3 streams each (nearest-hit chain + two shadow/shading streams): with HIP's
        # default of 4 hardware queues they alias and the frames serialise; 16 gives each stream
        # its own queue (set before anything initialises HIP, in this process and the ranks it starts;
        # the GPU boxes export the default 4, so a lower value is raised, not kept)
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
            os.environ["GPU_MAX_HW_QUEUES"] = "16"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "gloo" and n_dev:
        local %= n_dev                               # rehearsal: several ranks per device
    elif world > 1 and not args.dry_run and local >= n_dev:
        raise SystemExit(f"rank {rank}: local rank {local} but only {n_dev} devices (one device per rank; "
                         f"--dist-backend gloo rehearses more ranks than devices)")
    if world > 1:
        if args.dist_backend == "nccl" and not args.dry_run:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    red_dev = "cpu" if (args.dist_backend == "gloo" or args.dry_run) else torch.device("cuda", local)

    def distinct_devices():
        """Devices the ranks render on (n_gpus counts devices, not ranks)."""
        t = torch.zeros(max(1, n_dev), dtype=torch.float64, device=red_dev)
        if not args.dry_run and n_dev:
            t[local] = 1
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.sum().item())

    if args.dry_run:
        n_gpus = distinct_devices()
        if rank == 0:
            dw, dh, _ = frame_of(args, world)
            cf = CONFIGS[args.config]
            print(json.dumps({"dry_run": True, "ranks": world, "n_gpus": n_gpus, "devices_visible": n_dev,
                              "scaling": args.scaling, "backend": args.dist_backend, "config": args.config,
                              "frame": [dw, dh],
                              "metric": metric_name(args.config, args.spheres or cf[1],
                                                    cf[2] if args.depth < 0 else args.depth, args.view, dw, dh,
                                                    args.scaling, world)}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    import numpy as np
    import libraytrace as lr
    from libraytrace import scenes, shard
    dev = torch.device("cuda", local)

    cfg = CONFIGS[args.config]
    path_cfg = args.config == "c1"
    band_world = args.shard_of if (args.shard_of > 1 and world == 1) else world
    args.width, args.height, base_wh = frame_of(args, band_world)
    args.spheres = args.spheres or cfg[1]
    args.depth = cfg[2] if args.depth < 0 else args.depth
    if path_cfg:
        spec = scenes.config1(args.width, args.height, max_depth=args.depth)
        if args.spp:
            spec.antialias = args.spp
    else:
        spec = scenes.random_spheres(args.spheres, args.width, args.height, args.depth, seed=cfg[3],
                                     box_scale=cfg[4], name=args.config, view=args.view)
    spp = spec.antialias
    jitter = lr.RT_JITTER_RANDOM if path_cfg else lr.RT_JITTER_CENTER
    W, H = spec.width, spec.height
    assert H % BAND == 0, "bench frames are whole bands"
    scene = lr.Scene.deserialize(spec.to_text())
    F = max(1, args.inflight)
    t0x = time.perf_counter()
    ctxs = [lr.Context(local, tuning="env") for _ in range(F)]
    create_ms = (time.perf_counter() - t0x) * 1e3 / F
    upload_ms = []
    for c in ctxs:
        # rt_scene_upload: host BVH + light-view grid builds + the blob's H2D copy, paid once per scene
        t0u = time.perf_counter()
        c.upload(scene)
        torch.cuda.synchronize(dev)
        upload_ms.append((time.perf_counter() - t0u) * 1e3)
    t0u = time.perf_counter()
    ctxs[0].upload(scene)                  # again: the blob exists, so no allocation (a caller's scene change)
    torch.cuda.synchronize(dev)
    upload_ms.append((time.perf_counter() - t0u) * 1e3)
    ctx = ctxs[0]
    rows = shard.local_rows(H, BAND, band_world, rank)
    algo = {"auto": lr.RT_ALGO_AUTO, "wavefront": lr.RT_ALGO_WAVEFRONT, "lds": lr.RT_ALGO_BRUTE_LDS,
            "global": lr.RT_ALGO_BRUTE_GLOBAL, "path": lr.RT_ALGO_PATH}[args.algo]
    common = dict(tile_h=len(rows), band=BAND, band_stride=band_world, band_phase=rank, max_depth=args.depth,
                  spp=spp, algo=algo, jitter=jitter, seed=cfg[3])
    opts = lr.render_opts(W, H, flags=lr.RT_OUT_RGB_F32 | lr.RT_OUT_BGR_U8, **common)
    pitch = 3 * W
    outs = [(torch.empty((len(rows), W, 3), dtype=torch.float32, device=dev),
             torch.empty((len(rows), pitch), dtype=torch.uint8, device=dev)) for _ in range(F)]
    out_rgb, out_bgr = outs[0]
    # a real (non-null) stream: the library launches on exactly this stream, so the
    # torch events below bracket the kernels (handle 0 would select the context's own stream)
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    stream = streams[0]

    # per-kernel-family launch durations come from K more frames that record HIP
    # events around every launch (RT_TIME_KERNELS), after the timed region: the
    # events sit between launches on both streams and would perturb the timing
    opts_timed = lr.render_opts(W, H, flags=opts.flags | lr.RT_TIME_KERNELS, **common)

    def step(o=opts, i=0):
        f = i % F
        ctxs[f].render_device(o, outs[f][0].data_ptr(), outs[f][1].data_ptr(), streams[f].cuda_stream)

    # rt_ctx_reserve (outside the timed region, like the upload): the schedule's streams and hardware
    # queues, the working set and the queues' scratch, so that the first frame runs warm
    reserve_ms = []
    for c, s_ in zip(ctxs, streams):
        t0r = time.perf_counter()
        c.reserve(opts, stream_ptr=s_.cuda_stream)
        reserve_ms.append((time.perf_counter() - t0r) * 1e3)
    # the first two frames after it, against each other: what a process that renders one frame (as
    # main.rs does) pays for its render once ctx_create, the upload and the reserve are done
    cold_ms = []
    for i in range(max(args.warmup, F)):
        t0c = time.perf_counter()
        step(i=i)
        if i < 2:
            torch.cuda.synchronize(dev)
            cold_ms.append((time.perf_counter() - t0c) * 1e3)
    torch.cuda.synchronize(dev)
    st = ctx.stats()                       # rays of one frame-slice (deterministic: same every step)
    local_rays, local_traced = st.rays, st.traced_rays
    ctx.kernel_times()                     # discard anything recorded before the timed region

    # one context: a pair of HIP events brackets the K renders on their stream (the per-render
    # device time is the span / K); an event pair per render would put two more marker packets
    # between consecutive renders on the device (rocprofv3 kernel trace of an 8-way C3 share: the
    # idle gap at the frame boundary 40 us with them, 32 us without)
    span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)] \
        if F > 1 else []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if F == 1:
        span[0].record(stream)
    for i in range(args.steps):
        if F > 1:
            evs[i][0].record(streams[i % F])
        step(i=i)
        if F > 1:
            evs[i][1].record(streams[i % F])
    if F == 1:
        span[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in evs] if F > 1 else [span[0].elapsed_time(span[1]) / args.steps]
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    if F > 1:
        # with frames in flight an event span covers other frames' work too: the roofline's
        # per-render duration comes from K more renders issued one at a time on one context
        evs1 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for i in range(args.steps):
            evs1[i][0].record(stream)
            step(i=0)
            evs1[i][1].record(stream)
            evs1[i][1].synchronize()
        kernel_ms = [a.elapsed_time(b) for a, b in evs1]
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

    # the frame end to end: every rank's rt_render of its bands straight into one
    # shared page-locked host frame, the gather overlapping the render (RT_OUT_FRAME_ROWS)
    hframe = None
    if not args.no_gather and not path_cfg:
        hframe = frame_gather(dist, world, rank, ctx, lr, W, H, pitch, common, args.steps, red_dev)

    # PCIe-inclusive rate: rt_render into reused pageable host buffers, kernels + D2H.
    # Reported beside `value`, never as it.
    host = {}
    if world == 1 and not args.no_pcie:
        hb = np.zeros((len(rows), pitch), np.uint8)
        hr = np.zeros((len(rows), W, 3), np.float32)
        for name, out in (("bgr", (None, hb)), ("rgb_bgr", (hr, hb))):
            # untimed: the first renders into a fresh pageable buffer run 2.5x slower (page faults and
            # page placement of the host buffer: 11.4-12.2 vs 4.3-4.7 ms for C3's BGR, settling after ~4 calls)
            for _ in range(4):
                ctx.render(opts, out=out, stats=False)
            ms = []
            for _ in range(5):
                t0h = time.perf_counter()
                ctx.render(opts, out=out, stats=False)
                ms.append((time.perf_counter() - t0h) * 1e3)
            host[name] = min(ms)
            host[name + "_samples"] = [round(x, 3) for x in ms]

    n_gpus = distinct_devices()
    t = torch.tensor([elapsed, float(local_rays), avg_kernel_ms, float(wst.sphere_tests), float(wst.box_tests),
                      float(local_traced)], dtype=torch.float64, device=red_dev)
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, avg_kernel_ms = mx[0].item(), mx[2].item()
        total_rays, total_traced = int(sm[1].item()), int(sm[5].item())
        sphere_tests, box_tests = int(sm[3].item()), int(sm[4].item())
    else:
        total_rays, total_traced = local_rays, local_traced
        sphere_tests, box_tests = wst.sphere_tests, wst.box_tests

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = total_traced * args.steps / elapsed / 1e6
        pixels_local = len(rows) * W
        scene_bytes = args.spheres * (32 + 4) + args.spheres * 128 + 2 * 56
        algo_bytes = pixels_local * (12 + 3) + scene_bytes          # f32 RGB + u8 BGR writes + scene read once
        achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9
        key = f"{args.config}_{W}x{H}_n{args.spheres}_d{args.depth}" + ("_dense" if args.view == "dense" else "")
        if world > 1:
            traffic, traffic_source = None, "per-rank PMC traffic is measured at N = 1 only"
        elif args.shard_of > 1:                 # one rank's bands only: not the whole frame the key names
            traffic, traffic_source = None, "PMC traffic is measured on whole frames, not on --shard-of shares"
        else:
            traffic, traffic_source = pmc_traffic(key, lr.sources_id())
        kernels = {}
        for fam, (ms, n) in ktimes.items():
            if n:
                kernels["wf_" + fam] = {"avg_launch_us": round(ms / n * 1e3, 2),
                                        "launches_per_frame": round(n / args.steps, 2),
                                        "ms_per_frame": round(ms / args.steps, 4)}
        path_kernel = path_cfg or args.algo == "path"
        if path_kernel:        # one launch of path_kernel per frame: its duration is the render's
            kernels = {"path_kernel": {"avg_launch_us": round(avg_kernel_ms * 1e3, 2), "launches_per_frame": 1.0,
                                       "ms_per_frame": round(avg_kernel_ms, 4)}}
        dominant = max(kernels, key=lambda k: kernels[k]["ms_per_frame"]) if kernels else None
        if path_cfg:
            workload = (f"C1: test_scene.txt (IndirectPhong Cornell box, no lights) at {W}x{H}, {spp} random AA "
                        f"samples per pixel (keyed draws, seed {cfg[3]}), depth {args.depth}")
            metric = f"Mrays/sec at {W}x{H}, test_scene.txt, {spp} AA samples, depth {args.depth}"
        else:
            cam_txt = ("camera at (0, 3, 10) looking into the sphere box" +
                       (" (71% of the camera rays miss every sphere)" if args.config == "c3" else "")
                       if args.view == "default" else
                       "dense view: camera at (0, 3.15, -0.5) inside the front of the sphere box looking in")
            workload = (f"{args.config.upper()}: {W}x{H}, {args.spheres} random Phong spheres, 2 point lights, "
                        f"depth {args.depth}, {spp} spp centre jitter (seed {cfg[3]}); {cam_txt}" +
                        (f"; one image tiled across {world} GPUs" if args.scaling == "strong" and world > 1 else "") +
                        (f"; weak scaling: the same view at {W}x{H} dealt in {BAND}-row bands over {world} GPUs, "
                         f"each rank a {base_wh[0]}x{base_wh[1]}-pixel share" if args.scaling == "weak" and world > 1
                         else ""))
            metric = metric_name(args.config, args.spheres, args.depth, args.view, W, H, args.scaling, band_world)
            if args.shard_of > 1 and world == 1:          # a diagnostic share, never the headline
                metric += f" (rank 0's row bands of a {band_world}-rank frame only)"
        line = {
            "metric": metric,
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload,
                       "width": W, "height": H, "spheres": args.spheres, "max_depth": args.depth, "spp": spp,
                       "rays_per_frame": total_rays, "traced_rays_per_frame": total_traced, "band_rows": BAND,
                       "parallelism": f"row-bands x{world}", "ranks": world, "frames_in_flight": F,
                       "algo": args.algo},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_source,
                         "kernel": "path_kernel" if path_kernel else
                                   "whole render (wavefront launches)" if args.algo in ("auto", "wavefront") else
                                   "trace_frame_kernel", "avg_kernel_ms": round(avg_kernel_ms, 4),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "kernels": kernels or None, "dominant_kernel": dominant,
                         "note": "latency-bound traversal (f64 exact tests, f32 BVH boxes); HBM fraction reported "
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
        if len(cold_ms) == 2:
            line["first_frame_ms"] = {"first": round(cold_ms[0], 3), "second": round(cold_ms[1], 3),
                                      "note": "wall clock of the first two renders after rt_scene_upload and "
                                              "rt_ctx_reserve (synchronised; reserve_ms: the working set's hipMalloc, "
                                              "the streams' hardware queues and scratch; ctx_create_ms: the context "
                                              "and the kernels' code objects)"}
            line["first_frame_ms"]["reserve_ms"] = round(reserve_ms[0], 3)
            line["first_frame_ms"]["ctx_create_ms"] = round(create_ms, 3)
        line["upload_ms"] = {"first": round(upload_ms[0], 3), "repeat": round(min(upload_ms[1:]), 3),
                             "note": "rt_scene_upload once per scene, outside the timed region: host SAH BVH + "
                                     "4-wide tree + light-view grids + camera view, then one H2D copy of the blob"}
        if hframe is not None:
            def hf(ms):
                return {"ms_per_frame": round(ms, 3), "value": round(total_traced / (ms * 1e-3) / 1e6, 3),
                        "unit": "Mrays/s", "vs_device_only": round(ms / ms_per_step, 3)}
            line["host_frame"] = {
                "bgr_only": hf(hframe["bgr_only"]), "rgb_and_bgr": hf(hframe["rgb_and_bgr"]),
                "pinned": hframe["pinned"], "bytes_per_frame": {"bgr_only": H * W * 3, "rgb_and_bgr": H * W * 15},
                "device_only_ms_per_frame": round(ms_per_step, 4),
                "note": ("every rank rt_render's its row bands straight into ONE shared page-locked host frame "
                         "(RT_OUT_FRAME_ROWS: the gather of SURVEY 8(e) overlapping the render: the frame copied after "
                         "the camera pass, then the packed segments of the chain pixels), K frames back to back; "
                         "the slowest rank's ms per frame" +
                         (f"; here rank 0's bands of a {band_world}-rank frame only" if band_world > world else ""))}
        if host:
            line["pcie_inclusive"] = {
                "bgr_only": {"ms_per_frame": round(host["bgr"], 3),
                             "value": round(total_traced / (host["bgr"] * 1e-3) / 1e6, 3), "unit": "Mrays/s"},
                "rgb_and_bgr": {"ms_per_frame": round(host["rgb_bgr"], 3),
                                "value": round(total_traced / (host["rgb_bgr"] * 1e-3) / 1e6, 3), "unit": "Mrays/s"},
                "samples_ms": {"bgr_only": host["bgr_samples"], "rgb_and_bgr": host["rgb_bgr_samples"]},
                "note": f"rt_render into reused pageable host buffers: kernels + D2H of {W * H * 3 / 1e6:.0f} MB "
                        f"BGR (+ {W * H * 12 / 1e6:.0f} MB f32 RGB) through the pinned staging slices: the frame "
                        f"after the camera pass, during the later generations, then the packed segments of the "
                        f"chain pixels (tuning sparse_out, DESIGN.md §3.11)"}
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
