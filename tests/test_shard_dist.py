"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path: row bands
dealt round-robin over ranks (libraytrace/shard.py), each
rank rendering only its bands through the band fields of rt_render_opts, then
a host-side gather.  No GPU here, so each rank renders its bands with the
oracle through the SAME band parameters the device path receives; the GPU
side of the same decomposition is tests/test_gpu_parity.py
::test_sharded_frame_is_bit_identical."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from libraytrace import scenes, shard
from oracle import ref64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, width, height, band, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec = scenes.config3(width, height)
        tile_h, b, stride, phase = shard.band_params(height, band, world, rank)
        parts_rgb, parts_bgr, rays = [], [], 0
        if tile_h:
            r = ref64.render(spec, tile_h=tile_h, band=b, band_stride=stride, band_phase=phase, threads=2,
                             want_rgb64=False)
            parts_rgb.append(r["rgb32"]); parts_bgr.append(r["bgr"]); rays += r["counts"]["rays"]
        if shard.tail_owner(height, band, world) == rank:
            tail = shard.tail_rows(height, band)
            r = ref64.render(spec, y0=int(tail[0]), tile_h=len(tail), threads=2, want_rgb64=False)
            parts_rgb.append(r["rgb32"]); parts_bgr.append(r["bgr"]); rays += r["counts"]["rays"]
        local_rgb = np.concatenate(parts_rgb) if parts_rgb else np.zeros((0, width, 3), np.float32)
        local_bgr = np.concatenate(parts_bgr) if parts_bgr else np.zeros((0, 3 * width), np.uint8)
        rgb = shard.gather_frame(local_rgb, height, band, world, rank)
        bgr = shard.gather_frame(local_bgr, height, band, world, rank)
        # bench.py's reduction: total rays = SUM over ranks, time = MAX over ranks
        import torch
        t = torch.tensor([float(rays), float(rank + 1)], dtype=torch.float64)
        sm, mx = t.clone(), t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        if rank == 0:
            np.save(out + "_rgb.npy", rgb)
            np.save(out + "_bgr.npy", bgr)
            np.save(out + "_red.npy", np.array([sm[0].item(), mx[1].item()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("width,height,band", [(48, 40, 8), (40, 37, 4)])   # 37: ragged tail band
def test_two_rank_bands_gather_to_the_untiled_frame(tmp_path, width, height, band):
    world = 2
    out = str(tmp_path / "frame")
    mp.start_processes(_worker, args=(world, _free_port(), width, height, band, out), nprocs=world,
                       join=True, start_method="spawn")
    full = ref64.render(scenes.config3(width, height), threads=2, want_rgb64=False)
    rgb = np.load(out + "_rgb.npy")
    bgr = np.load(out + "_bgr.npy")
    red = np.load(out + "_red.npy")
    assert np.array_equal(bgr, full["bgr"])
    assert np.array_equal(rgb.view(np.uint32), full["rgb32"].view(np.uint32))
    assert red[0] == full["counts"]["rays"]
    assert red[1] == world
