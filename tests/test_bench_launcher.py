"""bench.py's multi-GPU launcher on CPU: `python bench.py --gpus 2` starts two
rank processes itself (no torchrun), forms the process group, and reports
n_gpus as the number of distinct devices rendered on (0 here: no GPU), not
the number of ranks.  The GPU side of the same code path runs on the box
(`python bench.py --gpus N`)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_gpus_two_spawns_two_ranks(backend):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", backend,
                          "--dry-run"], capture_output=True, text=True, timeout=180, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["ranks"] == 2
    assert d["n_gpus"] == d["devices_visible"] == 0
    assert d["scaling"] == "weak"              # the path partitions: per-GPU work fixed as N grows
    assert d["config"] == "c3"                  # every N measures the headline config


def test_config_defaults(monkeypatch):
    """Every N measures the headline config C3 (the driver's bench line is
    `--gpus 1`); --config selects BASELINE's other configs."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]
    import bench
    for argv, cfg, gpus in ((["bench.py"], "c3", 1), (["bench.py", "--gpus", "1"], "c3", 1),
                            (["bench.py", "--gpus", "8"], "c3", 8), (["bench.py", "--gpus", "4", "--config", "c4"], "c4", 4)):
        monkeypatch.setattr(sys, "argv", argv)
        a = bench.parse()
        assert (a.config, a.gpus) == (cfg, gpus)


def test_weak_scaling_keeps_the_per_rank_share():
    """Weak scaling: every rank of an N-GPU run renders (within band rounding)
    the 4096^2 pixels of the N = 1 headline frame, dealt in 16-row bands."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]
    import bench
    from libraytrace import shard
    for n in (1, 2, 4, 8):
        w, h = bench.weak_frame(4096, 4096, n) if n > 1 else (4096, 4096)
        assert w % 16 == 0 and h % 16 == 0
        for r in range(n):
            px = len(shard.local_rows(h, bench.BAND, n, r)) * w
            assert abs(px / 4096 ** 2 - 1) < 0.01, (n, r, px)


def test_cpu_baseline_sample_is_bounded():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]
    import bench
    from libraytrace import scenes
    r = bench.cpu_sample(scenes.config3(256, 256), threads=2, budget_s=1.0, draws={})
    assert r["rays"] > 0 and r["value"] > 0 and r["seconds"] < 10
    assert bench.cpu_share() >= 1 and bench.cpu_model()
