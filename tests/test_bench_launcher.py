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
    assert d["scaling"] == "strong"            # the headline frame itself dealt over the ranks
    assert d["config"] == "c3"                  # every N measures the headline config
    assert d["frame"] == [4096, 4096]
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"].replace("\u00d7", "x")


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


def test_default_scaling_is_strong_and_weak_lines_name_their_frame(monkeypatch):
    """N > 1 deals the 4096^2 headline frame itself over the ranks unless weak
    scaling is asked for; a weak line's metric names its larger frame, so it is
    never read as the headline."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]
    import bench
    headline = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"].replace("\u00d7", "x")
    assert bench.HEADLINE_METRIC == headline
    for n in (1, 2, 4, 8):
        monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", str(n)])
        a = bench.parse()
        assert a.scaling == "strong"
        w, h, base = bench.frame_of(a, n)
        assert (w, h) == base == (4096, 4096)
        assert bench.metric_name(a.config, 1000, 8, a.view, w, h, a.scaling, n) == headline
    for n in (2, 4, 8):
        monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", str(n), "--scaling", "weak"])
        a = bench.parse()
        w, h, base = bench.frame_of(a, n)
        assert base == (4096, 4096) and w > 4096 and h > 4096
        m = bench.metric_name(a.config, 1000, 8, a.view, w, h, a.scaling, n)
        assert m != headline and f"{w}x{h}" in m and "weak" in m
    # any other frame names itself
    assert bench.metric_name("c3", 1000, 8, "dense", 4096, 4096) != headline
    assert bench.metric_name("c4", 10000, 8, "default", 8192, 8192).startswith("Mrays/sec at 8192x8192")


def test_weak_dry_run_names_the_larger_frame():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                          "--scaling", "weak", "--dry-run"], capture_output=True, text=True, timeout=180, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["scaling"] == "weak" and d["frame"][0] > 4096
    assert f"{d['frame'][0]}x{d['frame'][1]}" in d["metric"]


def test_cpu_baseline_sample_is_bounded():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]
    import bench
    from libraytrace import scenes
    r = bench.cpu_sample(scenes.config3(256, 256), threads=2, budget_s=1.0, draws={})
    assert r["rays"] > 0 and r["value"] > 0 and r["seconds"] < 10
    assert bench.cpu_share() >= 1 and bench.cpu_model()
