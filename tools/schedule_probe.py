"""Print the schedule the library picks (tuning verbose=1 -> stderr) for the
deep-chain parity scene, C3 and C4 at small sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd"), os.path.join(ROOT, "tests")]
import libraytrace as lr  # noqa: E402
from libraytrace import scenes  # noqa: E402


def deep_chain():
    s = scenes.config2(80, 60)
    s.max_depth = 6
    for i in range(46):
        r = 0.9 * 2.0 ** -i            # sphere i at x = -2 + 4 (1 - 2^-i): each level of the SAH peels one
        s.sphere((-2.0 + 4.0 * (1.0 - 2.0 ** -i), 1.5, -6.0), r,
                 scenes.phong((0.5, 0.4, 0.3), (0.5, 0.5, 0.5), 20.0, (0.01, 0.01, 0.01)))
    rng = scenes.SplitMix64(9)
    for _ in range(150):
        s.sphere((rng.uniform(-6, 6), rng.uniform(0.2, 4), rng.uniform(-14, -3)), rng.uniform(0.05, 0.4),
                 scenes.phong((0.3, 0.6, 0.9), (0.4, 0.4, 0.4), 30.0, (0, 0, 0)))
    return s


for name, spec in (("deep_chain", deep_chain()), ("c3", scenes.config3(64, 64)), ("c4", scenes.config4(64, 64))):
    with lr.Context(0, tuning="env") as ctx:
        ctx.set_tuning("verbose", 1)
        ctx.upload(lr.Scene.deserialize(spec.to_text()))
        print(name, flush=True)
        sys.stderr.flush()
        ctx.render(lr.render_opts(spec.width, spec.height, max_depth=spec.max_depth, spp=1, algo=lr.RT_ALGO_WAVEFRONT))
        sys.stderr.flush()
