"""Per-generation traversal work: render C3 with RT_COUNT_WORK at max_depth
0..D and difference the counters (generation k's queries appear when depth
k is allowed).  Prints nearest / shadow queries and box / sphere tests per
query for each added generation."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "rust-raytrace_amd")]
import libraytrace as lr
from libraytrace import scenes

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
D = int(sys.argv[2]) if len(sys.argv) > 2 else 8
spec = scenes.random_spheres(1000, W, W, D, seed=3, name="c3")
ctx = lr.Context(0, tuning="env")
ctx.upload(lr.Scene.deserialize(spec.to_text()))
prev = None
print("depth  nearest  shadow  box/nearest  sph/nearest  box/shadow  sph/shadow")
for d in range(D + 1):
    o = lr.render_opts(W, W, max_depth=d, spp=1, flags=lr.RT_OUT_RGB_F32 | lr.RT_COUNT_WORK)
    _, _, st = ctx.render(o, rgb=True, bgr=False)
    cur = dict(near=st.rays - st.shadow_rays, sh=st.shadow_rays, nb=st.box_tests - st.shadow_box_tests,
               ns=st.sphere_tests - st.shadow_sphere_tests, sb=st.shadow_box_tests, ss=st.shadow_sphere_tests)
    dlt = cur if prev is None else {k: cur[k] - prev[k] for k in cur}
    prev = cur
    f = lambda a, b: a / b if b else 0.0
    print(f"{d:5d} {dlt['near']:8d} {dlt['sh']:7d} {f(dlt['nb'], dlt['near']):11.1f} {f(dlt['ns'], dlt['near']):11.2f}"
          f" {f(dlt['sb'], dlt['sh']):10.1f} {f(dlt['ss'], dlt['sh']):10.2f}")
