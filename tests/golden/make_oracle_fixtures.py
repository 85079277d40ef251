"""Generate small golden renders with the CPU oracle (oracle/ref64.c).

These are committed so the GPU box can check the HIP path against fixed bytes
without trusting anything built there; tests/test_fixtures.py checks that the
oracle still reproduces them (guards against oracle drift).

Each fixture: <name>.npz with rgb32 (f32 HxWx3, the f64 result rounded once),
bgr (u8 HxWx3 in B,G,R order per color.rs:628-632), rays / shadow_rays (the
number of Scene::intersect calls the reference makes), and the scene text.
sha256 of the full BMP file (header + padded rows) is stored in fixtures.json.

Usage:  python tests/golden/make_oracle_fixtures.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-raytrace_amd")]

from oracle import ref64  # noqa: E402
from libraytrace import scenes  # noqa: E402


def fixture_specs():
    c2 = scenes.config2(96, 54)
    c3 = scenes.config3(64, 64)
    mirror = scenes.random_spheres(40, 48, 40, 16, seed=11, plane=True, name="mirror16")
    for o in mirror.objects:   # strong mirrors: significance never falls below 1/512 -> full depth
        o["material"] = dict(o["material"], specular=(0.9, 0.8, 0.95))
    c2f = scenes.config2_fresnel(80, 45)      # FresnelMaterial + directional light
    return {"c2_96x54": c2, "c3_64x64": c3, "mirror16_48x40": mirror, "c2fresnel_80x45": c2f}


def bmp_bytes(w, h, bgr_rows):
    pitch = (3 * w + 3) & ~3
    hdr, _ = ref64.bmp_header(w, h)
    body = bytearray()
    for y in range(h):
        body += bgr_rows[y].tobytes() + b"\0" * (pitch - 3 * w)
    return hdr + bytes(body)


def main():
    meta = {}
    for name, spec in fixture_specs().items():
        out = ref64.render(spec, want_rgb64=False)
        h, w = spec.height, spec.width
        bgr = out["bgr"].reshape(h, w, 3)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rgb32=out["rgb32"], bgr=bgr,
                            rays=np.uint64(out["counts"]["rays"]),
                            shadow_rays=np.uint64(out["counts"]["shadow_rays"]),
                            max_depth=np.uint32(spec.max_depth),
                            scene_text=np.array(spec.to_text()))
        meta[name] = {"width": w, "height": h, "max_depth": spec.max_depth,
                      "rays": out["counts"]["rays"], "shadow_rays": out["counts"]["shadow_rays"],
                      "bmp_sha256": hashlib.sha256(bmp_bytes(w, h, out["bgr"])).hexdigest()}
        print(name, meta[name])
    with open(os.path.join(HERE, "fixtures.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
