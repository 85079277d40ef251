"""The committed oracle fixtures (tests/golden/*.npz) are reproduced by the
oracle, and the scene text inside each parses back to the same scene."""
import hashlib
import json
import os

import numpy as np
import pytest

import libraytrace as lr
from oracle import ref64

GOLD = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(GOLD, "fixtures.json")))


def load_fixture(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def bmp_bytes(w, h, bgr):
    pitch = (3 * w + 3) & ~3
    hdr, _ = lr.bmp_header(w, h)
    body = b"".join(bgr[y].reshape(-1).tobytes() + b"\0" * (pitch - 3 * w) for y in range(h))
    return hdr + body


@pytest.mark.parametrize("name", sorted(META))
def test_oracle_reproduces_fixture(name):
    import sys
    sys.path.insert(0, GOLD)
    from make_oracle_fixtures import fixture_specs
    spec = fixture_specs()[name]
    fx = load_fixture(name)
    assert str(fx["scene_text"]) == spec.to_text()
    out = ref64.render(spec, want_rgb64=False)
    assert np.array_equal(out["rgb32"], fx["rgb32"])
    assert np.array_equal(out["bgr"].reshape(fx["bgr"].shape), fx["bgr"])
    assert out["counts"]["rays"] == int(fx["rays"])
    assert out["counts"]["shadow_rays"] == int(fx["shadow_rays"])
    m = META[name]
    assert hashlib.sha256(bmp_bytes(m["width"], m["height"], fx["bgr"])).hexdigest() == m["bmp_sha256"]
