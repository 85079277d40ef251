"""Extract the reference's own golden data into small committed fixtures.

Run HERE (the build container), never on the GPU box: it reads
/root/reference, which does not exist there.  The outputs are DATA only
(numbers and header bytes), not reference source:

  * srgb_tables.json   -- SRGB_VALUES[256] / SRGB_AVERAGE[255] from
                          color.rs:75-332 and color.rs:335-591, as f64 hex.
  * out_bmp_header.hex -- the 122-byte header of /root/reference/out.bmp
                          (written by bmp.rs:10-61 for 800x800).
  * out_bmp_stats.json -- 8x8 grid of 100x100-pixel block means per BGR
                          channel of out.bmp (a stochastic 1024-spp render of
                          test_scene.txt, main.rs:45-59), plus the whole-image
                          mean and the sha256 of the file.
  * test_scene.txt     -- the reference's scene fixture (test_scene.txt:1-113),
                          an input data file of the reference's own.

Usage:  python tests/golden/make_reference_fixtures.py
"""
import hashlib
import json
import os
import re
import struct

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _table(src, name):
    m = re.search(name + r": \[f64; (\d+)\] = \[(.*?)\];", src, re.S)
    n = int(m.group(1))
    vals = [float(v) for v in re.findall(r"[-+0-9.eE]+", m.group(2))]
    assert len(vals) == n, (name, len(vals), n)
    return vals


def main():
    src = open(os.path.join(REF, "src/color.rs")).read()
    values = _table(src, "SRGB_VALUES")
    average = _table(src, "SRGB_AVERAGE")
    with open(os.path.join(HERE, "srgb_tables.json"), "w") as f:
        json.dump({"source": "color.rs:75-332 (SRGB_VALUES), color.rs:335-591 (SRGB_AVERAGE)",
                   "SRGB_VALUES": [v.hex() for v in values],
                   "SRGB_AVERAGE": [v.hex() for v in average]}, f, indent=0)

    bmp = open(os.path.join(REF, "out.bmp"), "rb").read()
    with open(os.path.join(HERE, "out_bmp_header.hex"), "w") as f:
        f.write(bmp[:122].hex() + "\n")

    w, h = struct.unpack("<ii", bmp[18:26])
    pitch = (3 * w + 3) & ~3
    pix = bmp[122:]
    blocks = 8
    bw, bh = w // blocks, h // blocks
    grid = [[[0.0, 0.0, 0.0] for _ in range(blocks)] for _ in range(blocks)]
    tot = [0.0, 0.0, 0.0]
    for y in range(h):
        row = pix[y * pitch:y * pitch + 3 * w]
        for x in range(w):
            for c in range(3):
                v = row[3 * x + c]
                grid[y // bh][x // bw][c] += v
                tot[c] += v
    for by in range(blocks):
        for bx in range(blocks):
            grid[by][bx] = [v / (bw * bh) for v in grid[by][bx]]
    with open(os.path.join(HERE, "out_bmp_stats.json"), "w") as f:
        json.dump({"source": "/root/reference/out.bmp (800x800, 1024 spp, OS-seeded RNG)",
                   "sha256": hashlib.sha256(bmp).hexdigest(),
                   "width": w, "height": h, "blocks": blocks,
                   "order": "grid[by][bx][c], by=0 is the BOTTOM band (first rows in the file), c = B,G,R",
                   "mean_bgr": [v / (w * h) for v in tot],
                   "grid": grid}, f, indent=1)

    scene = open(os.path.join(REF, "test_scene.txt")).read()
    with open(os.path.join(HERE, "test_scene.txt"), "w") as f:
        f.write(scene)


if __name__ == "__main__":
    main()
