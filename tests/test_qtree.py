"""The quantised 4-wide sphere tree (host_bvh.cpp quantize_bvh4, DevQNode4) on
the CPU: an independent numpy decoder of the 48-B nodes that rt_scene_upload
ships checks that every decoded child box CONTAINS the f32 child box it was
rounded from (the condition under which the device's slab test on the
quantised box culls a subset of what the f32 test culls),
that every decoded bound is an exact f32 value, and that the child refs reach
every sphere exactly once.  Through rt_qtree_nodes (host only, no GPU)."""
import numpy as np
import pytest

import libraytrace as lr
from libraytrace import scenes


def _decode(nodes):
    f = nodes["frame"].astype(np.int64)
    m = ((f & 0xFFFFFF) ^ 0x800000) - 0x800000                 # the low 24 bits, signed
    e = (f >> 24) & 0xFF
    s = np.ldexp(1.0, (e - 127).astype(np.int64))            # [n, 3]
    shift = np.arange(4) * 8
    qlo = (nodes["lo"][:, :, None].astype(np.int64) >> shift) & 0xFF     # [n, 3 axes, 4 children]
    qhi = (nodes["hi"][:, :, None].astype(np.int64) >> shift) & 0xFF
    lo = (m[:, :, None] + qlo) * s[:, :, None]
    hi = (m[:, :, None] + qhi) * s[:, :, None]
    return m, e, lo.transpose(0, 2, 1), hi.transpose(0, 2, 1)      # [n, 4 children, 3 axes]


def _check_tree(spec, leaf_max=0):
    sc = lr.Scene.deserialize(spec.to_text())
    nodes, boxes, first, count, (n, need, leaf) = sc.qtree_nodes(leaf_max)
    assert n > 0, "quantised tree not built"
    assert need <= 32
    m, e, lo, hi = _decode(nodes)
    assert (e >= 127 - 100).all() and (e <= 127 + 104).all()
    assert (np.abs(m) < 2 ** 23 + 1).all()
    used = nodes["child"] != 0xFFFF
    f32lo, f32hi = boxes[:, :, :3].astype(np.float64), boxes[:, :, 3:].astype(np.float64)
    u = used[:, :, None].repeat(3, axis=2)
    # every decoded box contains the f32 box, and every decoded bound is an f32 value
    assert (lo[u] <= f32lo[u]).all(), "a quantised lower bound lies inside the f32 box"
    assert (hi[u] >= f32hi[u]).all(), "a quantised upper bound lies inside the f32 box"
    assert (lo[u].astype(np.float32).astype(np.float64) == lo[u]).all()
    assert (hi[u].astype(np.float32).astype(np.float64) == hi[u]).all()
    assert np.isnan(boxes[~used]).all()
    # child refs: inner nodes later in breadth-first order, leaves = base + offset, every sphere once
    ch = nodes["child"].astype(np.int64)
    inner = used & (ch < 0x8000)
    leafs = used & (ch >= 0x8000)
    idx = np.arange(len(nodes))[:, None].repeat(4, axis=1)
    assert (ch[inner] > idx[inner]).all() and (ch[inner] < len(nodes)).all()
    assert len(np.unique(ch[inner])) == inner.sum() == len(nodes) - 1       # a tree: every node but the root once
    got_first = nodes["base"][:, None].astype(np.int64) + ((ch >> 3) & 0xFFF)
    got_count = (ch & 7) + 1
    assert (got_first[leafs] == first[leafs]).all() and (got_count[leafs] == count[leafs]).all()
    assert (count[leafs] <= leaf).all()
    n_spheres = sum(1 for o in spec.objects if o["shape"] == "sphere")
    cover = np.zeros(n_spheres, np.int64)
    for f0, c0 in zip(first[leafs], count[leafs]):
        cover[f0:f0 + c0] += 1
    assert (cover == 1).all()
    # how loose the rounding is (informational): mean widening relative to the box size
    ext = np.maximum(f32hi[u] - f32lo[u], 1e-30)
    return len(nodes), float(np.mean(((f32lo[u] - lo[u]) + (hi[u] - f32hi[u])) / ext))


def _extreme():
    s = scenes.config2(57, 41)
    rng = scenes.SplitMix64(9)
    for _ in range(300):
        c = (rng.uniform(-30, 30), rng.uniform(0.001, 4), rng.uniform(-60, 0))
        s.sphere(c, 10 ** rng.uniform(-4, 0.3), scenes.phong((0.3, 0.6, 0.9), (0.6, 0.6, 0.6), 50.0, (0, 0, 0)))
    s.sphere((0.0, -1e4, -5.0), 1e4, scenes.phong((0.2, 0.2, 0.2), (0.5, 0.5, 0.5), 5.0, (0, 0, 0)))
    s.sphere((1e5, 3.0, -1e5), 2e3, scenes.phong((0.9, 0.9, 0.2), (0.2, 0.2, 0.2), 5.0, (0, 0, 0)))
    return s


def _coincident_and_tiny():
    """Coincident spheres, spheres far from the origin with radii of 1e-6 (steps far
    below their coordinates: the 24-bit origin forces coarser steps), negative
    coordinates on every axis."""
    s = scenes.config2(33, 31)
    rng = scenes.SplitMix64(77)
    for _ in range(40):
        s.sphere((0.0, 0.0, -6.0), 1.5, scenes.phong((0.5, 0.5, 0.5), (0.3, 0.3, 0.3), 20.0, (0, 0, 0)))
    for _ in range(200):
        c = (rng.uniform(-900, -800), rng.uniform(-5e3, 5e3), rng.uniform(1000, 1001))
        s.sphere(c, 1e-6 * rng.uniform(1, 9), scenes.phong((0.5, 0.5, 0.5), (0.3, 0.3, 0.3), 20.0, (0, 0, 0)))
    return s


@pytest.mark.parametrize("name,leaf", [("c3", 0), ("c3", 2), ("c3", 4), ("c4", 0), ("c4", 3), ("extreme", 0),
                                       ("coincident_tiny", 0), ("c5", 0)])
def test_quantised_boxes_contain_f32_boxes(name, leaf):
    spec = {"c3": lambda: scenes.config3(64, 64), "c4": lambda: scenes.config4(64, 64),
            "c5": lambda: scenes.config5(64, 64), "extreme": _extreme, "coincident_tiny": _coincident_and_tiny}[name]()
    n, loose = _check_tree(spec, leaf)
    print(f"{name} leaf {leaf}: {n} nodes ({n * 48 / 1024:.1f} KB), mean widening {loose:.4f} of the box size")


def test_c4_tree_fits_the_nearest_hit_lds_share():
    """C4 (10k spheres, leaf size 4 as the upload picks it): the whole quantised
    tree fits the nearest-hit kernel's 72 KB LDS share (src 25), so two
    1024-thread workgroups stay resident per CU."""
    nodes, *_ , (n, need, leaf) = lr.Scene.deserialize(scenes.config4(64, 64).to_text()).qtree_nodes()
    assert leaf == 4 and n * 48 <= 72 * 1024, (n, leaf)


def test_not_representable_trees_are_refused():
    """A sphere far beyond the f32 range (its f32 box bound rounds to infinity):
    no quantised tree (0 nodes), the upload keeps the f32 / binary16 trees."""
    s = scenes.config2(16, 16)
    s.sphere((1e300, 0.0, -5.0), 1.0, scenes.phong((0.5, 0.5, 0.5), (0.3, 0.3, 0.3), 20.0, (0, 0, 0)))
    nodes, boxes, first, count, info = lr.Scene.deserialize(s.to_text()).qtree_nodes()
    assert info[0] == 0 and len(nodes) == 0


def test_size_query_fills_info_only():
    """cap_nodes 0 with null buffers is a size query: RT_OK and info[]
    as the full call reports it; a buffer too small is RT_E_INVALID."""
    import ctypes as C
    sc = lr.Scene.deserialize(scenes.config3(32, 32).to_text())
    info = np.zeros(3, np.int64)
    rc = lr.lib.rt_qtree_nodes(sc.handle, 0, None, None, None, None, 0, info.ctypes.data_as(C.POINTER(C.c_int64)))
    assert rc == lr.RT_OK and info[0] > 1
    assert tuple(int(x) for x in info) == sc.qtree_nodes()[4]
    with pytest.raises(lr.RtError) as e:
        sc.qtree_nodes(cap=1)
    assert e.value.code == lr.RT_E_INVALID
