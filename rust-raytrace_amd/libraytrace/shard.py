"""Row-band sharding of one frame across devices / ranks.

Pixels are independent (main.rs:45-57), so a frame splits into bands of `band`
rows dealt round-robin: rank r renders bands r, r+N, r+2N, ...  Interleaving
balances the per-row cost (reflection-heavy rows cluster).  The C ABI renders
a rank's bands in one launch (rt_render_opts.band / band_stride / band_phase)
into a compact local buffer; `local_rows` maps its rows back to the frame.
"""
import numpy as np


def full_bands(height, band):
    return height // band


def local_rows(height, band, world, rank):
    """Frame rows rendered by `rank`, in local-buffer order (full bands only)."""
    nb = full_bands(height, band)
    rows = []
    for b in range(rank, nb, world):
        rows.extend(range(b * band, (b + 1) * band))
    return np.array(rows, dtype=np.int64)


def tail_owner(height, band, world):
    """Rank that renders the ragged last band (height % band rows), or None."""
    if height % band == 0:
        return None
    return full_bands(height, band) % world


def tail_rows(height, band):
    nb = full_bands(height, band)
    return np.arange(nb * band, height, dtype=np.int64)


def assemble(frame, rows, local):
    """Scatter a rank's local rows into the frame (host-side gather)."""
    frame[rows] = local[: len(rows)]
    return frame
