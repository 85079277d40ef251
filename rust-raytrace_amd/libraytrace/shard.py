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


def band_params(height, band, world, rank):
    """rt_render_opts fields for `rank`'s full bands: (tile_h, band, band_stride, band_phase)."""
    return len(local_rows(height, band, world, rank)), band, world, rank


def gather_frame(local, height, band, world, rank, group=None):
    """Host-side gather over torch.distributed (any backend with all_gather;
    the data path itself needs no collective): every rank contributes its
    local rows (full bands, plus the ragged tail band on its owner, appended
    after them) and every rank gets the assembled frame.  `local` is a numpy
    array of shape (rows_of_rank, ...)."""
    import torch
    import torch.distributed as dist

    rows = [local_rows(height, band, world, r) for r in range(world)]
    owner = tail_owner(height, band, world)
    if owner is not None:
        rows[owner] = np.concatenate([rows[owner], tail_rows(height, band)])
    cap = max(len(r) for r in rows)
    row_shape = local.shape[1:]
    pad = np.zeros((cap,) + row_shape, dtype=local.dtype)
    pad[: len(local)] = local
    mine = torch.from_numpy(pad.view(np.uint8).copy())
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    frame = np.zeros((height,) + row_shape, dtype=local.dtype)
    for r in range(world):
        part = parts[r].numpy().view(local.dtype).reshape((cap,) + row_shape)
        assemble(frame, rows[r], part)
    return frame
