"""Binning utilities, same API as the reference's gsplat/gsplat/utils.py.

Every function keeps the reference's name, arguments and return values
(utils.py:12-167); the work runs in the gfx950 kernels of binning.hip instead
of torch.cumsum / torch.sort / torch.gather.
"""
from __future__ import annotations

import os
from typing import NamedTuple, Optional, Tuple

import torch
from torch import Tensor

from . import ops as _C

# Upper bound, in entries, on the intersection buffers the sync-free binning
# may allocate (its capacity is num_points * num_tiles, which cannot
# overflow).  Above it the rasterizers read M on the host first.
BIN_CAPACITY_BUDGET = int(os.environ.get("GSVC_BIN_CAPACITY_BUDGET", str(1 << 30)))
TILE_KEEP = 256  # entries per tile the sum rasterizer blends (config.h BLOCK_SIZE)


def mark_zero_depths(depths: Tensor) -> Tensor:
    """Record that ``depths`` is identically zero (project_gaussians_2d's
    output): the rasterizers may then order entries by (tile, splat id)
    without reading the depth bits back.  Any in-place change clears it."""
    depths._gsvc_zero_version = depths._version
    return depths


def depths_known_zero(depths: Optional[Tensor]) -> bool:
    return depths is None or getattr(depths, "_gsvc_zero_version", None) == depths._version


class _LazyCount:
    """Last intersection count seen on a device, refreshed every ``period``
    calls through a non-blocking copy to pinned memory (no host sync).  Used
    only to pick a kernel variant, so a stale value is harmless."""

    def __init__(self, period=16):
        self.period = period
        self.value = 0
        self.calls = 0
        self.buf = None
        self.event = None

    def update(self, m_dev: Tensor) -> int:
        self.calls += 1
        if self.calls % self.period != 1 and self.period != 1:
            return self.value
        if torch.cuda.is_current_stream_capturing():
            return self.value  # no event query or copy inside a graph capture
        if self.event is not None and self.event.query():
            self.value = int(self.buf[0])
            self.event = None
        if self.event is None:
            if self.buf is None:
                self.buf = torch.empty((1,), dtype=torch.int32, pin_memory=True)
            self.buf.copy_(m_dev[:1], non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record()
        return self.value


_lazy_counts = {}


def _density_hint(m_dev: Tensor) -> int:
    key = m_dev.device.index
    if key not in _lazy_counts:
        _lazy_counts[key] = _LazyCount()
    return _lazy_counts[key].update(m_dev)


class TileBinning(NamedTuple):
    """Binned intersections for a rasterizer.  ``num_intersects`` is the host
    int when it was read (sized path), else None and ``m_dev`` holds M on the
    device; ``density_hint`` estimates M for the kernel choice."""
    num_intersects: Optional[int]
    m_dev: Optional[Tensor]
    gaussian_ids_sorted: Optional[Tensor]
    tile_bins: Optional[Tensor]
    density_hint: int


def map_gaussian_to_intersects(num_points: int, num_intersects: int, xys: Tensor, depths: Tensor,
                               radii: Tensor, cum_tiles_hit: Tensor,
                               tile_bounds: Tuple[int, int, int]) -> Tuple[Tensor, Tensor]:
    """utils.py:12-50: (isect_ids int64 [M] = tile << 32 | depth bits,
    gaussian_ids int32 [M]) in splat order, row-major over each splat's tiles."""
    return _C.map_gaussian_to_intersects(num_points, num_intersects, xys.contiguous(),
                                         depths.contiguous(), radii.contiguous(),
                                         cum_tiles_hit.contiguous(), tile_bounds)


def get_tile_bin_edges(num_intersects: int, isect_ids_sorted: Tensor) -> Tensor:
    """utils.py:53-74: tile_bins[tile] = [start, end) of the tile in the sorted
    intersections."""
    return _C.get_tile_bin_edges(num_intersects, isect_ids_sorted.contiguous())


def compute_cov2d_bounds(cov2d: Tensor) -> Tuple[Tensor, Tensor]:
    """utils.py:77-96: (conics [N,3], radii [N,1] float) from upper-triangular cov2d."""
    assert cov2d.shape[-1] == 3, (
        f"Expected input cov2d to be of shape (*batch, 3) (upper triangular values), "
        f"but got {tuple(cov2d.shape)}")
    num_pts = cov2d.shape[0]
    assert num_pts > 0
    return _C.compute_cov2d_bounds(num_pts, cov2d.contiguous())


def compute_cumulative_intersects(num_tiles_hit: Tensor) -> Tuple[int, Tensor]:
    """utils.py:99-118: (num_intersects as a Python int, int32 inclusive cumsum).
    Reading M is this function's one device->host sync, as in the reference."""
    cum, meta = _C.cumulative_intersects(num_tiles_hit)
    return int(meta[0].item()), cum


def bin_and_sort_gaussians(num_points: int, num_intersects: int, xys: Tensor, depths: Tensor,
                           radii: Tensor, cum_tiles_hit: Tensor, tile_bounds: Tuple[int, int, int]):
    """utils.py:121-167: (isect_ids, gaussian_ids, isect_ids_sorted,
    gaussian_ids_sorted, tile_bins).  The sort is a stable radix sort of the
    full signed int64 key, i.e. torch.sort order with ties in input order."""
    isect_ids, gaussian_ids = map_gaussian_to_intersects(num_points, num_intersects, xys, depths,
                                                         radii, cum_tiles_hit, tile_bounds)
    isect_ids_sorted, gaussian_ids_sorted = _C.sort_isect_pairs(isect_ids, gaussian_ids)
    rows = max(int(num_intersects), int(tile_bounds[0]) * int(tile_bounds[1]))
    tile_bins = _C.get_tile_bin_edges(num_intersects, isect_ids_sorted, num_rows=rows)
    return isect_ids, gaussian_ids, isect_ids_sorted, gaussian_ids_sorted, tile_bins


def bin_and_sort_for_raster(num_points: int, xys: Tensor, depths: Tensor, radii: Tensor,
                            num_tiles_hit: Tensor, tile_bounds: Tuple[int, int, int]):
    """Hot-path binning used by the rasterizers (utils.py:99-167 fused).

    One scan kernel produces cum_tiles_hit plus {M, depth-bit OR/AND}; the host
    reads those four ints in one sync (the reference's ``.item()``).  When every
    emitting splat has the same depth bits -- always the case after
    project_gaussians_2d, which writes depth 0 -- the 64-bit key order equals
    the tile order, so the fused 13-bit tile sort is used; otherwise the full
    int64 path of ``bin_and_sort_gaussians``.
    Returns (num_intersects, gaussian_ids_sorted, tile_bins[#tiles,2]).
    """
    cum, meta = _C.cumulative_intersects(num_tiles_hit, depths)
    m, dor, dand, _ = (int(x) for x in meta.tolist())
    if m < 1:
        return m, None, None
    if dor == dand:
        gids, bins, _ = _C.bin_and_sort_tiles(num_points, m, xys, depths, radii, cum, tile_bounds)
        return m, gids, bins
    _, _, _, gids, bins = bin_and_sort_gaussians(num_points, m, xys, depths, radii, cum, tile_bounds)
    return m, gids, bins


def bin_for_raster(num_points: int, xys: Tensor, depths: Optional[Tensor], radii: Tensor,
                   num_tiles_hit: Tensor, tile_bounds: Tuple[int, int, int]) -> TileBinning:
    """Binning front of the rasterizers (utils.py:99-167 as the reference's
    rasterize_sum.py:110-118 uses it).

    When the depths are known to be zero (project_gaussians_2d's output) the
    (tile, splat id) order IS the reference's sorted order, and the sync-free
    CSR binning runs (no host round trip) keeping each tile's first 256
    entries -- all the sum rasterizer reads (forward.cu:569-571,613) -- so the
    id buffers are tiles * min(num_points, 256) ints (8.4 MB at 1080p);
    otherwise -- or when that capacity exceeds BIN_CAPACITY_BUDGET -- M is read
    on the host and the sorted path of ``bin_and_sort_for_raster`` runs.
    """
    ntiles = int(tile_bounds[0]) * int(tile_bounds[1])
    per_tile = min(int(num_points), TILE_KEEP)
    cap = per_tile * ntiles
    if depths_known_zero(depths) and cap <= BIN_CAPACITY_BUDGET:
        gids, bins, meta = _C.bin_tiles_counted(num_points, xys, radii, tile_bounds, cap,
                                                TILE_KEEP if int(num_points) > TILE_KEEP else 0)
        m_dev = meta[:1]
        return TileBinning(None, m_dev, gids, bins, _density_hint(m_dev))
    m, gids, bins = bin_and_sort_for_raster(num_points, xys, depths, radii, num_tiles_hit,
                                            tile_bounds)
    return TileBinning(m, None, gids, bins, m)
