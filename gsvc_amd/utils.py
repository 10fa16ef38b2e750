"""Binning utilities, same API as the reference's gsplat/gsplat/utils.py.

Every function keeps the reference's name, arguments and return values
(utils.py:12-167); the work runs in the gfx950 kernels of binning.hip instead
of torch.cumsum / torch.sort / torch.gather.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import ops as _C


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
