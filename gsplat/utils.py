"""Re-export of gsvc_amd.utils (reference gsplat/utils.py)."""
from gsvc_amd.utils import (  # noqa: F401
    bin_and_sort_gaussians,
    compute_cov2d_bounds,
    compute_cumulative_intersects,
    get_tile_bin_edges,
    map_gaussian_to_intersects,
)
