"""Native op table of the drop-in (reference gsplat/cuda/__init__.py:14-30).

The reference resolved each name lazily to the compiled CUDA extension; here
each name is the gfx950 op of gsvc_amd.ops.  Out-of-scope ops (3DGS projection,
SH, C != 3 rasterizers) are absent, so ``getattr`` raises AttributeError, as
the reference did for its unexported ``nd_rasterize_sum_*``.
"""
from gsvc_amd.ops import (  # noqa: F401
    compute_cov2d_bounds,
    get_tile_bin_edges,
    map_gaussian_to_intersects,
    project_gaussians_2d_backward,
    project_gaussians_2d_forward,
    rasterize_backward,
    rasterize_forward,
    rasterize_sum_backward,
    rasterize_sum_forward,
)
