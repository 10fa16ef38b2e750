"""Re-export of gsvc_amd.rasterize_sum (reference gsplat/rasterize_sum.py)."""
from gsvc_amd.rasterize_sum import _RasterizeGaussiansSum, rasterize_gaussians_sum  # noqa: F401
