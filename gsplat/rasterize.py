"""Re-export of gsvc_amd.rasterize (reference gsplat/rasterize.py)."""
from gsvc_amd.rasterize import _RasterizeGaussians, rasterize_gaussians  # noqa: F401
