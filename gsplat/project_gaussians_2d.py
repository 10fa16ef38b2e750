"""Re-export of gsvc_amd.project_gaussians_2d (reference gsplat/project_gaussians_2d.py)."""
from gsvc_amd.project_gaussians_2d import _ProjectGaussians2d, project_gaussians_2d  # noqa: F401
