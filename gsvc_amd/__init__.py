"""gsvc_amd: MI355X-native 2D Gaussian-splat rasterizer for GSVC.

Drop-in replacement of the 2D path of the gsplat 0.1.3 package vendored by
ac-freeman/GSVC (reference gsplat/gsplat/__init__.py:1-47): the same public
functions and deprecated ``Function`` shims, backed by hand-written gfx950
kernels behind a C ABI (include/gsvc_amd.h).  The repo-root ``gsplat`` package
re-exports this module so GSVC's ``from gsplat.project_gaussians_2d import
project_gaussians_2d`` / ``from gsplat.rasterize_sum import
rasterize_gaussians_sum`` run unchanged on ROCm.

Out of scope (3DGS and unused 2D variants): ``project_gaussians``,
``project_gaussians_2d_scale_rot``, ``spherical_harmonics`` and the C != 3
``nd_*`` rasterizers; they are importable and raise NotImplementedError.
"""
from __future__ import annotations

import warnings
from typing import Any

import torch

from .project_gaussians_2d import project_gaussians_2d
from .rasterize import rasterize_gaussians
from .rasterize_sum import rasterize_gaussians_sum
from .utils import (
    bin_and_sort_gaussians,
    compute_cov2d_bounds,
    compute_cumulative_intersects,
    get_tile_bin_edges,
    map_gaussian_to_intersects,
)
from .version import __version__


def _out_of_scope(name):
    def fn(*args, **kwargs):
        raise NotImplementedError(
            f"{name} belongs to the 3DGS / unused parts of gsplat and is out of scope for "
            "gsvc_amd (DESIGN.md §7)")
    fn.__name__ = name
    return fn


project_gaussians = _out_of_scope("project_gaussians")
project_gaussians_2d_scale_rot = _out_of_scope("project_gaussians_2d_scale_rot")
spherical_harmonics = _out_of_scope("spherical_harmonics")


def _deprecated(name, target, new):
    class _Shim(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *args, **kwargs):
            warnings.warn(f"{name} is deprecated, use {new} instead", DeprecationWarning)
            return target(*args, **kwargs)

        @staticmethod
        def backward(ctx: Any, *grad_outputs: Any) -> Any:
            raise NotImplementedError

    _Shim.__name__ = _Shim.__qualname__ = name
    return _Shim


# reference gsplat/gsplat/__init__.py:52-212
MapGaussiansToIntersects = _deprecated("MapGaussiansToIntersects", map_gaussian_to_intersects,
                                       "map_gaussian_to_intersects")
ComputeCumulativeIntersects = _deprecated("ComputeCumulativeIntersects",
                                          compute_cumulative_intersects,
                                          "compute_cumulative_intersects")
ComputeCov2dBounds = _deprecated("ComputeCov2dBounds", compute_cov2d_bounds, "compute_cov2d_bounds")
GetTileBinEdges = _deprecated("GetTileBinEdges", get_tile_bin_edges, "get_tile_bin_edges")
BinAndSortGaussians = _deprecated("BinAndSortGaussians", bin_and_sort_gaussians,
                                  "bin_and_sort_gaussians")
ProjectGaussians = _deprecated("ProjectGaussians", project_gaussians, "project_gaussians")
ProjectGaussians2d = _deprecated("ProjectGaussians2d", project_gaussians_2d, "project_gaussians_2d")
ProjectGaussians2dScaleRot = _deprecated("ProjectGaussians2dScaleRot",
                                         project_gaussians_2d_scale_rot,
                                         "project_gaussians_2d_scale_rot")
RasterizeGaussians = _deprecated("RasterizeGaussians", rasterize_gaussians, "rasterize_gaussians")
RasterizeGaussiansSum = _deprecated("RasterizeGaussiansSum", rasterize_gaussians_sum,
                                    "rasterize_gaussians")
NDRasterizeGaussians = _deprecated("NDRasterizeGaussians", rasterize_gaussians,
                                   "rasterize_gaussians")
SphericalHarmonics = _deprecated("SphericalHarmonics", spherical_harmonics, "spherical_harmonics")

__all__ = [
    "__version__",
    "project_gaussians",
    "project_gaussians_2d",
    "project_gaussians_2d_scale_rot",
    "rasterize_gaussians",
    "rasterize_gaussians_sum",
    "spherical_harmonics",
    # utils
    "bin_and_sort_gaussians",
    "compute_cumulative_intersects",
    "compute_cov2d_bounds",
    "get_tile_bin_edges",
    "map_gaussian_to_intersects",
    # Function.apply() will be deprecated
    "ProjectGaussians",
    "ProjectGaussians2d",
    "ProjectGaussians2dScaleRot",
    "RasterizeGaussians",
    "RasterizeGaussiansSum",
    "BinAndSortGaussians",
    "ComputeCumulativeIntersects",
    "ComputeCov2dBounds",
    "GetTileBinEdges",
    "MapGaussiansToIntersects",
    "SphericalHarmonics",
    "NDRasterizeGaussians",
]
