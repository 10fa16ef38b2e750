"""2D projection operator, same API as gsplat/gsplat/project_gaussians_2d.py.

``project_gaussians_2d`` (reference :12-57) and its autograd Function
(reference :59-141) keep the signature, saved tensors and gradient routing of
the reference; the kernels are gsvc_amd/csrc/project2d.hip.  The Function runs
as C++ (csrc/torch_ops.cpp, ProjectFn: one call into the C ABI per forward,
no Python in the backward); ``_ProjectGaussians2d`` below is the same in
Python over ctypes, which the diagnostic library (its A/B knobs) uses.
"""
from __future__ import annotations

from typing import Tuple

from torch import Tensor
from torch.autograd import Function

from . import _lib
from . import ops as _C


def project_gaussians_2d(
    means2d: Tensor,
    L_elements: Tensor,
    img_height: int,
    img_width: int,
    tile_bounds: Tuple[int, int, int],
    clip_thresh: float = 0.01,
):
    """Project 2D Gaussians given by centre (NDC, [-1, 1]) and Cholesky factor
    (l11, l21, l22) to pixel space.

    Differentiable w.r.t. ``means2d`` and ``L_elements``.

    Returns (xys [N,2], depths [N] (zeros), radii [N] int32, conics [N,3],
    num_tiles_hit [N] int32).
    """
    if means2d.device.type == "cpu":  # CPU tensors: the CPU dispatch (gsvc_amd/cpu.py)
        from . import cpu
        return cpu.project_gaussians_2d(means2d, L_elements, img_height, img_width, tile_bounds,
                                        clip_thresh)
    if _lib.product_active():
        tb = tile_bounds
        xys, depths, radii, conics, nth = _lib.torch_ops().project_gaussians_2d(
            means2d, L_elements, int(img_height), int(img_width), int(tb[0]), int(tb[1]),
            int(tb[2]), float(clip_thresh))
        # the 2D projection writes depth 0 for every splat (foward2d.cu:67,122)
        depths._gsvc_zero_version = depths._version
        return xys, depths, radii, conics, nth
    return _ProjectGaussians2d.apply(
        means2d.contiguous(),
        L_elements.contiguous(),
        img_height,
        img_width,
        tile_bounds,
        clip_thresh,
    )


class _ProjectGaussians2d(Function):
    """Project 2D gaussians (reference project_gaussians_2d.py:59-141)."""

    @staticmethod
    def forward(ctx, means2d, L_elements, img_height, img_width, tile_bounds, clip_thresh=0.01):
        num_points = means2d.shape[-2]
        xys, depths, radii, conics, num_tiles_hit = _C.project_gaussians_2d_forward(
            num_points, means2d, L_elements, img_height, img_width, tile_bounds, clip_thresh)
        ctx.img_height = img_height
        ctx.img_width = img_width
        ctx.num_points = num_points
        ctx.save_for_backward(means2d, L_elements, radii, conics)
        ctx.mark_non_differentiable(radii, num_tiles_hit)
        return xys, depths, radii, conics, num_tiles_hit

    @staticmethod
    def backward(ctx, v_xys, v_depths, v_radii, v_conics, v_num_tiles_hit):
        means2d, L_elements, radii, conics = ctx.saved_tensors
        if v_xys is None:
            v_xys = means2d.new_zeros((ctx.num_points, 2))
        if v_conics is None:
            v_conics = means2d.new_zeros((ctx.num_points, 3))
        _v_cov2d, v_mean2d, v_L_elements = _C.project_gaussians_2d_backward(
            ctx.num_points, means2d, L_elements, ctx.img_height, ctx.img_width, radii, conics,
            v_xys, v_depths, v_conics)
        return v_mean2d, v_L_elements, None, None, None, None
