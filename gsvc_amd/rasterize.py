"""Alpha-compositing rasterizer, same API as gsplat/gsplat/rasterize.py.

``rasterize_gaussians`` (reference :14-86) and ``_RasterizeGaussians``
(reference :89-253): front-to-back compositing with background, the path the
north star names.  Kernels: gsvc_amd/csrc/raster_alpha.hip.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor
from torch.autograd import Function

from . import ops as _C
from .utils import bin_and_sort_for_raster


def rasterize_gaussians(
    xys: Tensor,
    depths: Tensor,
    radii: Tensor,
    conics: Tensor,
    num_tiles_hit: Tensor,
    colors: Tensor,
    opacity: Tensor,
    img_height: int,
    img_width: int,
    BLOCK_H: int = 16,
    BLOCK_W: int = 16,
    background: Optional[Tensor] = None,
    return_alpha: Optional[bool] = False,
):
    """Rasterize 2D gaussians with front-to-back alpha compositing
    (reference forward.cu:252-374).  Differentiable w.r.t. ``xys``,
    ``conics``, ``colors``, ``opacity``.  Returns out_img [H, W, 3]
    (and out_alpha = 1 - final_Ts when ``return_alpha``)."""
    if colors.dtype == torch.uint8:
        colors = colors.float() / 255

    if background is not None:
        assert background.shape[0] == colors.shape[-1], (
            f"incorrect shape of background color tensor, expected shape {colors.shape[-1]}")
    else:
        background = torch.ones(colors.shape[-1], dtype=torch.float32, device=colors.device)

    if xys.ndimension() != 2 or xys.size(1) != 2:
        raise ValueError("xys must have dimensions (N, 2)")

    if colors.ndimension() != 2:
        raise ValueError("colors must have dimensions (N, D)")

    return _RasterizeGaussians.apply(
        xys.contiguous(),
        depths.contiguous(),
        radii.contiguous(),
        conics.contiguous(),
        num_tiles_hit.contiguous(),
        colors.contiguous(),
        opacity.contiguous(),
        img_height,
        img_width,
        BLOCK_H,
        BLOCK_W,
        background.contiguous(),
        return_alpha,
    )


class _RasterizeGaussians(Function):
    """Rasterizes 2D gaussians (reference rasterize.py:89-253)."""

    @staticmethod
    def forward(ctx, xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height,
                img_width, BLOCK_H=16, BLOCK_W=16, background=None, return_alpha=False):
        num_points = xys.size(0)
        BLOCK_X, BLOCK_Y = BLOCK_W, BLOCK_H
        tile_bounds = ((img_width + BLOCK_X - 1) // BLOCK_X, (img_height + BLOCK_Y - 1) // BLOCK_Y, 1)
        block = (BLOCK_X, BLOCK_Y, 1)
        img_size = (img_width, img_height, 1)

        if colors.shape[-1] != 3:
            raise NotImplementedError(
                "nd_rasterize_forward (C != 3) is out of scope for gsvc_amd (see DESIGN.md §7)")

        num_intersects, gaussian_ids_sorted, tile_bins = bin_and_sort_for_raster(
            num_points, xys, depths, radii, num_tiles_hit, tile_bounds)

        if num_intersects < 1:
            out_img = (torch.ones(img_height, img_width, colors.shape[-1], device=xys.device)
                       * background)
            gaussian_ids_sorted = torch.zeros(0, 1, device=xys.device)
            tile_bins = torch.zeros(0, 2, device=xys.device)
            final_Ts = torch.zeros(img_height, img_width, device=xys.device)
            final_idx = torch.zeros(img_height, img_width, device=xys.device)
        else:
            out_img, final_Ts, final_idx = _C.rasterize_forward(
                tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys, conics, colors,
                opacity, background)

        ctx.img_width = img_width
        ctx.img_height = img_height
        ctx.BLOCK_H = BLOCK_H
        ctx.BLOCK_W = BLOCK_W
        ctx.num_intersects = num_intersects
        ctx.save_for_backward(gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity,
                              background, final_Ts, final_idx)

        if return_alpha:
            out_alpha = 1 - final_Ts
            return out_img, out_alpha
        return out_img

    @staticmethod
    def backward(ctx, v_out_img, v_out_alpha=None):
        img_height = ctx.img_height
        img_width = ctx.img_width
        num_intersects = ctx.num_intersects

        if v_out_alpha is None:
            v_out_alpha = torch.zeros_like(v_out_img[..., 0])

        (gaussian_ids_sorted, tile_bins, xys, conics, colors, opacity, background, final_Ts,
         final_idx) = ctx.saved_tensors

        if num_intersects < 1:
            v_xy = torch.zeros_like(xys)
            v_conic = torch.zeros_like(conics)
            v_colors = torch.zeros_like(colors)
            v_opacity = torch.zeros_like(opacity)
        else:
            v_xy, v_conic, v_colors, v_opacity = _C.rasterize_backward(
                img_height, img_width, ctx.BLOCK_H, ctx.BLOCK_W, gaussian_ids_sorted, tile_bins,
                xys, conics, colors, opacity, background, final_Ts, final_idx, v_out_img,
                v_out_alpha)
            v_opacity = v_opacity.reshape(opacity.shape) if opacity.dim() != 2 else v_opacity

        return (v_xy, None, None, v_conic, None, v_colors, v_opacity, None, None, None, None, None,
                None)
