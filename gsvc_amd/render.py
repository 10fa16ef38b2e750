"""Forward-only frame render: the inference side of GSVC's hot path.

``render_sum_frame`` computes exactly what GSVC's frame forward
(GaussianSplats_Represent.py:83-90) returns --

    xys, depths, radii, conics, nth = project_gaussians_2d(means2d, L, H, W, tb)
    img = rasterize_gaussians_sum(xys, depths, radii, conics, nth, colors, opacity, H, W)
    img = torch.clamp(img, 0, 1).view(-1, H, W, 3).permute(0, 3, 1, 2).contiguous()

-- as four device steps with no host synchronisation: the projection kernel,
the sync-free tile binning (binning.hip, tile_count/scan/fill/segsort), and
the sum rasterizer writing clamp(img) straight into the [1, 3, H, W] planes
(the clamp + permute + contiguous epilogue fused into its store, final_idx not
written since no backward follows).  Results are bit-identical to the
autograd path (tests/test_gpu_parity.py::test_render_frame_matches_op_path).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops as _C
from .utils import bin_for_raster


def render_sum_frame(means2d: Tensor, L_elements: Tensor, colors: Tensor, opacity: Tensor,
                     img_height: int, img_width: int, tile_bounds: Tuple[int, int, int],
                     background: Optional[Tensor] = None, BLOCK_H: int = 16, BLOCK_W: int = 16,
                     clip_thresh: float = 0.01, out: Optional[Tensor] = None) -> Tensor:
    """Render one frame to a clamped [1, 3, H, W] float32 image (no autograd)."""
    if BLOCK_H != 16 or BLOCK_W != 16:
        raise ValueError("only 16x16 tiles are supported (reference config.h:1-2)")
    if colors.dtype == torch.uint8:
        colors = colors.float() / 255
    if colors.dim() != 2:
        raise ValueError("colors must have dimensions (N, D)")
    if colors.shape[-1] != 3:
        raise AttributeError("nd_rasterize_sum_forward: only 3-channel colors are supported")
    if background is None:
        background = torch.ones(3, dtype=torch.float32, device=colors.device)
    H, W = int(img_height), int(img_width)
    n = means2d.shape[-2]
    with torch.no_grad():
        xys, depths, radii, conics, nth = _C.project_gaussians_2d_forward(
            n, means2d.contiguous(), L_elements.contiguous(), H, W, tile_bounds, clip_thresh)
        binned = bin_for_raster(n, xys, depths, radii, nth, tile_bounds)
        if binned.num_intersects is not None and binned.num_intersects < 1:
            img = torch.clamp(background.view(3, 1, 1).expand(3, H, W), 0, 1)
            if out is None:
                return img.reshape(1, 3, H, W).contiguous()
            out.view(3, H, W).copy_(img)
            return out.view(1, 3, H, W)
        img, _ = _C.rasterize_sum_forward_ex(
            tile_bounds, (BLOCK_W, BLOCK_H, 1), (W, H, 1), binned.gaussian_ids_sorted,
            binned.tile_bins, xys, conics, colors.contiguous(), opacity.contiguous(),
            background.contiguous(), num_intersects_dev=binned.m_dev,
            density_hint=binned.density_hint, layout=_C.LAYOUT_CHW_CLAMPED, want_idx=False,
            out=out)
    return img.view(1, 3, H, W)
