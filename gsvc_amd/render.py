"""Forward-only frame render: the inference side of GSVC's hot path.

``render_frame_sum`` computes exactly what GSVC's frame forward
(GaussianSplats_Represent.py:57-90) returns --

    means2d = tanh(_xyz); L = _cholesky + cholesky_bound; colors = _features_dc * rgb_W
    xys, depths, radii, conics, nth = project_gaussians_2d(means2d, L, H, W, tb)
    img = rasterize_gaussians_sum(xys, depths, radii, conics, nth, colors, ones, H, W)
    img = torch.clamp(img, 0, 1).view(-1, H, W, 3).permute(0, 3, 1, 2).contiguous()

-- in ONE C call (gsvc_render_frame_sum, csrc/frame.hip), two kernels, no host
synchronisation: activations + projection + per-tile 256-slot slabs of splat
ids, then the sum rasterizer sorting each tile's slab in LDS and writing
clamp(img) straight into the [1, 3, H, W] planes (final_idx is not written: no
backward follows).  The workspace (slabs, per-splat records; ~1 KB per tile +
64 B per splat) is cached per device and stream and reused across frames.
Results are bit-identical to the autograd path (tests/test_gpu_sync_free.py).

``render_sum_frame`` is the same for already-activated inputs (means2d, L,
colors, opacity), the signature of the two reference ops it replaces.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib as L
from .utils import _LazyCount


class _FrameWorkspace:
    def __init__(self):
        self.buf = None
        self.hw = None
        self.dirty = True
        self.meta = None
        self.frame = 0
        self.hint = _LazyCount()


_workspaces = {}


def _workspace(dev: torch.device, n: int, H: int, W: int) -> _FrameWorkspace:
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    fw = _workspaces.get(key)
    if fw is None:
        fw = _workspaces[key] = _FrameWorkspace()
        fw.meta = torch.zeros((2,), dtype=torch.int32, device=dev)
    need = L.size("gsvc_render_frame_workspace_bytes", n, H, W)
    if fw.buf is None or fw.buf.numel() < need:
        fw.buf = torch.empty((need,), dtype=torch.uint8, device=dev)
        fw.dirty = True
    if fw.dirty or fw.hw != (H, W):
        # the per-tile counters start at zero; every call leaves them zero
        fw.buf[: L.size("gsvc_render_frame_zeroed_bytes", H, W)].zero_()
        fw.frame = 0
        fw.hw = (H, W)
        fw.dirty = False
    return fw


def _f32c(t: Optional[Tensor], name: str) -> Optional[Tensor]:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    return t.detach().to(torch.float32).contiguous()


def render_frame_sum(xyz: Tensor, cholesky: Tensor, features: Tensor, img_height: int,
                     img_width: int, background: Tensor, xyz_tanh: bool = True,
                     cholesky_bound: Optional[Tensor] = None, rgb_w: Optional[Tensor] = None,
                     opacity: Optional[Tensor] = None) -> Tensor:
    """One frame of GSVC's model to a clamped [1, 3, H, W] image (no autograd).

    xyz [N,2] (tanh applied when ``xyz_tanh``), cholesky [N,3] (+ bound [3]),
    features [N,3] (* rgb_w [N,1]), opacity [N,1] or None for ones.
    """
    H, W = int(img_height), int(img_width)
    n = xyz.shape[0]
    dev = xyz.device
    xyz_c = _f32c(xyz, "xyz")
    chol_c = _f32c(cholesky, "cholesky")
    feat_c = _f32c(features, "features")
    bound_c = _f32c(cholesky_bound, "cholesky_bound")
    rgbw_c = _f32c(rgb_w, "rgb_w")
    opac_c = _f32c(opacity, "opacity")
    bg_c = _f32c(background, "background")
    if xyz_c.shape != (n, 2) or chol_c.shape != (n, 3) or feat_c.shape != (n, 3):
        raise ValueError("xyz [N,2], cholesky [N,3] and features [N,3] expected")
    if bg_c.numel() != 3 or (bound_c is not None and bound_c.numel() != 3):
        raise ValueError("background and cholesky_bound need 3 elements")
    for t, nm in ((rgbw_c, "rgb_w"), (opac_c, "opacity")):
        if t is not None and t.numel() != n:
            raise ValueError(f"{nm} needs N elements")
    fw = _workspace(dev, n, H, W)
    out = torch.empty((1, 3, H, W), dtype=torch.float32, device=dev)
    hint = fw.hint.value
    try:
        L.call("gsvc_render_frame_sum", n, L.ptr(xyz_c), 1 if xyz_tanh else 0, L.ptr(chol_c),
               L.ptr(bound_c), L.ptr(feat_c), L.ptr(rgbw_c), L.ptr(opac_c), L.ptr(bg_c), H, W,
               fw.frame, hint, L.ptr(fw.meta), L.ptr(fw.buf), fw.buf.numel(), L.ptr(out),
               L.stream(dev))
    except Exception:
        fw.dirty = True
        raise
    fw.frame += 1
    fw.hint.update(fw.meta)
    return out


def render_sum_frame(means2d: Tensor, L_elements: Tensor, colors: Tensor, opacity: Tensor,
                     img_height: int, img_width: int, tile_bounds: Tuple[int, int, int],
                     background: Optional[Tensor] = None, BLOCK_H: int = 16, BLOCK_W: int = 16,
                     clip_thresh: float = 0.01) -> Tensor:
    """project_gaussians_2d + rasterize_gaussians_sum + clamp + NCHW for
    activated inputs, as one frame render (no autograd)."""
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
    return render_frame_sum(means2d, L_elements, colors, img_height, img_width, background,
                            xyz_tanh=False, opacity=opacity)
