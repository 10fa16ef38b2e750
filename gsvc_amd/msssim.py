"""SSIM / MS-SSIM on gfx950 behind pytorch_msssim's API.

GSVC imports ``from pytorch_msssim import ms_ssim, ssim`` for the SSIM-family
losses (utils.py:29-40: 'SSIM', 'Fusion1', 'Fusion2', 'Fusion4',
'Fusion_hinerv') and the per-frame MS-SSIM metric
(train_video_Represent.py:145).  pytorch_msssim is unpinned
(requirements.txt:5) and absent from this image; these functions keep its
published signatures, checks and arithmetic (Gaussian window, valid separable
filtering, C1/C2, per-channel means, the 5-level average-pool pyramid with
relu'd cs / ssim terms) and run them as the kernels of csrc/ssim.hip, forward
and backward, without a host sync.  Parity is against oracle/oracle.py's
float64 restatement and a torch fp32 restatement (tests/test_ssim.py):
"parity unpinned" against the package itself.

CUDA (HIP) tensors only: there is no CPU fallback.  3-D volumes (5-d input)
and custom ``win`` tensors are not provided.
"""
from __future__ import annotations

import ctypes
import warnings
from typing import Optional, Sequence

import torch
from torch import Tensor, nn

from . import _lib as L

_DEFAULT_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)
_raw_stream = torch._C._cuda_getCurrentRawStream


def _check(X: Tensor, Y: Tensor, win_size: int, win) -> tuple:
    if not X.shape == Y.shape:
        raise ValueError(f"Input images should have the same dimensions, but got {X.shape} and "
                         f"{Y.shape}.")
    for d in range(len(X.shape) - 1, 1, -1):
        X = X.squeeze(dim=d)
        Y = Y.squeeze(dim=d)
    if len(X.shape) == 5:
        raise NotImplementedError("gsvc_amd.msssim: 3-D (5-d) inputs are not provided")
    if len(X.shape) != 4:
        raise ValueError(f"Input images should be 4-d or 5-d tensors, but got {X.shape}")
    if not X.type() == Y.type():
        raise ValueError(f"Input images should have the same dtype, but got {X.type()} and "
                         f"{Y.type()}.")
    if win is not None:
        raise NotImplementedError("gsvc_amd.msssim: custom `win` tensors are not provided")
    if not (win_size % 2 == 1):
        raise ValueError("Window size should be odd.")
    if win_size > 11:
        raise NotImplementedError("gsvc_amd.msssim: window sizes above 11 are not provided")
    for i, s in enumerate(X.shape[2:]):
        if s < win_size:
            warnings.warn(f"Skipping Gaussian Smoothing at dimension 2+{i} for input: {X.shape} "
                          f"and win size: {win_size}")
    return X, Y


class _SsimFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, Y, win_size, win_sigma, C1, C2, weights, flags):
        if not (X.is_cuda and Y.is_cuda):
            raise RuntimeError("gsvc_amd.msssim needs CUDA (HIP) tensors; there is no CPU fallback")
        B, C, H, W = X.shape
        Xc = X.detach().float().contiguous()
        Yc = Y.detach().float().contiguous()
        levels = len(weights) if weights else 1
        ws_bytes = L.size("gsvc_ssim_workspace_bytes", B * C, H, W, win_size, levels)
        ws = torch.empty((ws_bytes,), dtype=torch.uint8, device=X.device)
        out = torch.empty((1,) if flags & 1 else (B,), dtype=torch.float32, device=X.device)
        w = (ctypes.c_double * max(levels, 1))(*(weights or [1.0]))
        L.call("gsvc_ssim_forward", B, C, H, W, Xc.data_ptr(), Yc.data_ptr(), win_size,
               float(win_sigma), C1, C2, levels, w if weights else None, flags, out.data_ptr(),
               ws.data_ptr(), ws_bytes, _raw_stream(X.device.index))
        ctx.save_for_backward(Xc, Yc, ws)
        ctx.cfg = (win_size, float(win_sigma), C1, C2, levels, flags)
        ctx.dtypes = (X.dtype, Y.dtype)
        res = out[0] if flags & 1 else out
        return res.to(X.dtype)

    @staticmethod
    def backward(ctx, grad):
        Xc, Yc, ws = ctx.saved_tensors
        win_size, win_sigma, C1, C2, levels, flags = ctx.cfg
        B, C, H, W = Xc.shape
        need_x, need_y = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        g = grad.detach().float().reshape(-1).contiguous()
        dX = torch.empty_like(Xc) if need_x else None
        dY = torch.empty_like(Yc) if need_y else None
        if need_x or need_y:
            sc_bytes = L.size("gsvc_ssim_backward_scratch_bytes", B * C, H, W, win_size, levels)
            scratch = torch.empty((sc_bytes,), dtype=torch.uint8, device=Xc.device)
            L.call("gsvc_ssim_backward", B, C, H, W, Xc.data_ptr(), Yc.data_ptr(), win_size,
                   win_sigma, C1, C2, levels, flags, g.data_ptr(),
                   dX.data_ptr() if need_x else None, dY.data_ptr() if need_y else None,
                   ws.data_ptr(), ws.numel(), scratch.data_ptr(), sc_bytes,
                   _raw_stream(Xc.device.index))
        if dX is not None:
            dX = dX.to(ctx.dtypes[0])
        if dY is not None:
            dY = dY.to(ctx.dtypes[1])
        return dX, dY, None, None, None, None, None, None


def _consts(data_range: float, K: Sequence[float]):
    K1, K2 = K
    return float((K1 * data_range) ** 2), float((K2 * data_range) ** 2)


def ssim(X: Tensor, Y: Tensor, data_range: float = 255, size_average: bool = True,
         win_size: int = 11, win_sigma: float = 1.5, win: Optional[Tensor] = None,
         K: Sequence[float] = (0.01, 0.03), nonnegative_ssim: bool = False) -> Tensor:
    """pytorch_msssim.ssim: the mean SSIM (size_average) or per-image [B]."""
    X, Y = _check(X, Y, win_size, win)
    C1, C2 = _consts(data_range, K)
    flags = (1 if size_average else 0) | (2 if nonnegative_ssim else 0)
    return _SsimFn.apply(X, Y, int(win_size), float(win_sigma), C1, C2, None, flags)


def ms_ssim(X: Tensor, Y: Tensor, data_range: float = 255, size_average: bool = True,
            win_size: int = 11, win_sigma: float = 1.5, win: Optional[Tensor] = None,
            weights: Optional[Sequence[float]] = None,
            K: Sequence[float] = (0.01, 0.03)) -> Tensor:
    """pytorch_msssim.ms_ssim: multi-scale SSIM over len(weights) levels."""
    X, Y = _check(X, Y, win_size, win)
    smaller_side = min(X.shape[-2:])
    assert smaller_side > (win_size - 1) * (2 ** 4), \
        "Image size should be larger than %d due to the 4 downsamplings in ms-ssim" % (
            (win_size - 1) * (2 ** 4))
    if weights is None:
        weights = _DEFAULT_WEIGHTS
    weights = [float(w) for w in (weights.tolist() if isinstance(weights, Tensor) else weights)]
    if not 1 <= len(weights) <= 8:
        raise NotImplementedError("gsvc_amd.msssim: 1 to 8 levels")
    C1, C2 = _consts(data_range, K)
    flags = 1 if size_average else 0
    return _SsimFn.apply(X, Y, int(win_size), float(win_sigma), C1, C2, weights, flags)


class SSIM(nn.Module):
    """pytorch_msssim.SSIM (2-D inputs, channel count free)."""

    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3,
                 spatial_dims=2, K=(0.01, 0.03), nonnegative_ssim=False):
        super().__init__()
        if spatial_dims != 2:
            raise NotImplementedError("gsvc_amd.msssim: 2-D only")
        self.win_size, self.win_sigma = win_size, win_sigma
        self.size_average, self.data_range, self.K = size_average, data_range, K
        self.nonnegative_ssim = nonnegative_ssim

    def forward(self, X, Y):
        return ssim(X, Y, data_range=self.data_range, size_average=self.size_average,
                    win_size=self.win_size, win_sigma=self.win_sigma, K=self.K,
                    nonnegative_ssim=self.nonnegative_ssim)


class MS_SSIM(nn.Module):
    """pytorch_msssim.MS_SSIM (2-D inputs)."""

    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3,
                 spatial_dims=2, weights=None, K=(0.01, 0.03)):
        super().__init__()
        if spatial_dims != 2:
            raise NotImplementedError("gsvc_amd.msssim: 2-D only")
        self.win_size, self.win_sigma = win_size, win_sigma
        self.size_average, self.data_range = size_average, data_range
        self.weights, self.K = weights, K

    def forward(self, X, Y):
        return ms_ssim(X, Y, data_range=self.data_range, size_average=self.size_average,
                       win_size=self.win_size, win_sigma=self.win_sigma, weights=self.weights,
                       K=self.K)
