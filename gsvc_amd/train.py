"""Fused training iteration of GSVC's per-frame model (one C call, no host sync).

``train_step_sum`` runs what ``GaussianVideo_frame.train_iter``
(GaussianSplats_Represent.py:191-207) does between ``forward()`` and
``scheduler.step()`` for the L2 / L1 losses and Adan -- forward, clamp, loss,
backward through the rasterizer, the projection and the activations, and the
Adan update of every parameter -- as three gfx950 kernels
(gsvc_amd/csrc/train.hip, ``gsvc_train_step_sum``).  ``GaussianVideoFrame``
(frame.py) takes this path on the iterations where the reference would not
prune or densify; it keeps the optimizer's state tensors, step counter and
learning rate, so fused and op-by-op iterations interleave freely.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch
from torch import Tensor

from . import _lib as L

LOSS_KIND = {"L2": 0, "L1": 1}


class _TrainWorkspace:
    def __init__(self):
        self.buf = None
        self.buf_ptr = 0
        self.hw = None
        self.dirty = True
        self.frame = 0
        self.shape = None


_workspaces = {}
_raw_stream = torch._C._cuda_getCurrentRawStream  # current stream handle, no Stream object


def _workspace(dev: torch.device, n: int, H: int, W: int) -> _TrainWorkspace:
    key = (dev.index, _raw_stream(dev.index))
    ws = _workspaces.get(key)
    if ws is None:
        ws = _workspaces[key] = _TrainWorkspace()
    if ws.shape == (n, H, W) and not ws.dirty:
        return ws
    ws.shape = (n, H, W)
    need = L.size("gsvc_train_step_workspace_bytes", n, H, W)
    if ws.buf is None or ws.buf.numel() < need:
        ws.buf = torch.empty((need,), dtype=torch.uint8, device=dev)
        ws.buf_ptr = ws.buf.data_ptr()
        ws.dirty = True
    if ws.dirty or ws.hw != (H, W):
        # per-tile counters and M slots start at zero; every call leaves them zero
        ws.buf[: L.size("gsvc_render_frame_zeroed_bytes", H, W)].zero_()
        ws.frame = 0
        ws.hw = (H, W)
        ws.dirty = False
    return ws


def _f32_ptr(t: Optional[Tensor], name: str, numel: int) -> int:
    if t is None:
        return 0
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if t.dtype is not torch.float32 or not t.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous float32 tensor")
    if t.numel() != numel:
        raise ValueError(f"{name} must have {numel} elements, got {t.numel()}")
    return t.data_ptr()


class BoundStep:
    """A fused training step bound to fixed tensors (parameters, Adan state,
    constants): pointers and the ctypes state array are built once, so a call
    costs one C call plus the loss tensor.  The owner rebuilds it when any
    bound tensor object changes (``matches``).  Parameters are updated in place
    through their storage (as ``p.data`` would be)."""

    def __init__(self, xyz, cholesky, features, rgb_w, rgb_w_trainable, cholesky_bound,
                 background, H, W, loss_type, adan_state):
        n = xyz.shape[0]
        self.tensors = (xyz, cholesky, features, rgb_w, cholesky_bound, background, *adan_state)
        self.ids = tuple(map(id, self.tensors))  # the objects stay alive via self.tensors
        self.n, self.H, self.W = n, int(H), int(W)
        self.dev = xyz.device
        self.kind = LOSS_KIND[loss_type]
        self.rgbw_train = 1 if rgb_w_trainable else 0
        self.p = [_f32_ptr(xyz, "xyz", 2 * n), _f32_ptr(cholesky, "cholesky", 3 * n),
                  _f32_ptr(cholesky_bound, "cholesky_bound", 3), _f32_ptr(features, "features", 3 * n),
                  _f32_ptr(rgb_w, "rgb_w", n), _f32_ptr(background, "background", 3)]
        self.state = (ctypes.c_void_p * 16)()
        numels = [2 * n, 3 * n, 3 * n, n]
        for k, t in enumerate(adan_state):
            self.state[k] = _f32_ptr(t, "adan_state", numels[k // 4]) or None
        # the storage pointers ``matches`` re-checks (parameters, constants, state)
        self.ptrs = tuple(None if t is None else t.data_ptr() for t in self.tensors)
        self.hp = (ctypes.c_double * 10)()
        self.fn = L.load().gsvc_train_step_sum
        self.host = None
        self.stream = None

    def matches(self, tensors) -> bool:
        # identity, plus every bound tensor's storage (Module.to, ``p.data = ...``,
        # ``state[k].data = ...`` or ``set_`` swap it under the same object)
        if tuple(map(id, tensors)) != self.ids:
            return False
        return all((t is None and q is None) or (t is not None and t.data_ptr() == q)
                   for t, q in zip(tensors, self.ptrs))

    def launch(self, gt: Tensor, adan_hparams, adan_flags: int) -> None:
        """Enqueue one fused step on the current stream.  The step's kernel
        writes the losses straight into a pinned host buffer (no copy kernel,
        no device tensor); ``result`` waits for them."""
        if not (gt.is_cuda and gt.dtype is torch.float32 and gt.is_contiguous()
                and gt.numel() == 3 * self.H * self.W):
            raise RuntimeError("gt must be a contiguous float32 CUDA tensor of 3*H*W elements")
        for k, x in enumerate(adan_hparams):
            self.hp[k] = x
        ws = _workspace(self.dev, self.n, self.H, self.W)
        if self.host is None:
            self.host = torch.zeros((4,), dtype=torch.float32, pin_memory=True)
            self.host_np = self.host.numpy()
        p = self.p
        self.stream = _raw_stream(self.dev.index)
        rc = self.fn(self.n, p[0], p[1], p[2], p[3], p[4], self.rgbw_train, p[5], gt.data_ptr(),
                     self.H, self.W, self.kind, ws.frame, self.state, self.hp, int(adan_flags),
                     self.host.data_ptr(), None, None, ws.buf_ptr, ws.buf.numel(), self.stream)
        if rc != 0:
            ws.dirty = True
            msg = L.load().gsvc_last_error().decode(errors="replace")
            raise RuntimeError(f"gsvc_train_step_sum failed (status {rc}): {msg}")
        ws.frame += 1

    def result(self):
        """(mean squared error, mean absolute error) of the last launched step:
        waits for the stream (the reference's PSNR ``.item()``)."""
        L.call("gsvc_stream_sync", self.stream)
        return float(self.host_np[0]), float(self.host_np[1])


def train_step_sum(xyz: Tensor, cholesky: Tensor, features: Tensor, rgb_w: Optional[Tensor],
                   rgb_w_trainable: bool, cholesky_bound: Optional[Tensor], background: Tensor,
                   gt: Tensor, img_height: int, img_width: int, loss_type: str = "L2",
                   adan_state: Sequence[Optional[Tensor]] = (), adan_hparams: Sequence[float] = (),
                   adan_flags: int = 0, render_out: Optional[Tensor] = None,
                   grads_out: Optional[Tensor] = None) -> Tensor:
    """One fused training step; returns a device tensor [2] = (mean squared
    error, mean absolute error) of clamp(render) against ``gt``.

    Parameters are updated in place (xyz [N,2], cholesky [N,3], features
    [N,3], and rgb_w [N,1] when ``rgb_w_trainable``) with Adan; ``adan_state``
    lists per parameter its exp_avg, exp_avg_sq, exp_avg_diff, neg_pre_grad
    (16 entries; rgb_w's may be None).  With ``grads_out`` [N,9] nothing is
    updated and the parameter gradients are written there instead.
    """
    H, W = int(img_height), int(img_width)
    if loss_type not in LOSS_KIND:
        raise ValueError(f"fused training supports the L2 and L1 losses, not {loss_type!r}")
    n = xyz.shape[0]
    dev = xyz.device
    p_xyz = _f32_ptr(xyz, "xyz", 2 * n)
    p_chol = _f32_ptr(cholesky, "cholesky", 3 * n)
    p_feat = _f32_ptr(features, "features", 3 * n)
    p_rgbw = _f32_ptr(rgb_w, "rgb_w", n)
    p_bound = _f32_ptr(cholesky_bound, "cholesky_bound", 3)
    p_bg = _f32_ptr(background, "background", 3)
    p_gt = _f32_ptr(gt, "gt", 3 * H * W)
    p_render = _f32_ptr(render_out, "render_out", 3 * H * W)
    p_grads = _f32_ptr(grads_out, "grads_out", 9 * n)
    state = (ctypes.c_void_p * 16)()
    if grads_out is None:
        if len(adan_state) != 16 or len(adan_hparams) != 10:
            raise ValueError("adan_state needs 16 tensors and adan_hparams 10 values")
        numels = [2 * n, 3 * n, 3 * n, n]
        for k, t in enumerate(adan_state):
            state[k] = _f32_ptr(t, "adan_state", numels[k // 4]) or None
    hp = (ctypes.c_double * 10)(*[float(x) for x in (list(adan_hparams) or [0.0] * 10)])
    ws = _workspace(dev, n, H, W)
    loss = torch.empty((2,), dtype=torch.float32, device=dev)
    rc = L.load().gsvc_train_step_sum(
        n, p_xyz, p_chol, p_bound, p_feat, p_rgbw, 1 if rgb_w_trainable else 0, p_bg, p_gt, H, W,
        LOSS_KIND[loss_type], ws.frame, state, hp, int(adan_flags), loss.data_ptr(), p_render,
        p_grads, ws.buf_ptr, ws.buf.numel(), _raw_stream(dev.index))
    if rc != 0:
        ws.dirty = True
        msg = L.load().gsvc_last_error().decode(errors="replace")
        raise RuntimeError(f"gsvc_train_step_sum failed (status {rc}): {msg}")
    ws.frame += 1
    return loss
