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
    def __init__(self, stream_handle):
        self.stream = stream_handle
        self.buf = None
        self.buf_ptr = 0
        self.hw = None
        self.dirty = True
        self.meta = None
        self.meta_ptr = 0
        self.frame = 0
        self.hint = _LazyCount()
        self.shape = None
        self.order_for = None  # the splat order (train.order_flags)
        self.order_age = 0


_workspaces = {}
_raw_stream = torch._C._cuda_getCurrentRawStream  # current stream handle, no Stream object


def _workspace(dev: torch.device, n: int, H: int, W: int) -> _FrameWorkspace:
    stream_handle = _raw_stream(dev.index)
    key = (dev.index, stream_handle)
    fw = _workspaces.get(key)
    if fw is None:
        fw = _workspaces[key] = _FrameWorkspace(stream_handle)
        fw.meta = torch.zeros((2,), dtype=torch.int32, device=dev)
        fw.meta_ptr = fw.meta.data_ptr()
    if fw.shape == (n, H, W) and not fw.dirty:
        return fw
    fw.shape = (n, H, W)
    need = L.size("gsvc_render_frame_workspace_bytes", n, H, W)
    if fw.buf is None or fw.buf.numel() < need:
        fw.buf = torch.empty((need,), dtype=torch.uint8, device=dev)
        fw.buf_ptr = fw.buf.data_ptr()
        fw.dirty = True
    if fw.dirty or fw.hw != (H, W):
        # the per-tile counters start at zero; every call leaves them zero
        fw.buf[: L.size("gsvc_render_frame_zeroed_bytes", H, W)].zero_()
        fw.frame = 0
        fw.hw = (H, W)
        fw.dirty = False
        fw.order_for = None
    return fw


_F32 = torch.float32


def _order_flags(fw) -> int:
    from .train import order_flags
    return order_flags(fw)


def _ptr_f32(t: Optional[Tensor], name: str, numel: int, keep: list) -> int:
    """Device address of t as contiguous float32 (a converted copy is kept
    alive in ``keep`` until the launch is enqueued)."""
    if t is None:
        return 0
    if t.dtype is _F32 and t.is_cuda and t.is_contiguous() and t.numel() == numel:
        return t.data_ptr()  # the common case, checked first
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if t.dtype is not torch.float32 or not t.is_contiguous():
        t = t.detach().to(torch.float32).contiguous()
        keep.append(t)
    if t.numel() != numel:
        raise ValueError(f"{name} must have {numel} elements, got {t.numel()}")
    return t.data_ptr()


def _render_frame_fn():
    """gsvc_render_frame_sum_ex of the active library: the frame render with the
    training path's splat order (projection in spatial order, windowed slot
    atomics)."""
    return L.load().gsvc_render_frame_sum_ex


class BoundRender:
    """render_frame_sum bound to one frame model's tensors: the pointer checks
    are done once, so a call costs the workspace lookup, the output
    allocation and the C call.  The owner rebuilds it when a bound tensor
    object or its storage changes (``matches``)."""

    def __init__(self, xyz, cholesky, features, img_height, img_width, background,
                 cholesky_bound=None, rgb_w=None):
        n = xyz.shape[0]
        self.tensors = (xyz, cholesky, features, background, cholesky_bound, rgb_w)
        self.H, self.W, self.n = int(img_height), int(img_width), n
        self.dev = xyz.device
        keep = []
        self.p = (_ptr_f32(xyz, "xyz", 2 * n, keep), _ptr_f32(cholesky, "cholesky", 3 * n, keep),
                  _ptr_f32(features, "features", 3 * n, keep),
                  _ptr_f32(background, "background", 3, keep),
                  _ptr_f32(cholesky_bound, "cholesky_bound", 3, keep), _ptr_f32(rgb_w, "rgb_w", n, keep))
        if keep:  # a converted copy would go stale: bind only tensors used in place
            raise ValueError("BoundRender needs contiguous float32 CUDA tensors")
        self.lib = L.load()
        self.fn = self.lib.gsvc_render_frame_sum_ex

    def matches(self, tensors) -> bool:
        return (len(tensors) == len(self.tensors)
                and all(a is b for a, b in zip(tensors, self.tensors))
                and all(t is None or t.data_ptr() == p for t, p in zip(tensors, self.p)))

    def __call__(self) -> Tensor:
        H, W, n = self.H, self.W, self.n
        fw = _workspace(self.dev, n, H, W)
        out = torch.empty((1, 3, H, W), dtype=_F32, device=self.dev)
        p = self.p
        rc = self.fn(n, p[0], 1, p[1], p[4], p[2], p[5], 0, p[3], H, W, fw.frame, fw.hint.value,
                     fw.meta_ptr, fw.buf_ptr, fw.buf.numel(), out.data_ptr(), fw.stream,
                     _order_flags(fw))
        if rc != 0:
            fw.dirty = True
            msg = self.lib.gsvc_last_error().decode(errors="replace")
            raise RuntimeError(f"gsvc_render_frame_sum failed (status {rc}): {msg}")
        fw.frame += 1
        fw.hint.update(fw.meta)
        return out


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
    keep = []
    p_xyz = _ptr_f32(xyz, "xyz", 2 * n, keep)
    p_chol = _ptr_f32(cholesky, "cholesky", 3 * n, keep)
    p_feat = _ptr_f32(features, "features", 3 * n, keep)
    p_bound = _ptr_f32(cholesky_bound, "cholesky_bound", 3, keep)
    p_rgbw = _ptr_f32(rgb_w, "rgb_w", n, keep)
    p_opac = _ptr_f32(opacity, "opacity", n, keep)
    p_bg = _ptr_f32(background, "background", 3, keep)
    fw = _workspace(dev, n, H, W)
    out = torch.empty((1, 3, H, W), dtype=torch.float32, device=dev)
    rc = _render_frame_fn()(
        n, p_xyz, 1 if xyz_tanh else 0, p_chol, p_bound, p_feat, p_rgbw, p_opac, p_bg, H, W,
        fw.frame, fw.hint.value, fw.meta_ptr, fw.buf_ptr, fw.buf.numel(), out.data_ptr(),
        fw.stream, _order_flags(fw))
    if rc != 0:
        fw.dirty = True
        msg = L.load().gsvc_last_error().decode(errors="replace")
        raise RuntimeError(f"gsvc_render_frame_sum failed (status {rc}): {msg}")
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


class _BatchWorkspace:
    def __init__(self):
        self.buf = None
        self.key = None
        self.call = 0
        self.meta = None
        self.offs = None
        self.offs_host = None
        # total M of a recent call for the kernel choice: meta [F, 2] copied to
        # pinned memory without a sync every 16 calls (stale values only cost speed)
        self.hint = 0
        self.pinned = None
        self.event = None

    def update_hint(self):
        if self.event is not None and self.event.query():
            self.hint = int(self.pinned[:, 0].sum())
            self.event = None
        if self.event is None and self.call % 16 == 1:
            if self.pinned is None or self.pinned.shape != self.meta.shape:
                self.pinned = torch.empty(self.meta.shape, dtype=torch.int32, pin_memory=True)
            self.pinned.copy_(self.meta, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record()


_batch_workspaces = {}


def render_frames_sum(xyz: Tensor, cholesky: Tensor, features: Tensor, frame_sizes,
                      img_height: int, img_width: int, background: Tensor, xyz_tanh: bool = True,
                      cholesky_bound: Optional[Tensor] = None, rgb_w: Optional[Tensor] = None,
                      opacity: Optional[Tensor] = None) -> Tensor:
    """Render a batch of frame models of one video in one call (two kernels
    over all frames; gsvc_render_frames_sum): the inputs are the frames'
    splats concatenated (frame b has ``frame_sizes[b]`` of them, in order),
    the output [F, 3, H, W] -- each image bit-identical to
    ``render_frame_sum`` of that frame alone.  A video decoder's GOP: GSVC
    stores one model per frame (train_video_Represent.py:379-384)."""
    import ctypes
    H, W = int(img_height), int(img_width)
    sizes = [int(x) for x in frame_sizes]
    F = len(sizes)
    if F < 1 or any(x < 0 for x in sizes):
        raise ValueError("frame_sizes must be a non-empty list of non-negative counts")
    n = xyz.shape[0]
    if sum(sizes) != n:
        raise ValueError(f"frame_sizes sum to {sum(sizes)}, inputs have {n} splats")
    dev = xyz.device
    keep = []
    p_xyz = _ptr_f32(xyz, "xyz", 2 * n, keep)
    p_chol = _ptr_f32(cholesky, "cholesky", 3 * n, keep)
    p_feat = _ptr_f32(features, "features", 3 * n, keep)
    p_bound = _ptr_f32(cholesky_bound, "cholesky_bound", 3, keep)
    p_rgbw = _ptr_f32(rgb_w, "rgb_w", n, keep)
    p_opac = _ptr_f32(opacity, "opacity", n, keep)
    p_bg = _ptr_f32(background, "background", 3, keep)
    stream_handle = torch.cuda.current_stream(dev).cuda_stream
    key = (dev.index, stream_handle)
    bw = _batch_workspaces.get(key)
    if bw is None:
        bw = _batch_workspaces[key] = _BatchWorkspace()
    need = L.size("gsvc_render_frames_workspace_bytes", F, n, H, W)
    if bw.buf is None or bw.buf.numel() < need or bw.key != (F, H, W):
        if bw.buf is None or bw.buf.numel() < need:
            bw.buf = torch.empty((need,), dtype=torch.uint8, device=dev)
        bw.buf[: L.size("gsvc_render_frames_zeroed_bytes", F, H, W)].zero_()
        bw.meta = torch.zeros((F, 2), dtype=torch.int32, device=dev)
        bw.key = (F, H, W)
        bw.call = 0
        bw.offs_host = None
        bw.hint, bw.event, bw.pinned = 0, None, None
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    if bw.offs_host is None or list(bw.offs_host) != offs:
        bw.offs_host = (ctypes.c_int * (F + 1))(*offs)
        bw.offs = torch.tensor(offs, dtype=torch.int32, device=dev)
    out = torch.empty((F, 3, H, W), dtype=torch.float32, device=dev)
    rc = L.load().gsvc_render_frames_sum(
        F, bw.offs_host, bw.offs.data_ptr(), p_xyz, 1 if xyz_tanh else 0, p_chol, p_bound, p_feat,
        p_rgbw, p_opac, p_bg, H, W, bw.call, bw.hint, bw.meta.data_ptr(), bw.buf.data_ptr(),
        bw.buf.numel(), out.data_ptr(), stream_handle)
    if rc != 0:
        bw.key = None
        msg = L.load().gsvc_last_error().decode(errors="replace")
        raise RuntimeError(f"gsvc_render_frames_sum failed (status {rc}): {msg}")
    bw.call += 1
    bw.update_hint()
    return out
