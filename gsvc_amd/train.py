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
import warnings
import weakref
from typing import Optional, Sequence

import torch
from torch import Tensor

from . import _lib as L

LOSS_KIND = {"L2": 0, "L1": 1}
TRAIN_LOSS_SEQ = 0x100  # include/gsvc_amd.h GSVC_TRAIN_LOSS_SEQ
TRAIN_ORDER = 0x200  # GSVC_TRAIN_ORDER
TRAIN_ORDER_REFRESH = 0x400  # GSVC_TRAIN_ORDER_REFRESH
ORDER_REFRESH_EVERY = 64  # fused steps between splat-order sorts (0: no order)
TRAIN_PROJECT_ONLY = 0x800  # GSVC_TRAIN_PROJECT_ONLY
TRAIN_PROJECTED = 0x1000  # GSVC_TRAIN_PROJECTED
TRAIN_PROJECT_NEXT = 0x2000  # GSVC_TRAIN_PROJECT_NEXT
TRAIN_DETERMINISTIC = 0x4000  # GSVC_TRAIN_DETERMINISTIC
DET_CAPACITY_PER_SPLAT = 8  # first det_capacity guess: M / N is ~2.5 at init, ~5 trained
PROJECT_AHEAD = True  # a bound step leaves the next step's frame projected behind itself
TRAIN_CARRY = 0x8000  # GSVC_TRAIN_CARRY
# Carried bins (GSVC_TRAIN_CARRY): a bound step's splat kernel projects the next
# frame itself and keeps the tile bins from step to step (at trained density
# ~160 of 50k splats change tile box per step, tools/bin_drift.py), so no
# projection kernel runs between steps; a projection rebuilds them every
# CARRY_REBUILD_EVERY steps (the bins only grow) and whenever PROJECT_AHEAD's
# checks fail.  False: the projection of the next frame is enqueued instead
# (GSVC_TRAIN_PROJECT_NEXT).
CARRY_BINS = True
CARRY_REBUILD_EVERY = 64
# Tile kernel ahead (GSVC_TRAIN_TILES_NEXT / GSVC_TRAIN_TILED, with the carried
# bins): a bound step also enqueues the NEXT iteration's tile kernel (forward,
# loss, backward: it depends on the parameters this step leaves and on gt, not
# on the next call's hyper-parameters) against this call's target, so the GPU
# goes on while the host returns the loss and makes the next call; that call
# then launches only the splat kernel (Adan with its own hyper-parameters).
# Used only when the next call passes the same target (same storage, no
# in-place change) and nothing touched the parameters (PROJECT_AHEAD's checks);
# otherwise the pending work is discarded by a rebuild.  Enqueued only when
# this call's target is the previous call's (a caller that alternates targets
# would discard every time).
TILES_AHEAD = True
TRAIN_TILES_NEXT = 0x10000  # GSVC_TRAIN_TILES_NEXT
TRAIN_TILED = 0x20000  # GSVC_TRAIN_TILED
TRAIN_REBUILD_NEXT = 0x40000  # GSVC_TRAIN_REBUILD_NEXT

# A step's projection of the NEXT frame is used only if nothing could have
# changed the parameters since: no other fused launch on the same parameters
# (_param_launches, keyed by the xyz storage: another model's launches on
# another stream no longer void it), no optimizer step or control of ours
# (_param_epoch, bump_param_epoch), no in-place op through the bound Parameters
# (their _version), the same bound step and workspace frame (a launch of any
# model on the same workspace advances its frame).  (In-place writes through
# ``.data`` bypass _version; call bump_param_epoch() after such writes.)
_param_launches = {}
_param_epoch = [0]


def _note_launch(xyz_ptr: int) -> int:
    n = _param_launches.get(xyz_ptr, 0) + 1
    _param_launches[xyz_ptr] = n
    return n


def bump_param_epoch() -> None:
    """Parameters or a training target changed outside the fused step:
    discard any projection or tile kernel a bound step enqueued ahead.

    The fused step reuses work it enqueued ahead only while the bound
    parameters and the target keep their storage and ``_version``; torch bumps
    ``_version`` on every in-place op.  A write that bypasses it -- through
    ``.data``, DLPack / CuPy views or a custom kernel -- must be followed by
    this call, or the next step may use gradients of the old values."""
    _param_epoch[0] += 1


class _TrainWorkspace:
    def __init__(self):
        self.buf = None
        self.buf_ptr = 0
        self.hw = None
        self.dirty = True
        self.frame = 0
        self.shape = None
        self.order_for = None  # (n, H, W) the workspace's splat order was sorted for
        self.order_age = 0     # steps since it was sorted
        self.pending = None    # the projection a bound step enqueued ahead (BoundStep.launch):
        #                        (weakref to the step, frame, launch count, epoch, versions,
        #                        tiles: None or (gt, gt version, background version, det
        #                        mode + workspace + capacity) of the tile kernel enqueued
        #                        ahead -- gt held so its storage stays alive and unreused
        #                        while that kernel may read it)
        self.det_buf = None    # GSVC_TRAIN_DETERMINISTIC workspace
        self.det_cap = 0
        self.carry_age = 0     # steps since the carried bins were rebuilt

    def det_workspace(self, dev: torch.device, n: int, pairs: int = 0):
        """The deterministic mode's slot buffer for n splats, with room for at
        least ``pairs`` (splat, tile) pairs (grown by half again when short)."""
        cap = max(self.det_cap, DET_CAPACITY_PER_SPLAT * n)
        if pairs > cap:
            cap = pairs + pairs // 2
        need = L.size("gsvc_train_step_det_workspace_bytes", n, cap)
        if self.det_buf is None or self.det_buf.numel() < need or cap != self.det_cap:
            self.det_buf = torch.empty((need,), dtype=torch.uint8, device=dev)
            self.det_cap = cap
        return self.det_buf, cap

    def order_flags(self) -> int:
        return order_flags(self)


def order_flags(ws) -> int:
    """For a workspace ``ws`` with ``shape`` (n, H, W), ``order_for`` and
    ``order_age``: GSVC_TRAIN_ORDER when it holds a valid order (sorted for the
    same n and image size), GSVC_TRAIN_ORDER_REFRESH every ORDER_REFRESH_EVERY
    calls (splats drift; a stale order costs speed only: any permutation of
    the splats gives the same results)."""
    if ORDER_REFRESH_EVERY <= 0:
        return 0
    flags = 0
    if ws.order_for == ws.shape:
        flags |= TRAIN_ORDER
        ws.order_age += 1
    if ws.order_for != ws.shape or ws.order_age >= ORDER_REFRESH_EVERY:
        flags |= TRAIN_ORDER_REFRESH
        ws.order_for = ws.shape
        ws.order_age = 0
    return flags


_workspaces = {}
_data_ptr = torch.Tensor.data_ptr


def _dropped_step(ws):
    """Weakref callback: the bound step whose work is pending in ``ws`` is gone
    (its model was freed) -- release what the pending entry holds (the target)
    and start the workspace's next user from zeroed counters."""
    def cb(ref):
        pend = ws.pending
        if pend is not None and pend[0] is ref:
            ws.pending = None
            ws.dirty = True
    return cb
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
        # per-tile counters and M slots start at zero; every call leaves them zero.
        # The frame counter keeps counting (it also numbers the loss read-backs).
        ws.buf[: L.size("gsvc_render_frame_zeroed_bytes", H, W)].zero_()
        ws.hw = (H, W)
        ws.dirty = False
        ws.order_for = None
        ws.pending = None
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


class _StepArgs(ctypes.Structure):
    """include/gsvc_amd.h gsvc_train_step_args."""
    _fields_ = [("num_points", ctypes.c_int), ("xyz", ctypes.c_void_p),
                ("cholesky", ctypes.c_void_p), ("cholesky_bound", ctypes.c_void_p),
                ("features", ctypes.c_void_p), ("rgb_w", ctypes.c_void_p),
                ("rgb_w_trainable", ctypes.c_int), ("background", ctypes.c_void_p),
                ("gt", ctypes.c_void_p), ("img_height", ctypes.c_uint), ("img_width", ctypes.c_uint),
                ("loss_kind", ctypes.c_int), ("frame_index", ctypes.c_int),
                ("adan_state", ctypes.c_void_p), ("adan_hparams", ctypes.c_void_p),
                ("adan_flags", ctypes.c_int), ("loss", ctypes.c_void_p),
                ("render_out", ctypes.c_void_p), ("grads_out", ctypes.c_void_p),
                ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_size_t),
                ("stream", ctypes.c_void_p), ("det_workspace", ctypes.c_void_p),
                ("det_workspace_bytes", ctypes.c_size_t), ("det_capacity", ctypes.c_longlong)]


class BoundStep:
    """A fused training step bound to fixed tensors (parameters, Adan state,
    constants): the C argument struct is built once and a call updates only
    the target, frame, flags, hyper-parameters and stream, so a step costs
    one single-pointer C call.  The owner rebuilds it when any bound tensor
    object or storage changes (``matches``).  Parameters are updated in place
    through their storage (as ``p.data`` would be)."""

    def __init__(self, xyz, cholesky, features, rgb_w, rgb_w_trainable, cholesky_bound,
                 background, H, W, loss_type, adan_state):
        n = xyz.shape[0]
        self.tensors = (xyz, cholesky, features, rgb_w, cholesky_bound, background, *adan_state)
        self.ids = tuple(map(id, self.tensors))  # the objects stay alive via self.tensors
        self.n, self.H, self.W = n, int(H), int(W)
        self.dev = xyz.device
        self.rgbw_train = 1 if rgb_w_trainable else 0
        self.state = (ctypes.c_void_p * 16)()
        numels = [2 * n, 3 * n, 3 * n, n]
        for k, t in enumerate(adan_state):
            self.state[k] = _f32_ptr(t, "adan_state", numels[k // 4]) or None
        # the storage pointers ``matches`` re-checks (parameters, constants, state)
        self.live = [k for k, t in enumerate(self.tensors) if t is not None]
        self.live_tensors = [self.tensors[k] for k in self.live]
        self.ptrs = list(map(_data_ptr, self.live_tensors))
        self.hp = (ctypes.c_double * 10)()
        a = self.args = _StepArgs()
        a.num_points = n
        a.xyz = _f32_ptr(xyz, "xyz", 2 * n)
        a.cholesky = _f32_ptr(cholesky, "cholesky", 3 * n)
        a.cholesky_bound = _f32_ptr(cholesky_bound, "cholesky_bound", 3)
        a.features = _f32_ptr(features, "features", 3 * n)
        a.rgb_w = _f32_ptr(rgb_w, "rgb_w", n)
        a.rgb_w_trainable = self.rgbw_train
        a.background = _f32_ptr(background, "background", 3)
        a.img_height, a.img_width = self.H, self.W
        a.loss_kind = LOSS_KIND[loss_type]
        a.adan_state = ctypes.addressof(self.state)
        a.adan_hparams = ctypes.addressof(self.hp)
        self.args_ref = ctypes.byref(a)
        self.lib = L.load()  # bound once: the library of every call of this step
        self.fn = self.lib.gsvc_train_step_sum_args
        self.host = None  # coherent host words: mse, l1, sequence, (det) pairs
        self.seq = 0
        self.stream = None
        self.det = False        # this step runs GSVC_TRAIN_DETERMINISTIC
        self.det_pairs = 0      # the (splat, tile) pairs its last det step reported
        self.det_overflows = 0  # det steps whose capacity was short (those fell back to atomics)
        self.ahead_steps = 0    # steps that used the projection the previous step enqueued
        self.tiled_steps = 0    # steps whose tile kernel the previous step enqueued
        self.last_gt = None     # (data_ptr, version) of the previous launch's target
        self.params = tuple(t for t in (xyz, cholesky, features, rgb_w) if t is not None)
        self.background = background

    def __del__(self):
        if getattr(self, "host", None) is not None:
            try:
                self.lib.gsvc_host_free(self.host)
            except Exception:  # interpreter shutdown
                pass
            self.host = None

    def matches(self, tensors) -> bool:
        # identity, plus every bound tensor's storage (Module.to, ``p.data = ...``,
        # ``state[k].data = ...`` or ``set_`` swap it under the same object)
        if tuple(map(id, tensors)) != self.ids:
            return False
        # (the same objects as self.tensors: their storages now)
        return list(map(_data_ptr, self.live_tensors)) == self.ptrs

    def launch(self, gt: Tensor, adan_hparams, adan_flags: int) -> None:
        """Enqueue one fused step on the current stream.  The step's last
        kernel stores the losses straight into coherent host memory, then a
        sequence word (GSVC_TRAIN_LOSS_SEQ); ``result`` waits for that word
        only, so the host goes on while the parameter update still runs --
        everything later on the stream is ordered after it, as for any
        asynchronous torch op."""
        if not (gt.is_cuda and gt.dtype is torch.float32 and gt.is_contiguous()
                and gt.numel() == 3 * self.H * self.W):
            raise RuntimeError("gt must be a contiguous float32 CUDA tensor of 3*H*W elements")
        hp = self.hp
        for k, x in enumerate(adan_hparams):
            hp[k] = x
        ws = _workspace(self.dev, self.n, self.H, self.W)
        lib = self.lib
        a = self.args
        if self.host is None:
            self.host = lib.gsvc_host_alloc(16)
            if not self.host:
                raise RuntimeError(lib.gsvc_last_error().decode(errors="replace"))
            self.host_f = (ctypes.c_float * 4).from_address(self.host)
            self.host_u = (ctypes.c_uint * 4).from_address(self.host)
            a.loss = self.host
        # a stale sequence word must not satisfy this step's wait (a workspace on
        # another stream counts its frames from 0 again)
        self.host_u[2] = 0
        self.stream = _raw_stream(self.dev.index)
        flags = int(adan_flags) | TRAIN_LOSS_SEQ
        # torch.use_deterministic_algorithms(True): bitwise reproducible gradients
        self.det = torch.are_deterministic_algorithms_enabled()
        if self.det:
            buf, cap = ws.det_workspace(self.dev, self.n, self.det_pairs)
            a.det_workspace, a.det_workspace_bytes, a.det_capacity = buf.data_ptr(), buf.numel(), cap
            flags |= TRAIN_DETERMINISTIC
            adan_flags = int(adan_flags) | TRAIN_DETERMINISTIC
        else:
            a.det_workspace, a.det_workspace_bytes, a.det_capacity = None, 0, 0
        tiles = None
        order = 0  # the order flags of a REBUILD_NEXT projection
        if PROJECT_AHEAD:
            versions = tuple(t._version for t in self.params)
            pend = ws.pending
            ahead = (pend is not None and pend[0]() is self and pend[1] == ws.frame
                     and pend[2] == _param_launches.get(a.xyz, 0) and pend[3] == _param_epoch[0]
                     and pend[4] == versions)
            tiled = False
            if ahead and pend[5] is not None:
                # this frame's tile kernel ran against the previous call's target
                # and background: usable only if they are this call's, unchanged
                pgt, pver, pbg, pdet = pend[5]
                tiled = (pgt.data_ptr() == gt.data_ptr() and gt._version == pver
                         and pgt._version == pver and self.background._version == pbg
                         and pdet == (self.det, a.det_workspace, a.det_capacity))
                ahead = tiled  # else its gradient sums are in the records: rebuild
            if pend is not None and not ahead:
                # an enqueued projection that cannot be used: its counts are in
                # the workspace -- start from zeroed counters
                ws.dirty = True
                ws = _workspace(self.dev, self.n, self.H, self.W)
            carry = TRAIN_CARRY if CARRY_BINS else 0
            if not ahead or (carry and ws.carry_age >= CARRY_REBUILD_EVERY):
                # (a step that enqueued its successor's tiles never leaves a rebuild due)
                self._call(ws, lib, gt, int(adan_flags) | TRAIN_PROJECT_ONLY | carry | ws.order_flags())
                ws.carry_age = 0
                tiled = False
            if ahead:
                self.ahead_steps += 1
            ws.carry_age += 1
            flags |= TRAIN_PROJECTED | (carry or TRAIN_PROJECT_NEXT)
            if tiled:
                flags |= TRAIN_TILED
                self.tiled_steps += 1
            gkey = (gt.data_ptr(), gt._version)
            if TILES_AHEAD and carry and gkey == self.last_gt:
                flags |= TRAIN_TILES_NEXT
                # (deterministic mode: the next call must keep this det workspace)
                tiles = (gt, gt._version, self.background._version,
                         (self.det, a.det_workspace, a.det_capacity))
                if ws.carry_age >= CARRY_REBUILD_EVERY:
                    # the next frame's bins are rebuilt behind this step, not at
                    # the start of the next call
                    flags |= TRAIN_REBUILD_NEXT
                    order = ws.order_flags()
                    ws.carry_age = 0
            self.last_gt = gkey
        self.seq = ((ws.frame + 1) & 0xFFFFFFFF) | 0x80000000
        # the order flags go with a projection (PROJECT_NEXT's, REBUILD_NEXT's or
        # the call's own)
        self._call(ws, lib, gt, flags | (order if flags & TRAIN_CARRY else ws.order_flags()))
        launches = _note_launch(a.xyz)
        if PROJECT_AHEAD:
            ws.pending = (weakref.ref(self, _dropped_step(ws)), ws.frame + 1, launches,
                          _param_epoch[0], versions, tiles)
        ws.frame += 1

    def _call(self, ws, lib, gt, flags):
        a = self.args
        a.gt = gt.data_ptr()
        a.frame_index = ws.frame
        a.adan_flags = flags
        a.workspace = ws.buf_ptr
        a.workspace_bytes = ws.buf.numel()
        a.stream = self.stream
        rc = self.fn(self.args_ref)
        if rc != 0:
            ws.dirty = True
            msg = lib.gsvc_last_error().decode(errors="replace")
            raise RuntimeError(f"gsvc_train_step_sum failed (status {rc}): {msg}")

    def result(self):
        """(mean squared error, mean absolute error) of the last launched step:
        waits for its sequence word (the reference's PSNR ``.item()``); after
        50 ms of spinning, for the whole stream, which reports a failed kernel."""
        L.call("gsvc_wait_host_seq", self.host + 8, self.seq, self.stream, 50000)
        if self.det:
            pairs = int(self.host_u[3])
            ws = _workspace(self.dev, self.n, self.H, self.W)
            self.det_pairs = pairs
            if pairs > ws.det_cap:
                # the pairs past the slot capacity were summed by float
                # atomics: this step's gradients are not bitwise reproducible
                # (the next step's capacity grows from this count)
                self.det_overflows += 1
                msg = (f"gsvc_train_step_sum: deterministic backward had {pairs} (splat, tile) "
                       f"pairs for {ws.det_cap} slots; the excess was summed by float atomics, "
                       "so this step is not bitwise reproducible (capacity grown for the next step)")
                if torch.is_deterministic_algorithms_warn_only_enabled():
                    warnings.warn(msg)
                else:
                    # the step has run (its Adan update is applied: the short
                    # capacity is only known from the step's own pair count);
                    # the work it enqueued for the next step used the same short
                    # capacity, so it is discarded and the next call rebuilds
                    ws.pending = None
                    ws.dirty = True
                    raise RuntimeError(msg + "; this step's parameter update has been applied")
        return self.host_f[0], self.host_f[1]


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
    if ws.pending is not None:  # a bound step's projection ahead: not for this call
        ws.dirty = True
        ws = _workspace(dev, n, H, W)
    _note_launch(p_xyz)
    loss = torch.empty((2,), dtype=torch.float32, device=dev)
    a = _StepArgs()
    a.num_points, a.xyz, a.cholesky, a.cholesky_bound = n, p_xyz, p_chol, p_bound
    a.features, a.rgb_w, a.rgb_w_trainable = p_feat, p_rgbw, 1 if rgb_w_trainable else 0
    a.background, a.gt, a.img_height, a.img_width = p_bg, p_gt, H, W
    a.loss_kind, a.frame_index = LOSS_KIND[loss_type], ws.frame
    a.adan_state, a.adan_hparams = ctypes.addressof(state), ctypes.addressof(hp)
    flags = int(adan_flags)
    if torch.are_deterministic_algorithms_enabled():
        # no pair count comes back without GSVC_TRAIN_LOSS_SEQ: room for 16 per
        # splat (pairs past it fall back to the atomics)
        buf, cap = ws.det_workspace(dev, n, 16 * n)
        a.det_workspace, a.det_workspace_bytes, a.det_capacity = buf.data_ptr(), buf.numel(), cap
        flags |= TRAIN_DETERMINISTIC
    a.adan_flags, a.loss, a.render_out, a.grads_out = flags, loss.data_ptr(), p_render, p_grads
    a.workspace, a.workspace_bytes, a.stream = ws.buf_ptr, ws.buf.numel(), _raw_stream(dev.index)
    rc = L.load().gsvc_train_step_sum_args(ctypes.byref(a))
    if rc != 0:
        ws.dirty = True
        msg = L.load().gsvc_last_error().decode(errors="replace")
        raise RuntimeError(f"gsvc_train_step_sum failed (status {rc}): {msg}")
    ws.frame += 1
    return loss
