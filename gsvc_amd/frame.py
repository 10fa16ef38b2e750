"""Per-frame model: a restatement of GSVC's caller of the hot path.

``GaussianVideoFrame`` mirrors ``GaussianVideo_frame``
(reference GaussianSplats_Represent.py:11-221): the same parameters and init
distributions (:28-38), activations (:57-70), forward (:83-90: project ->
sum-rasterize -> clamp -> NCHW), ``train_iter`` (:191-207: L2 loss, PSNR via
``.item()``, Adan step, zero_grad, StepLR), and the prune / densify controls
(:98-172).  It is used by bench.py, the tests and the video driver; GSVC's own
file also runs unchanged on top of the ``gsplat`` drop-in package.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import msssim
from .adan import Adan
from .project_gaussians_2d import project_gaussians_2d
from .rasterize_sum import rasterize_gaussians_sum
from .prune import prune_lowest
from .render import BoundRender, render_frame_sum
from .train import LOSS_KIND, BoundStep


def loss_fn(pred, target, loss_type="L2", lambda_value=0.7):
    """utils.py:21-41.  The SSIM terms are gsvc_amd.msssim (pytorch_msssim's
    ssim / ms_ssim on the gfx950 kernels, CUDA tensors only); as in the
    reference they need 4-d inputs, so train_iter's squeezed [3,H,W] images
    raise for them there (GaussianSplats_Represent.py:194) and pre_train_iter's
    NCHW ones (:213) work."""
    target = target.detach()
    pred = pred.float()
    target = target.float()
    if loss_type == "L2":
        return F.mse_loss(pred, target)
    if loss_type == "L1":
        return F.l1_loss(pred, target)
    if loss_type == "SSIM":
        return 1 - msssim.ssim(pred, target, data_range=1, size_average=True)
    if loss_type == "Fusion1":
        return lambda_value * F.mse_loss(pred, target) + (1 - lambda_value) * (
            1 - msssim.ssim(pred, target, data_range=1, size_average=True))
    if loss_type == "Fusion2":
        return lambda_value * F.l1_loss(pred, target) + (1 - lambda_value) * (
            1 - msssim.ssim(pred, target, data_range=1, size_average=True))
    if loss_type == "Fusion3":
        return lambda_value * F.mse_loss(pred, target) + (1 - lambda_value) * F.l1_loss(pred, target)
    if loss_type == "Fusion4":
        return lambda_value * F.l1_loss(pred, target) + (1 - lambda_value) * (
            1 - msssim.ms_ssim(pred, target, data_range=1, size_average=True))
    if loss_type == "Fusion_hinerv":
        return lambda_value * F.l1_loss(pred, target) + (1 - lambda_value) * (
            1 - msssim.ms_ssim(pred, target, data_range=1, size_average=True, win_size=5))
    # the reference falls through to `return loss` with loss unassigned
    raise UnboundLocalError(f"loss_fn: unknown loss_type {loss_type!r}")


class GaussianVideoFrame(nn.Module):
    def __init__(self, loss_type="L2", **kwargs):
        super().__init__()
        self.loss_type = loss_type
        self.init_num_points = kwargs["num_points"]
        self.max_num_points = kwargs["max_num_points"]
        self.densification_interval = kwargs["densification_interval"]
        self.iterations = kwargs["iterations"]
        self.H, self.W = kwargs["H"], kwargs["W"]
        self.BLOCK_W, self.BLOCK_H = kwargs["BLOCK_W"], kwargs["BLOCK_H"]
        self.tile_bounds = ((self.W + self.BLOCK_W - 1) // self.BLOCK_W,
                            (self.H + self.BLOCK_H - 1) // self.BLOCK_H, 1)
        self.device = kwargs["device"]
        self.removal_rate = kwargs["removal_rate"]
        n = self.init_num_points
        self._xyz = nn.Parameter(torch.atanh(2 * (torch.rand(n, 2) - 0.5)))
        self._cholesky = nn.Parameter(torch.rand(n, 3))
        self.isdensity = kwargs["isdensity"]
        self.isremoval = kwargs["isremoval"]
        if self.isremoval:
            self.rgb_W = nn.Parameter(0.01 * torch.ones(n, 1))
        elif self.isdensity:
            self.rgb_W = nn.Parameter(torch.ones(n, 1))
        else:
            self.register_buffer("rgb_W", torch.ones((n, 1)))
        self._features_dc = nn.Parameter(torch.rand(n, 3))
        self.last_size = (self.H, self.W)
        self.quantize = kwargs.get("quantize", False)
        self.register_buffer("background", torch.ones(3))
        self.register_buffer("bound", torch.tensor([0.5, 0.5]).view(1, 2))
        self.register_buffer("cholesky_bound", torch.tensor([0.5, 0, 0.5]).view(1, 3))
        self.lr = kwargs["lr"]
        self.opt_type = kwargs["opt_type"]
        # whole train_iter as one fused call (gsvc_amd/train.py) where it applies
        self.fused_train = kwargs.get("fused_train", str(self.device).startswith("cuda"))
        # forward() without autograd as the one-call frame render (render.py);
        # False: GSVC's own op sequence (project -> rasterize -> clamp -> NCHW)
        self.fused_render = kwargs.get("fused_render", True)
        self.fused_steps = 0
        self._bound_step = None
        self._bound_render = None
        self._fused_ok = None
        self.update_optimizer()
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=20000, gamma=0.5)

    @property
    def get_xyz(self):
        return torch.tanh(self._xyz)

    @property
    def get_features(self):
        return self._features_dc * self.get_rgb_W

    @property
    def get_rgb_W(self):
        return self.rgb_W

    @property
    def get_cholesky_elements(self):
        return self._cholesky + self.cholesky_bound

    def _ones_opacity(self):
        n = self._xyz.shape[0]
        o = getattr(self, "_opacity_ones", None)
        if o is None or o.shape[0] != n or o.device != self._xyz.device:
            o = torch.ones(n, 1, device=self._xyz.device)
            self._opacity_ones = o
        return o

    def forward(self):
        if (not torch.is_grad_enabled() and self.fused_render and self.BLOCK_H == 16
                and self.BLOCK_W == 16):
            # inference: same image from the sync-free path with the clamp +
            # NCHW epilogue fused into the rasterizer (gsvc_amd/render.py)
            # (activations fused into the frame kernel: tanh, + bound, * rgb_W)
            bound = (self._xyz, self._cholesky, self._features_dc, self.background,
                     self.cholesky_bound, self.rgb_W)
            br = self._bound_render
            if br is None or not br.matches(bound):
                try:
                    br = self._bound_render = BoundRender(
                        self._xyz, self._cholesky, self._features_dc, self.H, self.W,
                        self.background, cholesky_bound=self.cholesky_bound, rgb_w=self.rgb_W)
                except ValueError:  # non-contiguous / non-fp32 tensors: the general call
                    self._bound_render = None
                    return {"render": render_frame_sum(
                        self._xyz, self._cholesky, self._features_dc, self.H, self.W,
                        self.background, xyz_tanh=True, cholesky_bound=self.cholesky_bound,
                        rgb_w=self.rgb_W)}
            return {"render": br()}
        # reference: torch.ones(N, 1).to(device) per call; same values
        _opacity = self._ones_opacity()
        self.xys, depths, self.radii, conics, num_tiles_hit = project_gaussians_2d(
            self.get_xyz, self.get_cholesky_elements, self.H, self.W, self.tile_bounds)
        out_img = rasterize_gaussians_sum(self.xys, depths, self.radii, conics, num_tiles_hit,
                                          self.get_features, _opacity, self.H, self.W, self.BLOCK_H,
                                          self.BLOCK_W, background=self.background,
                                          return_alpha=False)
        out_img = torch.clamp(out_img, 0, 1)
        out_img = out_img.view(-1, self.H, self.W, 3).permute(0, 3, 1, 2).contiguous()
        return {"render": out_img}

    def update_optimizer(self):
        from .train import bump_param_epoch
        bump_param_epoch()  # new parameters / optimizer: nothing projected ahead applies
        if self.opt_type == "adam":
            self.optimizer = torch.optim.Adam(self.parameters(), lr=self.lr)
        else:
            self.optimizer = Adan(self.parameters(), lr=self.lr)

    def _remove_lowest(self, remove_count):
        # norm + torch.sort + boolean mask + p[keep] (GaussianSplats_Represent.py:
        # 101-125, 149-166) as one radix select and compaction on the GPU
        with torch.no_grad():
            ps = prune_lowest(self.rgb_W, [self._xyz, self._cholesky, self._features_dc, self.rgb_W],
                              remove_count)
            self._xyz, self._cholesky, self._features_dc, self.rgb_W = (nn.Parameter(p) for p in ps)

    def _refresh_groups(self):
        for param_group in self.optimizer.param_groups:
            param_group["params"] = [p for p in self.parameters() if p.requires_grad]

    def removal_control(self, iter):
        """GaussianSplats_Represent.py:98-128 (I-frame pruning)."""
        iter_threshold_remove = 4000
        if iter > iter_threshold_remove:
            return
        removal_rate_per_step = self.removal_rate / int(iter_threshold_remove / self.densification_interval)
        if iter < iter_threshold_remove:
            self._remove_lowest(int(removal_rate_per_step * self.max_num_points))
            self._refresh_groups()
        elif iter == iter_threshold_remove:
            remove_count = self._xyz.shape[0] - int(self.max_num_points * (1 - self.removal_rate))
            if remove_count > 0:
                self._remove_lowest(remove_count)
            self.update_optimizer()

    def adaptive_control(self, iter):
        """GaussianSplats_Represent.py:130-172 (P-frame densify then prune)."""
        iter_threshold_remove = 500
        iter_threshold_add = 500
        densification_num = int(self.max_num_points * self.removal_rate)
        if iter > iter_threshold_add + iter_threshold_remove or iter < iter_threshold_add:
            if iter == 1 and densification_num > 0:
                dev = self._xyz.device
                new_xyz = torch.atanh(2 * (torch.rand(densification_num, 2) - 0.5)).to(dev)
                new_cholesky = torch.rand(densification_num, 3).to(dev)
                new_features_dc = torch.rand(densification_num, 3).to(dev)
                new_rgb_W = 0.01 * torch.ones(densification_num, 1).to(dev)
                self._xyz = nn.Parameter(torch.cat((self._xyz, new_xyz), dim=0))
                self._cholesky = nn.Parameter(torch.cat((self._cholesky, new_cholesky), dim=0))
                self._features_dc = nn.Parameter(torch.cat((self._features_dc, new_features_dc), dim=0))
                self.rgb_W = nn.Parameter(torch.cat((self.rgb_W, new_rgb_W), dim=0))
                self._refresh_groups()
            return
        if iter < iter_threshold_add + iter_threshold_remove:
            remove_count = int(densification_num / int(iter_threshold_remove / self.densification_interval))
            self._remove_lowest(remove_count)
            self._refresh_groups()
        elif iter == iter_threshold_add + iter_threshold_remove:
            remove_count = self._xyz.shape[0] - int(self.max_num_points * (1 - self.removal_rate))
            if remove_count > 0:
                self._remove_lowest(remove_count)
            self.update_optimizer()

    def _control_replaces_params(self, iter):
        """Whether train_iter's prune / densify at this iteration replaces the
        parameters (adaptive_control / removal_control below): densify at
        iteration 1, pruning inside their windows, and the final prune when it
        removes anything.  Not the final update_optimizer alone, whose new
        optimizer still steps on this iteration's gradients."""
        final_remove = self._xyz.shape[0] - int(self.max_num_points * (1 - self.removal_rate)) > 0
        if (iter == 1 or iter % self.densification_interval == 0) and self.isdensity:
            if iter == 1:
                return int(self.max_num_points * self.removal_rate) > 0
            if iter < 500 or iter > 1000:
                return False
            return iter < 1000 or final_remove
        if iter % self.densification_interval == 0 and self.isremoval:
            if iter > 4000:
                return False
            return iter < 4000 or final_remove
        return False

    def _fused_train_params(self, gt_image):
        """(rgb_W trainable?) when this iteration can run as one fused step
        (train.py): L2 / L1 loss, Adan without gradient clipping, the model's
        own parameters in one group, no gradients pending; else None.  The
        configuration checks are cached against the objects they looked at
        (optimizer, its group list, the parameters); per call only the pending
        gradients and the target are checked."""
        P = self._parameters
        ps = (P.get("_xyz"), P.get("_cholesky"), P.get("_features_dc"),
              P["rgb_W"] if "rgb_W" in P else self._buffers.get("rgb_W"))
        opt = self.optimizer
        c = self._fused_ok
        if (c is not None and c[0] is opt and len(opt.param_groups) == 1
                and c[1] is opt.param_groups[0]["params"] and all(a is b for a, b in zip(c[2], ps))
                and c[4] == (self.fused_train, self.loss_type, opt.defaults["max_grad_norm"])):
            for p in c[3]:
                if (p.grad is not None or not p.requires_grad or p.dtype is not torch.float32
                        or not p.is_contiguous()):
                    return None
            if gt_image.numel() != 3 * self.H * self.W or gt_image.device != ps[0].device:
                return None
            return c[5]
        r = self._fused_train_params_full(gt_image)
        self._fused_ok = None
        if r is not None:
            params = ps[:3] + ((ps[3],) if r else ())
            self._fused_ok = (opt, opt.param_groups[0]["params"], ps, params,
                              (self.fused_train, self.loss_type, opt.defaults["max_grad_norm"]), r)
        return r

    def _fused_train_params_full(self, gt_image):
        if not self.fused_train or self.loss_type not in LOSS_KIND or self.opt_type == "adam":
            return None
        if self.BLOCK_H != 16 or self.BLOCK_W != 16 or not self._xyz.is_cuda:
            return None
        opt = self.optimizer
        if not isinstance(opt, Adan) or len(opt.param_groups) != 1 or opt.defaults["max_grad_norm"] > 0:
            return None
        rgbw_train = isinstance(self.rgb_W, nn.Parameter) and self.rgb_W.requires_grad
        params = [self._xyz, self._cholesky, self._features_dc] + ([self.rgb_W] if rgbw_train else [])
        group = opt.param_groups[0]["params"]
        if len(group) != len(params) or {id(p) for p in group} != {id(p) for p in params}:
            return None
        for p in params:
            if (p.grad is not None or not p.requires_grad or p.dtype != torch.float32
                    or not p.is_contiguous()):
                return None
        if gt_image.numel() != 3 * self.H * self.W or gt_image.device != self._xyz.device:
            return None
        return rgbw_train

    def _train_iter_fused(self, gt_image, rgbw_train):
        """train_iter (GaussianSplats_Represent.py:191-207) as one fused call:
        forward, loss, backward and the Adan step of optimizer.py:124-235 with
        this optimizer's state, step counter and learning rate."""
        opt = self.optimizer
        group = opt.param_groups[0]
        group["step"] = group.get("step", 0) + 1
        step = group["step"]
        b1, b2, b3 = group["betas"]
        hparams = [b1, b2, b3, 1.0 - b1 ** step, 1.0 - b2 ** step, math.sqrt(1.0 - b3 ** step),
                   group["lr"], group["weight_decay"], group["eps"], 1.0]
        flags = 1 if group["no_prox"] else 0
        P = self._parameters
        xyz, chol, feat = P["_xyz"], P["_cholesky"], P["_features_dc"]
        rgbw = P["rgb_W"] if "rgb_W" in P else self._buffers.get("rgb_W")  # a buffer when fixed
        state = []
        for q, p in enumerate((xyz, chol, feat, rgbw if rgbw_train else None)):
            if p is None:
                state += [None] * 4
                continue
            st = opt.state[p]
            if len(st) == 0:
                st["exp_avg"] = torch.zeros_like(p)
                st["exp_avg_sq"] = torch.zeros_like(p)
                st["exp_avg_diff"] = torch.zeros_like(p)
            if "neg_pre_grad" not in st or step == 1:
                st["neg_pre_grad"] = torch.empty_like(p)  # the kernel starts it at -grad
                flags |= 1 << (1 + q)
            state += [st["exp_avg"], st["exp_avg_sq"], st["exp_avg_diff"], st["neg_pre_grad"]]
        gt = gt_image.detach() if gt_image.requires_grad else gt_image
        if gt.dtype is not torch.float32 or not gt.is_contiguous():
            gt = gt.float().contiguous()
        # the step bound to these tensors: pointers built once, rebuilt when any
        # parameter, state tensor or constant object changes
        B = self._buffers
        bound = (xyz, chol, feat, rgbw, B["cholesky_bound"], B["background"], *state)
        bs = self._bound_step
        if bs is None or bs.rgbw_train != int(rgbw_train) or not bs.matches(bound):
            bs = self._bound_step = BoundStep(*bound[:4], rgbw_train, *bound[4:6], self.H, self.W,
                                              self.loss_type, state)
        bs.launch(gt, hparams, flags)
        # the step ran (keeps StepLR's call-order check quiet; the scheduler may
        # hold the optimizer from before update_optimizer, as in the reference).
        # The scheduler only sets the next iteration's lr, so it steps while the
        # kernels run, before the PSNR read-back waits for them.
        opt._opt_called = True
        self.scheduler.optimizer._opt_called = True
        self.__dict__["fused_steps"] += 1  # a plain counter: skip Module.__setattr__
        self.scheduler.step()
        # the loss as a host scalar tensor (callers take .item() / float() of it),
        # made while the kernels run: after the wait only its value is stored
        loss = torch.empty(())
        loss_np = loss.numpy()
        mse, l1 = bs.result()  # the reference's PSNR .item(): one stream wait
        loss_np[...] = l1 if self.loss_type == "L1" else mse
        psnr = 10 * math.log10(1.0 / mse)
        return loss, psnr

    def train_iter(self, gt_image, iter):
        """GaussianSplats_Represent.py:191-207: one training iteration on
        ``gt_image``; returns (loss, psnr).  The fused step may enqueue work of
        the NEXT iteration against this target and these parameters: writes to
        either that bypass torch's version counter (``.data``, DLPack views, a
        custom kernel) must be followed by ``gsvc_amd.train.bump_param_epoch()``."""
        controls = (((iter == 1 or iter % self.densification_interval == 0) and self.isdensity)
                    or (iter % self.densification_interval == 0 and self.isremoval))
        rgbw_train = None if controls else self._fused_train_params(gt_image)
        if rgbw_train is not None:
            return self._train_iter_fused(gt_image, rgbw_train)
        if controls and self.fused_train and self._control_replaces_params(iter):
            # the gradients of this iteration would be dropped unused: the
            # control swaps in new Parameters (no .grad), so Adan only advances
            # its step count.  Forward only (the same image bits and loss).
            with torch.no_grad():
                image = self.forward()["render"]
                loss = loss_fn(image.squeeze(0), gt_image.squeeze(0), self.loss_type, lambda_value=0)
                psnr = 10 * math.log10(1.0 / F.mse_loss(image, gt_image).item())
            if (iter == 1 or iter % self.densification_interval == 0) and self.isdensity:
                self.adaptive_control(iter)
            else:
                self.removal_control(iter)
            self.optimizer.step()
            self.optimizer.zero_grad(set_to_none=True)
            self.scheduler.step()
            return loss, psnr
        render_pkg = self.forward()
        image = render_pkg["render"]
        loss = loss_fn(image.squeeze(0), gt_image.squeeze(0), self.loss_type, lambda_value=0)
        loss.backward()
        with torch.no_grad():
            mse_loss = F.mse_loss(image, gt_image)
            psnr = 10 * math.log10(1.0 / mse_loss.item())
        if (iter == 1 or iter % self.densification_interval == 0) and self.isdensity:
            self.adaptive_control(iter)
        elif iter % self.densification_interval == 0 and self.isremoval:
            self.removal_control(iter)
        self.optimizer.step()
        self.optimizer.zero_grad(set_to_none=True)
        self.scheduler.step()
        return loss, psnr

    def train_iter_trace(self, gt_image, iter):
        """GaussianSplats_Represent.py:175-188: train_iter returning the render."""
        render_pkg = self.forward()
        image = render_pkg["render"]
        loss = loss_fn(image.squeeze(0), gt_image.squeeze(0), self.loss_type, lambda_value=0)
        loss.backward()
        if (iter == 1 or iter % self.densification_interval == 0) and self.isdensity:
            self.adaptive_control(iter)
        elif iter % self.densification_interval == 0 and self.isremoval:
            self.removal_control(iter)
        self.optimizer.step()
        self.optimizer.zero_grad(set_to_none=True)
        self.scheduler.step()
        return image

    def pre_train_iter(self, gt_image):
        """GaussianSplats_Represent.py:210-222 (the K-frame detector's step): no
        pruning or densification, the loss on the NCHW images with lambda 0.7.
        L2 / L1 take the fused step (lambda does not enter them)."""
        rgbw_train = self._fused_train_params(gt_image)
        if rgbw_train is not None:
            return self._train_iter_fused(gt_image, rgbw_train)
        render_pkg = self.forward()
        image = render_pkg["render"]
        loss = loss_fn(image, gt_image, self.loss_type, lambda_value=0.7)
        loss.backward()
        with torch.no_grad():
            mse_loss = F.mse_loss(image, gt_image)
            psnr = 10 * math.log10(1.0 / mse_loss.item())
        self.optimizer.step()
        self.optimizer.zero_grad(set_to_none=True)
        self.scheduler.step()
        return loss, psnr


def make_frame_model(H, W, num_points, device, seed=None, lr=1e-3, isremoval=False,
                     isdensity=False, removal_rate=0.1, max_num_points=None,
                     densification_interval=100, fused_train=None, fused_render=None):
    """Construct like SimpleTrainer2d does (train_video_Represent.py:51-55).
    fused_train / fused_render False: train_iter / forward() take GSVC's own op
    sequence through the gsplat operators (the unchanged-caller path)."""
    if seed is not None:
        torch.manual_seed(seed)
    model = GaussianVideoFrame(
        loss_type="L2", opt_type="adan", num_points=num_points,
        max_num_points=max_num_points or num_points, densification_interval=densification_interval,
        iterations=30000, H=H, W=W, BLOCK_H=16, BLOCK_W=16, device=device, lr=lr, quantize=False,
        removal_rate=removal_rate, isdensity=isdensity, isremoval=isremoval,
        **({} if fused_train is None else {"fused_train": fused_train}),
        **({} if fused_render is None else {"fused_render": fused_render})).to(device)
    return model


def synthetic_gt(H, W, seed, device):
    """Seeded smooth procedural RGB frame in [0, 1]: a sum of 8
    random sinusoids per channel."""
    g = torch.Generator().manual_seed(int(seed))
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    chans = []
    for _ in range(3):
        acc = torch.zeros(H, W)
        for _ in range(8):
            fx, fy, ph = (torch.rand(3, generator=g) * torch.tensor([12.0, 12.0, 6.28])).tolist()
            acc += torch.sin(fx * xx + fy * yy + ph)
        chans.append(0.5 + 0.5 * acc / 8)
    return torch.stack(chans)[None].clamp(0, 1).to(device)
