"""Adan for GSVC's per-frame models, every update one gfx950 kernel.

GSVC optimises each frame's splats with Adan (reference optimizer.py:39-362;
GaussianSplats_Represent.py:92-96 builds it with lr only, so betas
(0.98, 0.92, 0.99), eps 1e-8, no weight decay, no gradient clipping).  This
optimizer keeps that configuration surface -- constructor keywords, the
per-group ``step`` counter, ``restart_opt``, the state tensor names
(exp_avg, exp_avg_sq, exp_avg_diff, neg_pre_grad) that the fused training
step (train.py) reads and writes -- and performs the update of all of a
group's tensors with ONE launch of gsvc_adan_step (csrc/adan.hip: the
foreach op sequence per element, 44 bytes of HBM traffic each) instead of the
reference's ~17 foreach passes.  There is no CPU path: parameters must be
fp32 CUDA tensors.  The foreach restatement the kernel is checked against
lives in tests/adan_checker.py.
"""
from __future__ import annotations

import math

import torch
from torch.optim.optimizer import Optimizer

_STATE = ("exp_avg", "exp_avg_sq", "exp_avg_diff", "neg_pre_grad")


def _check(name, value, lo, hi=None):
    ok = value >= lo and (hi is None or value < hi)
    if not ok:
        bound = f">= {lo}" if hi is None else f"in [{lo}, {hi})"
        raise ValueError(f"Adan: {name} must be {bound}, got {value}")


class Adan(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.98, 0.92, 0.99), eps=1e-8, weight_decay=0.0,
                 max_grad_norm=0.0, no_prox=False, foreach: bool = True, fused: bool = True):
        _check("lr", lr, 0.0)
        _check("eps", eps, 0.0)
        _check("max_grad_norm", max_grad_norm, 0.0)
        for k, b in enumerate(betas):
            _check(f"betas[{k}]", b, 0.0, 1.0)
        # foreach / fused are accepted for the reference's signature; the update
        # is always the fused kernel with the foreach op sequence
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay, max_grad_norm=max_grad_norm,
                                      no_prox=no_prox, foreach=foreach, fused=fused))

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("no_prox", False)

    @torch.no_grad()
    def restart_opt(self):
        """Zero the moments and the step counters (optimizer.py's restart_opt)."""
        for group in self.param_groups:
            group["step"] = 0
            for p in group["params"]:
                if p.requires_grad:
                    st = self.state[p]
                    for k in _STATE[:3]:
                        st[k] = torch.zeros_like(p)

    def _clip_factor(self) -> float:
        """min(1, max_grad_norm / (||all grads|| + eps)) (optimizer.py:129-147),
        1 when clipping is off."""
        mx = self.defaults["max_grad_norm"]
        if mx <= 0:
            return 1.0
        grads = [p.grad for g in self.param_groups for p in g["params"] if p.grad is not None]
        if not grads:
            return 1.0
        sq = torch.zeros(1, device=grads[0].device)
        for g in grads:
            sq.add_(g.pow(2).sum())
        eps = self.param_groups[-1]["eps"]
        return float(torch.clamp(mx / (sq.sqrt() + eps), max=1.0))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from . import ops
        from .train import bump_param_epoch
        bump_param_epoch()  # a fused step's projection enqueued ahead is stale now
        clip = self._clip_factor()
        for group in self.param_groups:
            live = [p for p in group["params"] if p.grad is not None]
            group["step"] = group.get("step", 0) + 1
            t = group["step"]
            if not live:
                continue
            b1, b2, b3 = group["betas"]
            cols = {k: [] for k in _STATE}
            for p in live:
                st = self.state[p]
                for k in _STATE[:3]:
                    if k not in st:
                        st[k] = torch.zeros_like(p)
                if t == 1 or "neg_pre_grad" not in st:
                    st["neg_pre_grad"] = p.grad.mul(-clip)  # optimizer.py:187-189
                for k in _STATE:
                    cols[k].append(st[k])
            ops.adan_step(live, [p.grad for p in live], cols["exp_avg"], cols["exp_avg_sq"],
                          cols["exp_avg_diff"], cols["neg_pre_grad"], beta1=b1, beta2=b2, beta3=b3,
                          bias_correction1=1.0 - b1 ** t, bias_correction2=1.0 - b2 ** t,
                          bias_correction3_sqrt=math.sqrt(1.0 - b3 ** t), lr=group["lr"],
                          weight_decay=group["weight_decay"], eps=group["eps"],
                          no_prox=group["no_prox"], clip_global_grad_norm=clip)
            if clip != 1.0:
                # the reference scales p.grad in place (optimizer.py:319)
                for p in live:
                    p.grad.mul_(clip)
        return loss
