"""Adan optimizer as used by GSVC (reference optimizer.py:39-362, foreach path).

``Adan`` keeps the reference's constructor defaults (lr 1e-3, betas
(0.98, 0.92, 0.99), eps 1e-8, weight_decay 0, max_grad_norm 0, no_prox False),
its per-group step counter, and the update order of ``_multi_tensor_adan``
(optimizer.py:296-362).  With ``fused=True`` the whole update of every
parameter of a group runs as one gfx950 kernel per tensor
(gsvc_amd/csrc/adan.hip) instead of ~17 foreach launches.
"""
from __future__ import annotations

import math
from typing import List

import torch
from torch import Tensor
from torch.optim.optimizer import Optimizer


class Adan(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.98, 0.92, 0.99), eps=1e-8, weight_decay=0.0,
                 max_grad_norm=0.0, no_prox=False, foreach: bool = True, fused: bool = False):
        if not 0.0 <= max_grad_norm:
            raise ValueError("Invalid Max grad norm: {}".format(max_grad_norm))
        if not 0.0 <= lr:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {}".format(eps))
        for i in range(3):
            if not 0.0 <= betas[i] < 1.0:
                raise ValueError("Invalid beta parameter at index {}: {}".format(i, betas[i]))
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm, no_prox=no_prox, foreach=foreach, fused=fused)
        super().__init__(params, defaults)

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("no_prox", False)

    @torch.no_grad()
    def restart_opt(self):
        for group in self.param_groups:
            group["step"] = 0
            for p in group["params"]:
                if p.requires_grad:
                    state = self.state[p]
                    state["exp_avg"] = torch.zeros_like(p)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                    state["exp_avg_diff"] = torch.zeros_like(p)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()

        if self.defaults["max_grad_norm"] > 0:
            device = self.param_groups[0]["params"][0].device
            global_grad_norm = torch.zeros(1, device=device)
            max_grad_norm = torch.tensor(self.defaults["max_grad_norm"], device=device)
            for group in self.param_groups:
                for p in group["params"]:
                    if p.grad is not None:
                        global_grad_norm.add_(p.grad.pow(2).sum())
            global_grad_norm = torch.sqrt(global_grad_norm)
            clip_global_grad_norm = torch.clamp(
                max_grad_norm / (global_grad_norm + group["eps"]), max=1.0).item()
        else:
            clip_global_grad_norm = 1.0

        for group in self.param_groups:
            params_with_grad, grads, exp_avgs, exp_avg_sqs, exp_avg_diffs, neg_pre_grads = (
                [], [], [], [], [], [])
            beta1, beta2, beta3 = group["betas"]
            group["step"] = group.get("step", 0) + 1
            bias_correction1 = 1.0 - beta1 ** group["step"]
            bias_correction2 = 1.0 - beta2 ** group["step"]
            bias_correction3 = 1.0 - beta3 ** group["step"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                params_with_grad.append(p)
                grads.append(p.grad)
                state = self.state[p]
                if len(state) == 0:
                    state["exp_avg"] = torch.zeros_like(p)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                    state["exp_avg_diff"] = torch.zeros_like(p)
                if "neg_pre_grad" not in state or group["step"] == 1:
                    state["neg_pre_grad"] = p.grad.clone().mul_(-clip_global_grad_norm)
                exp_avgs.append(state["exp_avg"])
                exp_avg_sqs.append(state["exp_avg_sq"])
                exp_avg_diffs.append(state["exp_avg_diff"])
                neg_pre_grads.append(state["neg_pre_grad"])
            if not params_with_grad:
                continue
            kwargs = dict(params=params_with_grad, grads=grads, exp_avgs=exp_avgs,
                          exp_avg_sqs=exp_avg_sqs, exp_avg_diffs=exp_avg_diffs,
                          neg_pre_grads=neg_pre_grads, beta1=beta1, beta2=beta2, beta3=beta3,
                          bias_correction1=bias_correction1, bias_correction2=bias_correction2,
                          bias_correction3_sqrt=math.sqrt(bias_correction3), lr=group["lr"],
                          weight_decay=group["weight_decay"], eps=group["eps"],
                          no_prox=group["no_prox"], clip_global_grad_norm=clip_global_grad_norm)
            if group["fused"]:
                from . import ops
                ops.adan_step(**kwargs)
            else:
                _multi_tensor_adan(**kwargs)
        return loss


def _multi_tensor_adan(params: List[Tensor], grads: List[Tensor], exp_avgs: List[Tensor],
                       exp_avg_sqs: List[Tensor], exp_avg_diffs: List[Tensor],
                       neg_pre_grads: List[Tensor], *, beta1: float, beta2: float, beta3: float,
                       bias_correction1: float, bias_correction2: float,
                       bias_correction3_sqrt: float, lr: float, weight_decay: float, eps: float,
                       no_prox: bool, clip_global_grad_norm):
    """optimizer.py:296-362, op for op."""
    if len(params) == 0:
        return
    torch._foreach_mul_(grads, clip_global_grad_norm)
    torch._foreach_add_(neg_pre_grads, grads)
    torch._foreach_mul_(exp_avgs, beta1)
    torch._foreach_add_(exp_avgs, grads, alpha=1 - beta1)
    torch._foreach_mul_(exp_avg_diffs, beta2)
    torch._foreach_add_(exp_avg_diffs, neg_pre_grads, alpha=1 - beta2)
    torch._foreach_mul_(neg_pre_grads, beta2)
    torch._foreach_add_(neg_pre_grads, grads)
    torch._foreach_mul_(exp_avg_sqs, beta3)
    torch._foreach_addcmul_(exp_avg_sqs, neg_pre_grads, neg_pre_grads, value=1 - beta3)
    denom = torch._foreach_sqrt(exp_avg_sqs)
    torch._foreach_div_(denom, bias_correction3_sqrt)
    torch._foreach_add_(denom, eps)
    step_size_diff = lr * beta2 / bias_correction2
    step_size = lr / bias_correction1
    if no_prox:
        torch._foreach_mul_(params, 1 - lr * weight_decay)
        torch._foreach_addcdiv_(params, exp_avgs, denom, value=-step_size)
        torch._foreach_addcdiv_(params, exp_avg_diffs, denom, value=-step_size_diff)
    else:
        torch._foreach_addcdiv_(params, exp_avgs, denom, value=-step_size)
        torch._foreach_addcdiv_(params, exp_avg_diffs, denom, value=-step_size_diff)
        torch._foreach_div_(params, 1 + lr * weight_decay)
    torch._foreach_zero_(neg_pre_grads)
    torch._foreach_add_(neg_pre_grads, grads, alpha=-1.0)
