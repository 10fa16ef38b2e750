"""The foreach Adan update of GSVC's optimizer (reference optimizer.py:296-362
``_multi_tensor_adan``, bias corrections :171-173,211, first-step neg_pre_grad
:187-189) as torch foreach ops, op for op.  Two users: the tests hold the
product optimizer (gsvc_amd/adan.py, one fused kernel) to this sequence, and
bench.py's op_path times GSVC's files with the reference optimizer's own
sequence (train_iters_per_s_foreach_adan).  Never imported by the product
path."""
import math

import torch


def foreach_adan(params, grads, exp_avgs, exp_avg_sqs, exp_avg_diffs, neg_pre_grads, *, beta1,
                 beta2, beta3, bias_correction1, bias_correction2, bias_correction3_sqrt, lr,
                 weight_decay, eps, no_prox, clip_global_grad_norm):
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


class ForeachAdan:
    """A minimal optimizer over ``foreach_adan`` with the reference's state
    handling (per-group step, lazily created state, no clipping)."""

    def __init__(self, params, lr=1e-3, betas=(0.98, 0.92, 0.99), eps=1e-8, weight_decay=0.0,
                 no_prox=False):
        self.params = list(params)
        self.lr, self.betas, self.eps, self.wd, self.no_prox = lr, betas, eps, weight_decay, no_prox
        self.t = 0
        self.state = {}

    @torch.no_grad()
    def step(self):
        self.t += 1
        b1, b2, b3 = self.betas
        live = [p for p in self.params if p.grad is not None]
        for p in live:
            st = self.state.setdefault(p, {})
            if not st:
                st.update(exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p),
                          exp_avg_diff=torch.zeros_like(p))
            if self.t == 1 or "neg_pre_grad" not in st:
                st["neg_pre_grad"] = p.grad.clone().mul_(-1.0)
        col = lambda k: [self.state[p][k] for p in live]  # noqa: E731
        foreach_adan(live, [p.grad for p in live], col("exp_avg"), col("exp_avg_sq"),
                     col("exp_avg_diff"), col("neg_pre_grad"), beta1=b1, beta2=b2, beta3=b3,
                     bias_correction1=1 - b1 ** self.t, bias_correction2=1 - b2 ** self.t,
                     bias_correction3_sqrt=math.sqrt(1 - b3 ** self.t), lr=self.lr,
                     weight_decay=self.wd, eps=self.eps, no_prox=self.no_prox,
                     clip_global_grad_norm=1.0)
