"""Fused Adan (gsvc_adan_step) against the foreach restatement of
optimizer.py:296-362 on the GPU, several steps, with and without weight decay
and no_prox, and against the reference's own first step (fixture).  fp32 bar:
rtol 2e-6 / atol 1e-7 per step on params and state (rounding only)."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _params(n, seed, dev):
    g = torch.Generator().manual_seed(seed)
    shapes = [(n, 2), (n, 3), (n, 3), (n, 1)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(dev)) for s in shapes]


@pytest.mark.parametrize("wd,no_prox", [(0.0, False), (0.02, False), (0.02, True)])
def test_fused_matches_foreach(cuda, wd, no_prox):
    from gsvc_amd.adan import Adan
    a = _params(5003, 1, cuda)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    oa = Adan(a, lr=1e-3, weight_decay=wd, no_prox=no_prox, fused=False)
    ob = Adan(b, lr=1e-3, weight_decay=wd, no_prox=no_prox, fused=True)
    g = torch.Generator().manual_seed(2)
    for step in range(6):
        for pa, pb in zip(a, b):
            grad = torch.randn(pa.shape, generator=g).to(cuda)
            pa.grad = grad.clone()
            pb.grad = grad.clone()
        oa.step()
        ob.step()
        for pa, pb in zip(a, b):
            torch.testing.assert_close(pb.detach(), pa.detach(), rtol=2e-6, atol=1e-7)
            for k in ("exp_avg", "exp_avg_sq", "exp_avg_diff", "neg_pre_grad"):
                torch.testing.assert_close(ob.state[pb][k], oa.state[pa][k], rtol=2e-6, atol=1e-7)


def test_fused_first_step_matches_reference_fixture(cuda):
    from gsvc_amd.adan import Adan
    z = load_golden("train_iter_64x64_n200")
    names = ["_xyz", "_cholesky", "_features_dc"]
    params = [torch.nn.Parameter(torch.from_numpy(z["init_" + k].copy()).to(cuda)) for k in names]
    opt = Adan(params, lr=1e-3, fused=True)
    for p, k in zip(params, names):
        p.grad = torch.from_numpy(z["grad_" + k].copy()).to(cuda)
    opt.step()
    for p, k in zip(params, names):
        np.testing.assert_allclose(p.detach().cpu().numpy(), z["step1_" + k], rtol=0, atol=2e-6)


def test_empty_and_errors(cuda):
    from gsvc_amd import ops
    ops.adan_step([], [], [], [], [], [], beta1=0.98, beta2=0.92, beta3=0.99, bias_correction1=1,
                  bias_correction2=1, bias_correction3_sqrt=1, lr=1e-3, weight_decay=0.0,
                  eps=1e-8, no_prox=False, clip_global_grad_norm=1.0)
    x = torch.zeros(4, device=cuda)
    with pytest.raises(RuntimeError):
        ops.adan_step([x], [x.double()], [x], [x], [x], [x], beta1=0.98, beta2=0.92, beta3=0.99,
                      bias_correction1=1, bias_correction2=1, bias_correction3_sqrt=1, lr=1e-3,
                      weight_decay=0.0, eps=1e-8, no_prox=False, clip_global_grad_norm=1.0)
