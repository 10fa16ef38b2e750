"""Fused Adan (gsvc_amd.adan.Adan over gsvc_adan_step) against the foreach
restatement of optimizer.py:296-362 (tools/foreach_adan.py) on the GPU,
several steps, with and without weight decay and no_prox, and against the
reference's own first step (fixture).  fp32 bar: rtol 2e-6 / atol 1e-7 per
step on params and state (rounding only).  Gradient clipping: the step's clip
factor and the in-place p.grad scaling of optimizer.py:319."""
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
    from foreach_adan import ForeachAdan
    from gsvc_amd.adan import Adan
    a = _params(5003, 1, cuda)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    oa = ForeachAdan(a, lr=1e-3, weight_decay=wd, no_prox=no_prox)
    ob = Adan(b, lr=1e-3, weight_decay=wd, no_prox=no_prox)
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


def test_clipping_scales_grads_like_reference(cuda):
    """max_grad_norm > 0: the update uses clip = min(1, max / (||g|| + eps))
    and p.grad is left scaled by it (optimizer.py:129-147, 319)."""
    from foreach_adan import foreach_adan
    from gsvc_amd.adan import Adan
    a = _params(777, 4, cuda)
    grads = [torch.randn(p.shape, generator=torch.Generator().manual_seed(9)).to(cuda) * 3.0
             for p in a]
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    opt = Adan(a, lr=1e-3, max_grad_norm=0.5)
    for p, g in zip(a, grads):
        p.grad = g.clone()
    opt.step()
    norm = torch.sqrt(sum((g ** 2).sum() for g in grads))
    clip = float(torch.clamp(0.5 / (norm + 1e-8), max=1.0))
    assert clip < 1.0
    gb = [g.clone() for g in grads]
    st = [dict(m=torch.zeros_like(p), v=torch.zeros_like(p), d=torch.zeros_like(p),
               n=g.clone().mul_(-clip)) for p, g in zip(b, gb)]
    with torch.no_grad():
        foreach_adan([p.data for p in b], gb, [s["m"] for s in st], [s["v"] for s in st],
                     [s["d"] for s in st], [s["n"] for s in st], beta1=0.98, beta2=0.92,
                     beta3=0.99, bias_correction1=0.02, bias_correction2=0.08,
                     bias_correction3_sqrt=0.1, lr=1e-3, weight_decay=0.0, eps=1e-8,
                     no_prox=False, clip_global_grad_norm=clip)
    for pa, pb, g in zip(a, b, grads):
        torch.testing.assert_close(pa.detach(), pb.detach(), rtol=2e-6, atol=1e-7)
        torch.testing.assert_close(pa.grad, g * clip, rtol=1e-6, atol=0)


def test_argument_checks():
    from gsvc_amd.adan import Adan
    p = [torch.nn.Parameter(torch.zeros(3))]
    for kw in (dict(lr=-1.0), dict(eps=-1.0), dict(max_grad_norm=-0.1), dict(betas=(0.9, 1.0, 0.9))):
        with pytest.raises(ValueError):
            Adan(p, **kw)


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
