"""SSIM / MS-SSIM (gsvc_amd/msssim.py, csrc/ssim.hip): pytorch_msssim's
algorithm behind its API, for GSVC's SSIM-family losses (utils.py:29-40) and
the per-frame MS-SSIM metric (train_video_Represent.py:145).

pytorch_msssim is absent here and unpinned (requirements.txt:5): parity is
"unpinned" against the package and pinned to two restatements of its published
algorithm -- the float64 oracle (oracle/oracle.py ssim/ms_ssim) and a torch
fp32 one below (F.conv2d with grouped 1-D Gaussian windows, F.avg_pool2d),
which also gives the autograd gradients the HIP backward is checked against.

CPU: the two restatements agree; argument checks.  GPU: values vs the oracle
(abs 2e-5: fp32 filtering vs float64), gradients w.r.t. X and Y vs torch
autograd of the fp32 restatement (relative to the largest element, 1e-3),
1080p, odd sizes, window 5, dimensions shorter than the window, per-image
output, the loss_fn variants end to end.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import REPO  # noqa: F401


# ---------------------------------------------------------------- torch fp32 restatement

def _t_gauss(size, sigma, dtype=torch.float):
    coords = torch.arange(size, dtype=dtype) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    return g.view(1, 1, 1, -1)


def _t_filter(x, win):
    C = x.shape[1]
    w = win.to(x.device, x.dtype).repeat(C, 1, 1, 1)
    out = x
    for i, s in enumerate(x.shape[2:]):
        if s >= w.shape[-1]:
            out = F.conv2d(out, w.transpose(2 + i, -1), groups=C)
    return out


def _t_terms(X, Y, win, C1, C2):
    mu1, mu2 = _t_filter(X, win), _t_filter(Y, win)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _t_filter(X * X, win) - mu1_sq
    s2 = _t_filter(Y * Y, win) - mu2_sq
    s12 = _t_filter(X * Y, win) - mu12
    cs_map = (2 * s12 + C2) / (s1 + s2 + C2)
    ssim_map = ((2 * mu12 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    return torch.flatten(ssim_map, 2).mean(-1), torch.flatten(cs_map, 2).mean(-1)


def t_ssim(X, Y, data_range=1.0, size_average=True, win_size=11, win_sigma=1.5,
           K=(0.01, 0.03), nonnegative_ssim=False, win_dtype=torch.float):
    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    s, _ = _t_terms(X, Y, _t_gauss(win_size, win_sigma, win_dtype), C1, C2)
    if nonnegative_ssim:
        s = torch.relu(s)
    return s.mean() if size_average else s.mean(1)


def t_ms_ssim(X, Y, data_range=1.0, size_average=True, win_size=11, win_sigma=1.5,
              weights=None, K=(0.01, 0.03), win_dtype=torch.float):
    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    w = X.new_tensor(weights or [0.0448, 0.2856, 0.3001, 0.2363, 0.1333])
    win = _t_gauss(win_size, win_sigma, win_dtype)
    mcs = []
    for i in range(w.shape[0]):
        s, cs = _t_terms(X, Y, win, C1, C2)
        if i < w.shape[0] - 1:
            mcs.append(torch.relu(cs))
            pad = [s_ % 2 for s_ in X.shape[2:]]
            X = F.avg_pool2d(X, kernel_size=2, padding=pad)
            Y = F.avg_pool2d(Y, kernel_size=2, padding=pad)
    s = torch.relu(s)
    val = torch.prod(torch.stack(mcs + [s], dim=0) ** w.view(-1, 1, 1), dim=0)
    return val.mean() if size_average else val.mean(1)


def _pair(shape, seed, noise=0.1):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(shape, generator=g)
    Y = (X + noise * torch.randn(shape, generator=g)).clamp(0, 1)
    return X, Y


# ---------------------------------------------------------------- CPU

@pytest.mark.parametrize("shape,win", [((1, 3, 64, 80), 11), ((2, 3, 37, 53), 11),
                                       ((1, 3, 7, 40), 11), ((1, 2, 30, 31), 5)])
def test_torch_restatement_matches_oracle_ssim(oracle, shape, win):
    X, Y = _pair(shape, 1)
    for avg in (True, False):
        # float64 throughout (the package builds an fp32 window: 1e-8 .. 2e-7 apart)
        got = t_ssim(X.double(), Y.double(), win_size=win, size_average=avg,
                     win_dtype=torch.float64).numpy()
        ref = oracle.ssim(X.numpy(), Y.numpy(), 1.0, size_average=avg, win_size=win)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)


@pytest.mark.parametrize("shape,win", [((1, 3, 176, 200), 11), ((2, 1, 97, 71), 5)])
def test_torch_restatement_matches_oracle_ms_ssim(oracle, shape, win):
    X, Y = _pair(shape, 2)
    got = t_ms_ssim(X.double(), Y.double(), win_size=win, win_dtype=torch.float64).item()
    ref = oracle.ms_ssim(X.numpy(), Y.numpy(), 1.0, win_size=win)
    assert abs(got - ref) < 1e-12


def test_argument_checks():
    from gsvc_amd.msssim import ms_ssim, ssim
    X = torch.rand(1, 3, 32, 32)
    with pytest.raises(ValueError, match="same dimensions"):
        ssim(X, torch.rand(1, 3, 32, 31))
    with pytest.raises(ValueError, match="odd"):
        ssim(X, X, win_size=10)
    with pytest.raises(ValueError, match="4-d or 5-d"):
        ssim(torch.rand(3, 32, 32), torch.rand(3, 32, 32))
    with pytest.raises(AssertionError, match="larger than 160"):
        ms_ssim(X, X, data_range=1)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ssim(X, X, data_range=1)


# ---------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("shape,win,avg,nonneg", [
    ((1, 3, 256, 256), 11, True, False), ((2, 3, 37, 53), 11, False, False),
    ((1, 3, 7, 40), 11, True, False), ((1, 2, 30, 31), 5, True, True),
    ((1, 3, 1080, 1920), 11, True, False)])
def test_ssim_matches_oracle(cuda, oracle, shape, win, avg, nonneg):
    from gsvc_amd.msssim import ssim
    X, Y = _pair(shape, 3)
    got = ssim(X.to(cuda), Y.to(cuda), data_range=1, size_average=avg, win_size=win,
               nonnegative_ssim=nonneg)
    ref = oracle.ssim(X.numpy(), Y.numpy(), 1.0, size_average=avg, win_size=win,
                      nonnegative_ssim=nonneg)
    np.testing.assert_allclose(got.cpu().double().numpy(), ref, rtol=0, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,win,avg", [((1, 3, 176, 200), 11, True),
                                           ((2, 3, 161, 171), 11, False),
                                           ((1, 3, 97, 71), 5, True),
                                           ((1, 3, 1080, 1920), 11, True)])
def test_ms_ssim_matches_oracle(cuda, oracle, shape, win, avg):
    from gsvc_amd.msssim import ms_ssim
    X, Y = _pair(shape, 4)
    got = ms_ssim(X.to(cuda), Y.to(cuda), data_range=1, size_average=avg, win_size=win)
    ref = oracle.ms_ssim(X.numpy(), Y.numpy(), 1.0, size_average=avg, win_size=win)
    np.testing.assert_allclose(got.cpu().double().numpy(), ref, rtol=0, atol=2e-5)


def _grad_close(got, ref, tol=1e-3):
    scale = float(ref.abs().max())
    err = float((got - ref).abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("multi,shape,win", [(False, (2, 3, 45, 70), 11), (False, (1, 3, 9, 33), 11),
                                             (True, (1, 3, 176, 200), 11),
                                             (True, (2, 3, 161, 171), 11), (True, (1, 3, 97, 71), 5)])
def test_gradients_match_torch_autograd(cuda, multi, shape, win):
    from gsvc_amd.msssim import ms_ssim, ssim
    X, Y = _pair(shape, 5)
    X, Y = X.to(cuda), Y.to(cuda)
    xa, ya = X.clone().requires_grad_(True), Y.clone().requires_grad_(True)
    xr, yr = X.clone().requires_grad_(True), Y.clone().requires_grad_(True)
    if multi:
        a = ms_ssim(xa, ya, data_range=1, win_size=win, size_average=False)
        r = t_ms_ssim(xr, yr, win_size=win, size_average=False)
    else:
        a = ssim(xa, ya, data_range=1, win_size=win, size_average=False)
        r = t_ssim(xr, yr, win_size=win, size_average=False)
    w = torch.linspace(0.5, 1.5, a.numel(), device=cuda)  # distinct per-image upstream
    (a * w).sum().backward()
    (r * w).sum().backward()
    _grad_close(xa.grad, xr.grad)
    _grad_close(ya.grad, yr.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("loss_type", ["SSIM", "Fusion1", "Fusion2", "Fusion4", "Fusion_hinerv"])
def test_loss_fn_ssim_variants(cuda, loss_type):
    from gsvc_amd.frame import loss_fn
    X, Y = _pair((1, 3, 180, 200), 6)
    pa = X.to(cuda).requires_grad_(True)
    pr = X.to(cuda).requires_grad_(True)
    gt = Y.to(cuda)
    la = loss_fn(pa, gt, loss_type, lambda_value=0.7)
    lam = 0.7
    if loss_type == "SSIM":
        lr = 1 - t_ssim(pr, gt)
    elif loss_type == "Fusion1":
        lr = lam * F.mse_loss(pr, gt) + (1 - lam) * (1 - t_ssim(pr, gt))
    elif loss_type == "Fusion2":
        lr = lam * F.l1_loss(pr, gt) + (1 - lam) * (1 - t_ssim(pr, gt))
    elif loss_type == "Fusion4":
        lr = lam * F.l1_loss(pr, gt) + (1 - lam) * (1 - t_ms_ssim(pr, gt))
    else:
        lr = lam * F.l1_loss(pr, gt) + (1 - lam) * (1 - t_ms_ssim(pr, gt, win_size=5))
    la.backward()
    lr.backward()
    assert abs(float(la) - float(lr)) < 2e-5
    _grad_close(pa.grad, pr.grad)
