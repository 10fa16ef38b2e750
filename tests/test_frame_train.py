"""The caller of the hot path: GaussianVideoFrame (frame.py) against the
reference GaussianVideo_frame (GaussianSplats_Represent.py:11-221) fixture
``train_iter_64x64_n200`` -- the reference model's own forward, L2 loss,
backward and two train_iter steps with its Adan (optimizer.py:39-362), run on
CPU with the oracle as its kernels (tests/golden/make_golden.py).

Bars: render within 1e-5 abs, loss within 1e-6 rel, parameter gradients within
1e-4 (abs + rel, north_star), parameters after each Adan step within 2e-6 abs
(an Adan step moves them by ~lr = 1e-3).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

FIX = "train_iter_64x64_n200"


def _load_init(model, z, prefix="init_"):
    sd = model.state_dict()
    new = {}
    for k in sd:
        new[k] = torch.from_numpy(z[prefix + k]).to(sd[k].device)
    model.load_state_dict(new)


def test_adan_step_matches_reference_cpu():
    """The foreach Adan checker (tests/adan_checker.py, what the fused kernel
    is held to) vs the reference's first Adan step, on CPU: same init, same
    gradients."""
    from adan_checker import ForeachAdan
    z = load_golden(FIX)
    names = ["_xyz", "_cholesky", "_features_dc"]
    params = [torch.nn.Parameter(torch.from_numpy(z["init_" + k].copy())) for k in names]
    opt = ForeachAdan(params, lr=1e-3)
    for p, k in zip(params, names):
        p.grad = torch.from_numpy(z["grad_" + k].copy())
    opt.step()
    for p, k in zip(params, names):
        np.testing.assert_allclose(p.detach().numpy(), z["step1_" + k], rtol=0, atol=2e-6,
                                   err_msg=k)


@pytest.mark.gpu
def test_train_iter_matches_reference(cuda):
    from gsvc_amd.frame import loss_fn, make_frame_model
    z = load_golden(FIX)
    H, W = int(z["H"]), int(z["W"])
    model = make_frame_model(H, W, z["init__xyz"].shape[0], cuda, seed=0)
    _load_init(model, z)
    model.update_optimizer()
    gt = torch.from_numpy(z["gt"]).to(cuda)

    img = model()["render"]
    np.testing.assert_allclose(img.detach().cpu().numpy(), z["render0"], rtol=0, atol=1e-5)
    loss0 = loss_fn(img.squeeze(0), gt.squeeze(0), "L2", lambda_value=0)
    np.testing.assert_allclose(float(loss0), float(z["loss0"]), rtol=1e-6)
    loss0.backward()
    for k, p in model.named_parameters():
        if "grad_" + k in z:
            g = p.grad.detach().cpu().numpy()
            ref = z["grad_" + k]
            np.testing.assert_allclose(g, ref, rtol=1e-4, atol=1e-4 * max(1.0, np.abs(ref).max()),
                                       err_msg=k)
    model.optimizer.zero_grad(set_to_none=True)

    for it in (1, 2):
        loss, psnr = model.train_iter(gt, it)
        np.testing.assert_allclose(float(loss), z["losses"][it - 1], rtol=1e-5)
        np.testing.assert_allclose(psnr, z["psnrs"][it - 1], rtol=1e-5)
        sd = model.state_dict()
        for k in ("_xyz", "_cholesky", "_features_dc"):
            np.testing.assert_allclose(sd[k].cpu().numpy(), z[f"step{it}_" + k], rtol=0,
                                       atol=2e-6, err_msg=f"step{it} {k}")


@pytest.mark.gpu
def test_train_iter_fused_render_agrees(cuda):
    """After training steps, the inference render (fused frame entry) equals
    the autograd forward the training used."""
    from gsvc_amd.frame import make_frame_model
    z = load_golden(FIX)
    H, W = int(z["H"]), int(z["W"])
    model = make_frame_model(H, W, z["init__xyz"].shape[0], cuda, seed=0)
    _load_init(model, z)
    model.update_optimizer()
    gt = torch.from_numpy(z["gt"]).to(cuda)
    for it in (1, 2, 3):
        model.train_iter(gt, it)
    with torch.no_grad():
        fast = model()["render"]
    assert torch.equal(fast, model()["render"].detach())
