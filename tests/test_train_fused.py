"""GPU parity of the fused training step (gsvc_train_step_sum, train.hip).

Against GSVC's op-by-op iteration (GaussianSplats_Represent.py:191-207 on the
parity-tested ops: forward, clamp, L2 / L1 loss, autograd backward, Adan):

* the fused step's clamped render is bit-identical to the autograd forward;
* its loss is the torch loss (rtol 1e-5: reduction order only);
* its parameter gradients (test hook ``grads_out``) match autograd within
  north_star's 1e-4 (abs + rel, with ``v_out`` of a real loss: gradient sums
  differ by atomic order only);
* trajectories of fused and op-by-op training agree (and the reference
  fixture's two train_iter steps are met by the fused path);
* tiles with more than 256 entries, an empty frame (M = 0: background, no
  gradient), a trainable rgb_W and densify iterations (op-by-op) interleaved
  with fused ones.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import knobs, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["band", "wg256"])
def tile_kernel(request, cuda):
    """The fused step's tile kernel: two 8-row band waves per tile (production)
    or the 256-thread workgroup per tile (gsvc_debug_set(8, 1), A/B)."""
    with knobs((8, 1 if request.param == "wg256" else 0)):
        yield request.param


def _model(H, W, n, dev, seed, chol_scale=1.0, **kw):
    from gsvc_amd.frame import make_frame_model
    m = make_frame_model(H, W, n, dev, seed=seed, **kw)
    if chol_scale != 1.0:
        with torch.no_grad():
            m._cholesky.mul_(chol_scale)
            m._cholesky.add_(m.cholesky_bound * (chol_scale - 1.0))
    return m


def _autograd(model, gt, loss_type):
    from gsvc_amd.frame import loss_fn
    model.fused_train = False
    img = model()["render"]
    loss = loss_fn(img.squeeze(0), gt.squeeze(0), loss_type, lambda_value=0)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    mse = float(F.mse_loss(img.detach(), gt))
    model.optimizer.zero_grad(set_to_none=True)
    return img.detach(), float(loss), mse, grads


def _fused_grads(model, gt, loss_type):
    from gsvc_amd.train import train_step_sum
    n, H, W = model._xyz.shape[0], model.H, model.W
    g = torch.empty((n, 9), device=gt.device)
    render = torch.empty((1, 3, H, W), device=gt.device)
    rgbw_train = isinstance(model.rgb_W, torch.nn.Parameter)
    losses = train_step_sum(model._xyz.data, model._cholesky.data, model._features_dc.data,
                            model.rgb_W.data, rgbw_train, model.cholesky_bound, model.background,
                            gt.contiguous(), H, W, loss_type, render_out=render, grads_out=g)
    return render, losses, g


def _close(a, ref, name):
    a = a.detach().cpu().numpy()
    ref = ref.detach().cpu().numpy()
    scale = max(1.0, float(np.abs(ref).max()))
    np.testing.assert_allclose(a, ref, rtol=1e-4, atol=1e-4 * scale, err_msg=name)


CASES = [(64, 64, 200, 1.0), (72, 120, 500, 1.0), (1080, 1920, 10000, 1.0),
         (1080, 1920, 50000, 1.0), (256, 256, 3000, 8.0), (37, 53, 150, 1.0), (17, 33, 60, 2.0)]


@pytest.mark.parametrize("H,W,n,chol", CASES)
@pytest.mark.parametrize("loss_type", ["L2", "L1"])
def test_fused_step_matches_autograd(cuda, tile_kernel, H, W, n, chol, loss_type):
    from gsvc_amd.frame import synthetic_gt
    model = _model(H, W, n, cuda, seed=n + 3, chol_scale=chol, isremoval=True)
    gt = synthetic_gt(H, W, 11, cuda)
    render, losses, g = _fused_grads(model, gt, loss_type)
    img, loss, mse, grads = _autograd(model, gt, loss_type)
    assert torch.equal(render, img)
    np.testing.assert_allclose(float(losses[0]), mse, rtol=1e-5)
    np.testing.assert_allclose(float(losses[1 if loss_type == "L1" else 0]), loss, rtol=1e-5)
    # (the magnitude of an L2 gradient is ~1 / numel; compare relative to it)
    sc = 1.0 / max(float(g.abs().max()), 1e-30)
    _close(g[:, 0:2] * sc, grads["_xyz"] * sc, "_xyz")
    _close(g[:, 2:5] * sc, grads["_cholesky"] * sc, "_cholesky")
    _close(g[:, 5:8] * sc, grads["_features_dc"] * sc, "_features_dc")
    _close(g[:, 8:9] * sc, grads["rgb_W"] * sc, "rgb_W")


def test_fused_step_overfull_tiles(cuda, tile_kernel):
    """Tiles with more than 256 entries (the slab overflow rebuild), ids spread
    over the whole range: 1500 splats piled on one spot."""
    from gsvc_amd.frame import synthetic_gt
    H, W, n = 64, 64, 6000
    model = _model(H, W, n, cuda, seed=5)
    with torch.no_grad():
        sel = torch.arange(0, n, 4, device=cuda)
        model._xyz[sel] = torch.atanh(torch.full((len(sel), 2), -0.25, device=cuda)
                                      + 0.05 * torch.rand(len(sel), 2, device=cuda))
        model._cholesky[sel] = torch.tensor([2.5, 0.3, 1.5], device=cuda)
    gt = synthetic_gt(H, W, 2, cuda)
    render, losses, g = _fused_grads(model, gt, "L2")
    img, loss, mse, grads = _autograd(model, gt, "L2")
    assert torch.equal(render, img)
    sc = 1.0 / float(g.abs().max())
    _close(g[:, 0:2] * sc, grads["_xyz"] * sc, "_xyz")
    _close(g[:, 2:5] * sc, grads["_cholesky"] * sc, "_cholesky")
    _close(g[:, 5:8] * sc, grads["_features_dc"] * sc, "_features_dc")


def test_fused_step_empty_frame(cuda, tile_kernel):
    """Every splat degenerate (L = 0): M = 0, the image is the background and
    no gradient flows (rasterize_sum.py:121-129)."""
    from gsvc_amd.frame import synthetic_gt
    H, W, n = 40, 56, 300
    model = _model(H, W, n, cuda, seed=6)
    with torch.no_grad():
        model._cholesky.copy_(-model.cholesky_bound.expand(n, 3))
        model.background.copy_(torch.tensor([0.25, 1.5, -0.5], device=cuda))
    gt = synthetic_gt(H, W, 3, cuda)
    render, losses, g = _fused_grads(model, gt, "L2")
    img, loss, mse, grads = _autograd(model, gt, "L2")
    assert torch.equal(render, img)
    np.testing.assert_array_equal(img[0, :, 0, 0].cpu().numpy(), [0.25, 1.0, 0.0])
    np.testing.assert_allclose(float(losses[0]), mse, rtol=1e-6)
    assert float(g.abs().max()) == 0.0


def test_fused_training_trajectory(cuda):
    """15 iterations fused vs op-by-op from one init (trainable rgb_W)."""
    from gsvc_amd.frame import synthetic_gt
    H, W, n = 144, 176, 2000
    a = _model(H, W, n, cuda, seed=9, isremoval=True, fused_train=True)
    b = _model(H, W, n, cuda, seed=9, isremoval=True, fused_train=False)
    b.load_state_dict(a.state_dict())
    gt = synthetic_gt(H, W, 4, cuda)
    for it in range(1, 16):
        if it % a.densification_interval == 0:
            continue
        la, pa = a.train_iter(gt, it)
        lb, pb = b.train_iter(gt, it)
        np.testing.assert_allclose(float(la), float(lb), rtol=1e-4)
        assert math.isclose(pa, pb, rel_tol=1e-5)
    assert a.fused_steps == 15 and b.fused_steps == 0
    for k, v in a.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), b.state_dict()[k].cpu().numpy(), rtol=0,
                                   atol=2e-5, err_msg=k)
    for pa_, pb_ in zip(a.optimizer.param_groups[0]["params"], b.optimizer.param_groups[0]["params"]):
        for key in ("exp_avg", "exp_avg_sq", "exp_avg_diff", "neg_pre_grad"):
            sa, sb = a.optimizer.state[pa_][key], b.optimizer.state[pb_][key]
            scale = float(sb.abs().max()) + 1e-30
            np.testing.assert_allclose((sa / scale).cpu().numpy(), (sb / scale).cpu().numpy(),
                                       rtol=0, atol=1e-3, err_msg=key)


def test_fused_path_meets_reference_fixture(cuda):
    """The reference's own two train_iter steps (tests/golden/make_golden.py)
    through the fused path."""
    from gsvc_amd.frame import make_frame_model
    z = load_golden("train_iter_64x64_n200")
    H, W = int(z["H"]), int(z["W"])
    model = make_frame_model(H, W, z["init__xyz"].shape[0], cuda, seed=0)
    sd = model.state_dict()
    model.load_state_dict({k: torch.from_numpy(z["init_" + k]).to(cuda) for k in sd})
    model.update_optimizer()
    gt = torch.from_numpy(z["gt"]).to(cuda)
    for it in (1, 2):
        loss, psnr = model.train_iter(gt, it)
        np.testing.assert_allclose(float(loss), z["losses"][it - 1], rtol=1e-5)
        np.testing.assert_allclose(psnr, z["psnrs"][it - 1], rtol=1e-5)
        for k in ("_xyz", "_cholesky", "_features_dc"):
            np.testing.assert_allclose(model.state_dict()[k].cpu().numpy(), z[f"step{it}_" + k],
                                       rtol=0, atol=2e-6, err_msg=f"step{it} {k}")
    assert model.fused_steps == 2


def test_densify_iterations_interleave(cuda):
    """P-frame densify/prune iterations (adaptive_control) run op by op, the
    rest fused; the run equals an all-op-by-op run from the same seeds."""
    from gsvc_amd.frame import synthetic_gt
    H, W, n = 96, 128, 1500
    gt = synthetic_gt(H, W, 7, cuda)
    runs = []
    for fused in (True, False):
        m = _model(H, W, n, cuda, seed=12, isdensity=True, densification_interval=4,
                   fused_train=fused)
        torch.manual_seed(99)
        for it in range(1, 10):
            m.train_iter(gt, it)
        runs.append(m)
    a, b = runs
    assert a.fused_steps > 0 and b.fused_steps == 0
    assert a._xyz.shape == b._xyz.shape
    for k, v in a.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), b.state_dict()[k].cpu().numpy(), rtol=0,
                                   atol=2e-5, err_msg=k)


@pytest.mark.parametrize("mode,it", [("removal", 400), ("removal", 4000), ("removal", 4100),
                                     ("densify", 1), ("densify", 600), ("densify", 1000),
                                     ("densify", 300)])
def test_control_iterations_match_op_path(cuda, mode, it):
    """A prune / densify iteration (removal_control / adaptive_control) of the
    fused model -- forward only when the control swaps in new Parameters --
    leaves the same parameters, loss, PSNR, Adan step count and lr as the
    op-by-op iteration (forward + backward + control + step); the next
    (fused vs op-by-op) iteration then agrees too."""
    from gsvc_amd.frame import synthetic_gt
    H, W, n = 96, 128, 1500
    gt = synthetic_gt(H, W, 3, cuda)
    kw = dict(isremoval=mode == "removal", isdensity=mode == "densify", densification_interval=100,
              max_num_points=n, removal_rate=0.1)
    a = _model(H, W, n, cuda, seed=21, fused_train=True, **kw)
    b = _model(H, W, n, cuda, seed=21, fused_train=False, **kw)
    b.load_state_dict(a.state_dict())
    for m in (a, b):  # one ordinary step first, so Adan has state to lose or keep
        m.train_iter(gt, 2)
    outs = []
    for m in (a, b):
        torch.manual_seed(5)
        loss, psnr = m.train_iter(gt, it)
        outs.append((float(loss), psnr))
    assert outs[0][0] == outs[1][0] and outs[0][1] == outs[1][1]
    assert a._xyz.shape == b._xyz.shape
    for k, v in a.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), b.state_dict()[k].cpu().numpy(), rtol=0,
                                   atol=2e-5, err_msg=k)
    assert a.optimizer.param_groups[0]["step"] == b.optimizer.param_groups[0]["step"]
    assert a.optimizer.param_groups[0]["lr"] == b.optimizer.param_groups[0]["lr"]
    la, _ = a.train_iter(gt, it + 1)
    lb, _ = b.train_iter(gt, it + 1)
    np.testing.assert_allclose(float(la), float(lb), rtol=1e-5)
    for k, v in a.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), b.state_dict()[k].cpu().numpy(), rtol=0,
                                   atol=2e-5, err_msg=k)
