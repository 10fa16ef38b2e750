"""BASELINE configs[2] at the state bench.py times ("pin the timed
state"): the bench's 1920x1080 / 50k frame (seed 1000, target seed 8) after
its 2000 settle + 20 warmup iterations -- trained density, M ~ 240k entries,
~30 per tile, the regime of the timed steps (more than 32 speculative slab
records, the dense-tile staging, the lane-group lists at their trained
occupancy).

Fixture ``train_state_1080p_n50k`` (tests/golden/make_golden.py ``trained``):
the state was trained on the CPU by the oracle's train_iter_sum
(tests/analysis/train_oracle_state.py); from it the reference's own Python
(GaussianSplats_Represent.py:83-90,191-207, gsplat glue, Adan; oracle kernels
injected, fresh optimizer) recorded the render (checksums + crops), the L2
loss, the parameter gradients and three train_iter steps.

CPU: the oracle reproduces the fixture (it is the fixture's kernels; this pins
the restated glue at trained density).
GPU: the fused step (gsvc_train_step_sum), the op path (GSVC's own autograd
through gsplat.*) and the render, held to the fixture and to the oracle on the
same inputs:
* render: against the oracle on the GPU's own activated inputs within 1e-5
  (v_exp_f32 vs exp2f); the fixture's crops within 1e-4
  (tanh on the GPU vs torch-CPU tanh moves centres by ~1e-4 px);
* loss within 2e-6 relative, PSNR within 1e-4 dB;
* gradients within 1e-4 of each parameter's largest gradient (north_star's
  1e-4, relative, since L2 gradients are ~1 / numel) against the oracle on
  the GPU's own activations; against the reference fixture within the
  envelope that a 1-ulp change of tanh produces in the reference's own
  arithmetic (_envelope: the gradient is discontinuous in the centres at
  trained density);
* the op path's rasterize_sum_backward against oracle.raster_sum_backward at
  full size, v_out ~ N(0, 1), same tolerance;
* three train_iter steps (a fresh Adan, as a P-frame's): step 1 as above;
  steps 2-3 within STEP_PSNR_TOL, the envelope the reference's own arithmetic
  shows under a 1-ulp tanh change; parameters by the trajectory test's
  quantile bars (Adan normalises near-zero gradient sums).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

FIX = "train_state_1080p_n50k"
H, W = 1080, 1920
# PSNR bar for train_iter steps 2 and 3 from the fixture (step 1 is held to
# 1e-4 dB): a fresh Adan moves every element by ~lr * sign(gradient), so an
# element whose gradient sign flips with a last-bit change of the inputs moves
# the other way; with the reference's own arithmetic and numpy's tanh in place
# of torch's the PSNR moves by 1.5e-4 and 9.5e-4 dB (test_oracle_reproduces_fixture)
STEP_PSNR_TOL = 2e-3


def _z():
    return load_golden(FIX)


def _gt(z, device):
    from gsvc_amd.frame import synthetic_gt
    return synthetic_gt(H, W, int(z["gt_seed"]), "cpu").to(device)


def _state_model(z, device, fused=True):
    from gsvc_amd.frame import make_frame_model
    n = int(z["n"])
    m = make_frame_model(H, W, n, device, seed=0, fused_train=fused)
    with torch.no_grad():
        for k in ("_xyz", "_cholesky", "_features_dc"):
            getattr(m, k).copy_(torch.from_numpy(z["state_" + k]))
    return m


def _rel_close(a, ref, name, tol=1e-4):
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = float(np.abs(ref).max())
    err = float(np.abs(a - ref).max())
    assert err <= tol * scale, f"{name}: max |gpu - ref| = {err:.3e} > {tol} * {scale:.3e}"
    return err / scale


def _crops(img_chw, z):
    return np.stack([img_chw[:, y:y + 16, x:x + 16] for y, x in z["crops"]])


# ---------------------------------------------------------------- CPU


def test_fixture_is_trained_density():
    z = _z()
    assert int(z["n"]) == 50000 and int(z["iters"]) == 2020
    # random init has M ~ 124k; the settled frame about twice that
    assert int(z["M"]) > 200000
    # a settled frame (bench.py's timed steps run at ~30 dB); the three steps
    # start a fresh Adan, as a P-frame does (train_video_Represent.py:364-366)
    assert 10 * np.log10(1 / float(z["loss0"])) > 25.0
    assert z["losses"].shape == (3,) and abs(z["losses"][0] - float(z["loss0"])) < 1e-12


def test_oracle_reproduces_fixture(oracle):
    """The oracle's forward / backward / train_iter on the state, with the
    fixture's own activations recomputed in numpy float32: render crops, loss
    and gradients (the fixture ran the same kernels under the reference glue;
    torch-CPU tanh vs numpy tanh is the only difference)."""
    z = _z()
    oracle.set_threads(8)
    try:
        params = {k: np.array(z["state_" + k], copy=True) for k in ("_xyz", "_cholesky",
                                                                      "_features_dc")}
        means = np.tanh(params["_xyz"]).astype(np.float32)
        L = (params["_cholesky"] + np.array([0.5, 0.0, 0.5], np.float32)).astype(np.float32)
        r = oracle.render_sum(means, L, params["_features_dc"], np.ones((50000, 1), np.float32), H, W)
        assert abs(r["m"] - int(z["M"])) <= 8
        img = np.clip(r["out"], 0, 1).transpose(2, 0, 1)
        np.testing.assert_allclose(_crops(img, z), z["render_crops"], rtol=0, atol=1e-4)
        np.testing.assert_allclose(img.astype(np.float64).sum(axis=(1, 2)), z["render_sum"],
                                   rtol=2e-6)
        gt = _gt(z, "cpu").numpy()[0]
        state = {}
        # the fixture's optimizer is fresh: Adan steps 1, 2, 3 (its own count)
        out = [oracle.train_iter_sum(params, gt, H, W, state, k + 1) for k in range(3)]
        losses, psnrs = np.array([o[0] for o in out]), np.array([o[1] for o in out])
        assert abs(losses[0] - z["losses"][0]) <= 2e-6 * z["losses"][0]
        assert abs(psnrs[0] - z["psnrs"][0]) <= 1e-4
        # the envelope of STEP_PSNR_TOL: numpy's tanh differs from torch's by an
        # ulp in a third of the centres; the fresh Adan's sign-normalised first
        # steps then move the PSNR by ~1e-3 dB (measured 1.5e-4, 9.5e-4)
        d = np.abs(psnrs - z["psnrs"])
        assert d[1:].max() <= STEP_PSNR_TOL, d
    finally:
        oracle.set_threads(1)


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
def test_trained_render_matches_oracle(cuda, oracle):
    """GaussianVideoFrame.forward (the fused frame render) and the op path's
    forward at trained density against the oracle on the same activations."""
    z = _z()
    m = _state_model(z, cuda)
    m.eval()
    with torch.no_grad():
        img = m()["render"][0].cpu().numpy()
        means = m.get_xyz.cpu().numpy()
        L = m.get_cholesky_elements.cpu().numpy()
        colors = m.get_features.cpu().numpy()
    oracle.set_threads(8)
    try:
        r = oracle.render_sum(means, L, colors, np.ones((len(means), 1), np.float32), H, W)
    finally:
        oracle.set_threads(1)
    ref = np.clip(r["out"], 0, 1).transpose(2, 0, 1)
    np.testing.assert_allclose(img, ref, rtol=0, atol=1e-5)
    np.testing.assert_allclose(_crops(img, z), z["render_crops"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(img.astype(np.float64).sum(axis=(1, 2)), z["render_sum"], rtol=2e-6)
    # the op path (autograd forward, GSVC's own files' route) gives the same bits
    m.fused_train = False
    m.train()
    with torch.no_grad():
        img_op = m()["render"][0].cpu().numpy()
    np.testing.assert_array_equal(img_op, img)


def _envelope(a, ref, name):
    """Against the reference fixture: the tanh of the GPU (ocml) and of
    torch-CPU differ by an ulp in a third of the centres, and at trained
    density the gradient is discontinuous in the centre (the alpha >= 1/255
    cut and the 3-sigma bbox truncation, forward.cu:600-606, helpers.cuh:
    27-43), so single elements move by up to 4.1e-3 of the largest and the
    99.9th percentile by 5.4e-4 -- measured with the reference's own
    arithmetic, the oracle fed numpy's tanh instead of torch's.
    Bars: max 1e-2, 99.9th percentile 1e-3 of the largest."""
    e = np.abs(np.asarray(a, np.float64) - ref)
    sc = float(np.abs(ref).max())
    assert e.max() <= 1e-2 * sc and np.percentile(e, 99.9) <= 1e-3 * sc, (
        name, e.max() / sc, np.percentile(e, 99.9) / sc)
    return e.max() / sc


def _oracle_grads(m, gt):
    """The oracle's gradients (train_grads_sum) on the model's own activated
    parameters as the GPU computed them: the kernel-parity reference."""
    import oracle as O
    with torch.no_grad():
        means = m.get_xyz.cpu().numpy()
        L = m.get_cholesky_elements.cpu().numpy()
        colors = m.get_features.cpu().numpy()
    O.set_threads(8)
    try:
        loss, img, vm, vL, vc = O.train_grads_sum(means, L, colors, gt.cpu().numpy()[0], H, W)
    finally:
        O.set_threads(1)
    return loss, img, dict(_xyz=(vm * (1.0 - means * means)).astype(np.float32), _cholesky=vL,
                           _features_dc=vc)


@pytest.mark.gpu
def test_trained_fused_step_matches_reference(cuda):
    """gsvc_train_step_sum on the settled state (gradients only): its render,
    loss and parameter gradients against the oracle on the same activations
    (1e-4 of the largest gradient) and against the reference's own
    forward / backward (the envelope of a 1-ulp tanh change, _envelope)."""
    from gsvc_amd.train import train_step_sum
    z = _z()
    m = _state_model(z, cuda)
    gt = _gt(z, cuda)
    n = int(z["n"])
    g = torch.empty((n, 9), device=cuda)
    render = torch.empty((1, 3, H, W), device=cuda)
    losses = train_step_sum(m._xyz.data, m._cholesky.data, m._features_dc.data, m.rgb_W.data, False,
                            m.cholesky_bound, m.background, gt.contiguous(), H, W, "L2",
                            render_out=render, grads_out=g)
    mse = float(losses[0])
    assert abs(mse - float(z["loss0"])) <= 2e-6 * float(z["loss0"])
    assert abs(10 * np.log10(1 / mse) - 10 * np.log10(1 / float(z["loss0"]))) <= 1e-4
    img = render[0].cpu().numpy()
    np.testing.assert_allclose(_crops(img, z), z["render_crops"], rtol=0, atol=1e-4)
    oloss, oimg, og = _oracle_grads(m, gt)
    np.testing.assert_allclose(img, oimg, rtol=0, atol=1e-5)
    assert abs(mse - oloss) <= 1e-6 * oloss
    gn = g.cpu().numpy()
    cols = dict(_xyz=slice(0, 2), _cholesky=slice(2, 5), _features_dc=slice(5, 8))
    errs = {}
    for k, sl in cols.items():
        errs[k] = (_rel_close(gn[:, sl], og[k], k), _envelope(gn[:, sl], z["grad_" + k], k))
    print("fused-step gradients, max err / largest (vs oracle, vs reference):", errs)


@pytest.mark.gpu
def test_trained_op_path_gradients_match_reference(cuda):
    """GSVC's own route -- autograd through gsplat.project_gaussians_2d /
    rasterize_gaussians_sum (forward, clamp, F.mse_loss, backward) -- at the
    settled state, against the oracle on the same activations and the
    reference's gradients."""
    from gsvc_amd.frame import loss_fn
    z = _z()
    m = _state_model(z, cuda, fused=False)
    gt = _gt(z, cuda)
    img = m()["render"]
    loss = loss_fn(img.squeeze(0), gt.squeeze(0), "L2", lambda_value=0)
    loss.backward()
    assert abs(float(loss) - float(z["loss0"])) <= 2e-6 * float(z["loss0"])
    _, _, og = _oracle_grads(m, gt)
    for k in ("_xyz", "_cholesky", "_features_dc"):
        gk = getattr(m, k).grad.cpu().numpy()
        _rel_close(gk, og[k], k)
        _envelope(gk, z["grad_" + k], k)


@pytest.mark.gpu
def test_trained_raster_backward_matches_oracle(cuda, oracle):
    """The op path's rasterize_sum_backward (backward.cu:696-862) at the settled
    state's full size against oracle.raster_sum_backward on identical inputs
    (the GPU's projection and binning, which are bit-exact), v_out ~ N(0, 1)."""
    from gsvc_amd import ops
    from gsvc_amd.utils import bin_and_sort_for_raster
    z = _z()
    m = _state_model(z, cuda)
    tb = m.tile_bounds
    with torch.no_grad():
        means, L, colors = m.get_xyz, m.get_cholesky_elements, m.get_features
        n = means.shape[0]
        xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, means, L, H, W, tb, 0.01)
        M, gids, bins = bin_and_sort_for_raster(n, xys, depths, radii, nth, tb)
        opac = torch.ones((n, 1), device=cuda)
        bg = torch.ones(3, device=cuda)
        _, _, idx = ops.rasterize_sum_forward(tb, (16, 16, 1), (W, H, 1), gids, bins, xys, conics,
                                              colors, opac, bg)
        v = torch.randn((H, W, 3), device=cuda, generator=torch.Generator(cuda).manual_seed(3))
        g = ops.rasterize_sum_backward(H, W, 16, 16, gids, bins, xys, conics, colors, opac, bg,
                                       None, idx, v, None)
    assert int(M) > 200000
    Np = lambda t: t.detach().cpu().numpy()  # noqa: E731
    bins_n = Np(bins)
    oracle.set_threads(8)
    try:
        ref = oracle.raster_sum_backward(tb, H, W, Np(gids), bins_n, Np(xys), Np(conics), Np(colors),
                                         Np(opac), Np(idx), Np(v))
    finally:
        oracle.set_threads(1)
    for a, b, nm in zip(g[:3], ref[:3], ("v_xy", "v_conic", "v_colors")):
        _rel_close(Np(a), b, nm)


def _check_params(model, z):
    keep = z["final__xyz"].shape[0]
    for k in ("_xyz", "_cholesky", "_features_dc"):
        p = getattr(model, k).detach().cpu().numpy()
        e = np.abs(p[:keep].astype(np.float64) - z["final_" + k])
        q50, q90, q99 = np.percentile(e, [50, 90, 99])
        assert q50 <= 1e-6 and q90 <= 2e-5 and q99 <= 2e-3 and e.max() <= 5e-2, (k, q50, q90, q99,
                                                                                  e.max())
        assert abs(p.astype(np.float64).sum() - z["sum_" + k]) <= 1e-5 * z["abssum_" + k], k


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
def test_trained_train_iter_steps_match_reference(cuda, fused):
    """Three GaussianVideoFrame.train_iter steps from the settled state (fresh
    Adan, as the fixture) on the fused step and on the op-by-op path."""
    z = _z()
    m = _state_model(z, cuda, fused=fused)
    gt = _gt(z, cuda)
    it0 = int(z["iters"])
    losses, psnrs = [], []
    for k in range(len(z["losses"])):
        loss, psnr = m.train_iter(gt, it0 + 1 + k)
        losses.append(float(loss))
        psnrs.append(psnr)
    assert m.fused_steps == (len(losses) if fused else 0)
    assert abs(psnrs[0] - z["psnrs"][0]) <= 1e-4
    assert abs(losses[0] - z["losses"][0]) <= 2e-6 * z["losses"][0]
    np.testing.assert_allclose(psnrs[1:], z["psnrs"][1:], rtol=0, atol=STEP_PSNR_TOL)
    np.testing.assert_allclose(losses[1:], z["losses"][1:], rtol=1e-3, atol=0)
    _check_params(m, z)
