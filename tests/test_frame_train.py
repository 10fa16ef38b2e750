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
    """The foreach Adan checker (tools/foreach_adan.py, what the fused kernel
    is held to) vs the reference's first Adan step, on CPU: same init, same
    gradients."""
    from foreach_adan import ForeachAdan
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


def _ahead_run(cuda, ahead, edits):
    """20 fused train_iter steps at 256x256 / 2000 splats with the next step's
    projection enqueued ahead (or not); ``edits`` maps step -> an in-place change
    of the parameters made between two steps."""
    from gsvc_amd import train as Tr
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    old = Tr.PROJECT_AHEAD
    Tr.PROJECT_AHEAD = ahead
    try:
        model = make_frame_model(256, 256, 2000, cuda, seed=3)
        gt = synthetic_gt(256, 256, 4, cuda)
        losses = []
        for it in range(1, 21):
            if it in edits:
                edits[it](model)
            loss, _ = model.train_iter(gt, it)
            losses.append(float(loss))
        assert model.fused_steps == 20
        return np.array(losses), model._xyz.detach().clone()
    finally:
        Tr.PROJECT_AHEAD = old


def test_projection_ahead_per_parameter_set(cuda):
    """Two models training interleaved on two streams keep their projections
    ahead (launches are counted per parameter set), and
    each trajectory is bitwise the one it has alone (deterministic backward)."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    prev = torch.are_deterministic_algorithms_enabled()
    prev_warn = torch.is_deterministic_algorithms_warn_only_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        specs = [(2000, 3), (3000, 7)]
        gts = [synthetic_gt(256, 256, 4, cuda), synthetic_gt(256, 256, 5, cuda)]
        streams = [torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)]

        def run(which):
            ms = {k: make_frame_model(256, 256, specs[k][0], cuda, seed=specs[k][1]) for k in which}
            torch.cuda.synchronize()
            out = {k: [] for k in which}
            for it in range(1, 13):
                for k in which:
                    with torch.cuda.stream(streams[k]):
                        out[k].append(float(ms[k].train_iter(gts[k], it)[0]))
            torch.cuda.synchronize()
            return ms, out

        both, lb = run([0, 1])
        for k in (0, 1):
            solo, ls = run([k])
            assert lb[k] == ls[k]
            assert torch.equal(both[k]._xyz, solo[k]._xyz)
            assert torch.equal(both[k]._features_dc, solo[k]._features_dc)
            # every step after the first used the projection its predecessor enqueued
            assert both[k].fused_steps == 12 and both[k]._bound_step.ahead_steps == 11
    finally:
        torch.use_deterministic_algorithms(prev, warn_only=prev_warn)


def _tiles_run(cuda, tiles, gts, schedule, rebuild_every=None):
    """20 fused iterations with TILES_AHEAD = tiles; schedule[it] picks the
    target (an index into gts, or a callable making one); returns the losses,
    the mse each iteration should report (the render of the parameters it
    starts from against its target, computed before the call) and the model."""
    from gsvc_amd import train as Tr
    from gsvc_amd.frame import make_frame_model
    old = Tr.TILES_AHEAD, Tr.CARRY_REBUILD_EVERY
    Tr.TILES_AHEAD = tiles
    if rebuild_every is not None:
        Tr.CARRY_REBUILD_EVERY = rebuild_every
    try:
        model = make_frame_model(256, 256, 2000, cuda, seed=3)
        losses, want = [], []
        for it in range(1, 21):
            g = schedule.get(it, 0)
            gt = g() if callable(g) else gts[g]
            with torch.no_grad():
                img = model.forward()["render"]  # same bits as the fused forward
                want.append(float(torch.mean((img - gt) ** 2)))
            loss, _ = model.train_iter(gt, it)
            losses.append(float(loss))
        assert model.fused_steps == 20
        return np.array(losses), np.array(want), model
    finally:
        Tr.TILES_AHEAD, Tr.CARRY_REBUILD_EVERY = old


def test_tiles_ahead_matches_and_honours_target_changes(cuda):
    """The next iteration's tile kernel, enqueued ahead against the current
    target, gives the trajectory of launching it in its own call, and its work
    is discarded when the next call's target differs: another tensor, the same
    tensor edited in place, a fresh copy each call.  Each iteration's loss is
    the mse of the render it starts from against ITS target."""
    from gsvc_amd.frame import synthetic_gt
    gts = [synthetic_gt(256, 256, 4, cuda), synthetic_gt(256, 256, 9, cuda)]

    def schedule():  # a fresh edited target per run
        edit = gts[0].clone()

        def edited():
            edit.mul_(0.97)  # in place: same storage, new _version
            return edit

        return {6: 1, 7: 1, 8: 0, 11: edited, 12: edited, 13: edited,
                15: lambda: gts[0].clone(), 16: lambda: gts[0].clone()}

    la, wa, ma = _tiles_run(cuda, True, gts, schedule())
    lb, wb, mb = _tiles_run(cuda, False, gts, schedule())
    # each loss is its own target's (a stale tile kernel would report the old one)
    np.testing.assert_allclose(la, wa, rtol=2e-5, atol=1e-8)
    np.testing.assert_allclose(lb, wb, rtol=2e-5, atol=1e-8)
    # float atomics in the backward: equal up to their summation order
    np.testing.assert_allclose(la, lb, rtol=2e-5, atol=1e-8)
    np.testing.assert_allclose(ma._xyz.detach().cpu().numpy(), mb._xyz.detach().cpu().numpy(),
                               rtol=1e-3, atol=1e-4)
    bs = ma._bound_step
    assert mb._bound_step.tiled_steps == 0
    # tiled: an iteration whose target is its predecessor's, which in turn
    # repeated the target before it (3-5, 10, 19-20); the edited and fresh-copy
    # targets never match
    assert bs.tiled_steps == 6, bs.tiled_steps


def test_tiles_ahead_with_rebuilds_ahead(cuda):
    """Bins rebuilt every 3 steps: the rebuild is enqueued behind the step
    before it (GSVC_TRAIN_REBUILD_NEXT) together with the next tile kernel, and
    the trajectory is the one of rebuilding at the start of the call."""
    from gsvc_amd.frame import synthetic_gt
    gts = [synthetic_gt(256, 256, 4, cuda)]
    la, wa, ma = _tiles_run(cuda, True, gts, {}, rebuild_every=3)
    lb, wb, mb = _tiles_run(cuda, False, gts, {}, rebuild_every=3)
    np.testing.assert_allclose(la, wa, rtol=2e-5, atol=1e-8)
    np.testing.assert_allclose(la, lb, rtol=2e-5, atol=1e-8)
    np.testing.assert_allclose(ma._xyz.detach().cpu().numpy(), mb._xyz.detach().cpu().numpy(),
                               rtol=1e-3, atol=1e-4)
    # every step after the second takes the tile kernel its predecessor enqueued
    assert ma._bound_step.tiled_steps == 18, ma._bound_step.tiled_steps


def test_tiles_ahead_deterministic_is_bitwise(cuda):
    """Under torch.use_deterministic_algorithms(True) the tile kernel ahead
    (with its slot offsets prepared behind the step) changes nothing: the
    trajectory with and without it is bitwise identical, rebuilds included."""
    from gsvc_amd.frame import synthetic_gt
    prev = torch.are_deterministic_algorithms_enabled()
    prev_warn = torch.is_deterministic_algorithms_warn_only_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        gts = [synthetic_gt(256, 256, 4, cuda), synthetic_gt(256, 256, 9, cuda)]
        sched = {9: 1, 10: 1}
        la, _, ma = _tiles_run(cuda, True, gts, sched, rebuild_every=5)
        lb, _, mb = _tiles_run(cuda, False, gts, sched, rebuild_every=5)
        assert la.tolist() == lb.tolist()
        assert torch.equal(ma._xyz, mb._xyz) and torch.equal(ma._cholesky, mb._cholesky)
        assert torch.equal(ma._features_dc, mb._features_dc)
        assert ma._bound_step.tiled_steps >= 12, ma._bound_step.tiled_steps
    finally:
        torch.use_deterministic_algorithms(prev, warn_only=prev_warn)


def test_projection_ahead_matches_and_honours_edits(cuda):
    """The fused step's projection of the next frame, enqueued ahead, gives the
    same trajectory as projecting at the start of each step, and is discarded
    when the parameters change in between: an in-place op through the
    Parameter (its _version), a write through .data announced with
    bump_param_epoch, and an optimizer step of the op path."""
    from gsvc_amd.train import bump_param_epoch

    def via_param(m):
        with torch.no_grad():
            m._xyz.add_(0.02)

    def via_data(m):
        m._xyz.data.mul_(0.99)
        bump_param_epoch()

    def via_optimizer(m):
        m._features_dc.grad = torch.full_like(m._features_dc, 0.1)
        m.optimizer.step()
        m.optimizer.zero_grad(set_to_none=True)

    edits = {6: via_param, 11: via_data, 16: via_optimizer}
    la, xa = _ahead_run(cuda, True, dict(edits))
    lb, xb = _ahead_run(cuda, False, dict(edits))
    # float atomics in the backward: equal up to their summation order
    np.testing.assert_allclose(la, lb, rtol=2e-5, atol=1e-8)
    np.testing.assert_allclose(xa.cpu().numpy(), xb.cpu().numpy(), rtol=1e-3, atol=1e-4)
    # the edits matter: without them the trajectory differs clearly
    lc, _ = _ahead_run(cuda, True, {})
    assert np.abs(lc[6:] - la[6:]).max() > 1e-4


def test_pending_work_released_with_its_model(cuda):
    """A model whose last step left work pending (the next projection / tile
    kernel, holding its target) releases it when the model is freed: the
    workspace forgets the pending entry and re-zeroes its counters for the next
    user, whose steps then match a fresh run."""
    import gc
    from gsvc_amd import train as Tr
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    gt = synthetic_gt(64, 64, 2, cuda)
    model = make_frame_model(64, 64, 200, cuda, seed=1)
    for it in range(1, 6):
        model.train_iter(gt, it)
    key = (cuda.index, torch._C._cuda_getCurrentRawStream(cuda.index))
    ws = Tr._workspaces[key]
    assert ws.pending is not None and ws.pending[5] is not None  # tiles ahead, target held
    del model
    gc.collect()
    assert ws.pending is None and ws.dirty
    # the next model on the same workspace trains as on a fresh one
    la = [float(make_frame_model(64, 64, 200, cuda, seed=1).train_iter(gt, 1)[0])]
    m2 = make_frame_model(64, 64, 200, cuda, seed=1)
    lb = [float(m2.train_iter(gt, it)[0]) for it in (1, 2, 3)]
    assert abs(la[0] - lb[0]) <= 1e-6 * abs(lb[0])
