"""The deterministic backward (SURVEY §7 "a deterministic
backward option makes PSNR-vs-ref comparisons repeatable").

Under ``torch.use_deterministic_algorithms(True)`` the fused training step
(GSVC_TRAIN_DETERMINISTIC) and the op path's rasterize_sum_backward
(gsvc_rasterize_sum_backward_det) store every (splat, tile) gradient sum in
its own slot instead of adding it with float atomics, and each splat adds its
slots in tile-bbox order (csrc/det.h).  The reference's backward.cu:843-859
adds with atomics, so it is not reproducible run to run; this option is.

* the same step twice: bitwise-equal gradients (fused and op path) at the
  bench's trained 1080p / 50k state and on tiles past 256 entries;
* the same values as the atomic path within 1e-4 of the largest gradient
  (only the summation order differs);
* two 30-iteration fused trajectories from one init at 1080p / 50k: every
  parameter and the Adan state bitwise equal, no capacity fallback;
* a too-small slot capacity falls back to the atomics (still correct).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

H, W = 1080, 1920


@pytest.fixture
def deterministic():
    prev = torch.are_deterministic_algorithms_enabled()
    prev_warn = torch.is_deterministic_algorithms_warn_only_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    yield
    torch.use_deterministic_algorithms(prev, warn_only=prev_warn)


def _state_model(device, fused=True):
    from gsvc_amd.frame import make_frame_model
    z = load_golden("train_state_1080p_n50k")
    m = make_frame_model(H, W, int(z["n"]), device, seed=0, fused_train=fused)
    with torch.no_grad():
        for k in ("_xyz", "_cholesky", "_features_dc"):
            getattr(m, k).copy_(torch.from_numpy(z["state_" + k]))
    return m, z


def _fused_grads(m, gt):
    from gsvc_amd.train import train_step_sum
    n = m._xyz.shape[0]
    g = torch.empty((n, 9), device=gt.device)
    train_step_sum(m._xyz.data, m._cholesky.data, m._features_dc.data, m.rgb_W.data, False,
                   m.cholesky_bound, m.background, gt.contiguous(), m.H, m.W, "L2", grads_out=g)
    return g


def _close(a, b, tol=1e-4):
    a = a.double()
    b = b.double()
    sc = float(b.abs().max())
    assert float((a - b).abs().max()) <= tol * sc, float((a - b).abs().max()) / sc


def test_fused_step_gradients_reproducible(cuda, deterministic):
    from gsvc_amd.frame import synthetic_gt
    m, z = _state_model(cuda)
    gt = synthetic_gt(H, W, int(z["gt_seed"]), "cpu").to(cuda)
    g1 = _fused_grads(m, gt)
    g2 = _fused_grads(m, gt)
    assert torch.equal(g1, g2)
    torch.use_deterministic_algorithms(False)
    ga = _fused_grads(m, gt)
    _close(g1, ga)


def test_fused_step_overfull_tiles_reproducible(cuda, deterministic):
    """Tiles past 256 entries (the slab overflow rebuild): 1500 splats on one spot."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    Hs, Ws, n = 64, 64, 6000
    m = make_frame_model(Hs, Ws, n, cuda, seed=5)
    with torch.no_grad():
        sel = torch.arange(0, n, 4, device=cuda)
        m._xyz[sel] = torch.atanh(torch.full((len(sel), 2), -0.25, device=cuda)
                                  + 0.05 * torch.rand(len(sel), 2, device=cuda))
        m._cholesky[sel] = torch.tensor([2.5, 0.3, 1.5], device=cuda)
    gt = synthetic_gt(Hs, Ws, 2, cuda)
    g1 = _fused_grads(m, gt)
    g2 = _fused_grads(m, gt)
    assert torch.equal(g1, g2)
    torch.use_deterministic_algorithms(False)
    _close(g1, _fused_grads(m, gt))


def test_short_capacity_falls_back_to_atomics(cuda, deterministic, monkeypatch):
    from gsvc_amd import train as T
    from gsvc_amd.frame import synthetic_gt
    m, z = _state_model(cuda)
    gt = synthetic_gt(H, W, int(z["gt_seed"]), "cpu").to(cuda)
    ref = _fused_grads(m, gt)
    # a fresh workspace whose slot buffer holds a tenth of the pairs
    ws = T._workspace(cuda, m._xyz.shape[0], H, W)
    old = (ws.det_buf, ws.det_cap)
    ws.det_buf, ws.det_cap = None, 0
    monkeypatch.setattr(T, "DET_CAPACITY_PER_SPLAT", 0)
    buf, cap = ws.det_workspace(cuda, m._xyz.shape[0], 20000)
    assert cap < 200000
    g = _fused_grads_with(ws, m, gt, buf, cap)
    _close(g, ref)
    ws.det_buf, ws.det_cap = old


def _fused_grads_with(ws, m, gt, buf, cap):
    """train_step_sum with this slot buffer (capacity ``cap``)."""
    import ctypes
    from gsvc_amd import _lib as L
    from gsvc_amd import train as T
    n = m._xyz.shape[0]
    g = torch.empty((n, 9), device=gt.device)
    loss = torch.empty((2,), device=gt.device)
    a = T._StepArgs()
    a.num_points, a.xyz, a.cholesky = n, m._xyz.data_ptr(), m._cholesky.data_ptr()
    a.cholesky_bound, a.features = m.cholesky_bound.data_ptr(), m._features_dc.data_ptr()
    a.rgb_w, a.rgb_w_trainable = m.rgb_W.data_ptr(), 0
    a.background, a.gt, a.img_height, a.img_width = m.background.data_ptr(), gt.data_ptr(), H, W
    hp = (ctypes.c_double * 10)()
    state = (ctypes.c_void_p * 16)()
    a.loss_kind, a.frame_index = 0, ws.frame
    a.adan_state, a.adan_hparams = ctypes.addressof(state), ctypes.addressof(hp)
    a.adan_flags, a.loss, a.grads_out = T.TRAIN_DETERMINISTIC, loss.data_ptr(), g.data_ptr()
    a.workspace, a.workspace_bytes = ws.buf_ptr, ws.buf.numel()
    a.stream = T._raw_stream(gt.device.index)
    a.det_workspace, a.det_workspace_bytes, a.det_capacity = buf.data_ptr(), buf.numel(), cap
    assert L.load().gsvc_train_step_sum_args(ctypes.byref(a)) == 0
    ws.frame += 1
    return g


def test_fused_trajectory_bitwise_reproducible(cuda, deterministic):
    """Two 30-iteration GaussianVideoFrame.train_iter runs (bound fused steps,
    projection ahead, Adan) from one init at 1080p / 50k: identical bits."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    gt = synthetic_gt(H, W, 8, "cpu").to(cuda)
    runs = []
    for _ in range(2):
        m = make_frame_model(H, W, 50000, cuda, seed=1000)
        ps = [m.train_iter(gt, it)[1] for it in range(1, 31)]
        torch.cuda.synchronize()
        assert m.fused_steps == 30
        step = m._bound_step if hasattr(m, "_bound_step") else None
        if step is not None:
            assert step.det and step.det_overflows == 0
        runs.append((m, ps))
    (a, pa), (b, pb) = runs
    assert pa == pb
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k
    for p, q in zip(a.optimizer.param_groups[0]["params"], b.optimizer.param_groups[0]["params"]):
        for key in ("exp_avg", "exp_avg_sq", "exp_avg_diff", "neg_pre_grad"):
            assert torch.equal(a.optimizer.state[p][key], b.optimizer.state[q][key]), key


def test_op_path_backward_reproducible(cuda, deterministic):
    """GSVC's own route (autograd through gsplat.*) at the trained state: the
    deterministic rasterize_sum_backward twice gives the same bits, and the
    atomic one the same values within 1e-4."""
    from gsvc_amd.frame import loss_fn, synthetic_gt
    m, z = _state_model(cuda, fused=False)
    gt = synthetic_gt(H, W, int(z["gt_seed"]), "cpu").to(cuda)

    def grads():
        img = m()["render"]
        loss_fn(img.squeeze(0), gt.squeeze(0), "L2", lambda_value=0).backward()
        g = {k: getattr(m, k).grad.clone() for k in ("_xyz", "_cholesky", "_features_dc")}
        m.optimizer.zero_grad(set_to_none=True)
        return g

    g1, g2 = grads(), grads()
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
    torch.use_deterministic_algorithms(False)
    ga = grads()
    for k in g1:
        _close(g1[k], ga[k])


def _overflow_model(cuda, monkeypatch):
    """A fresh 256x256 / 2000-splat frame whose first fused step gets one slot
    per splat (about 2.5 pairs per splat at random init: the capacity is short)."""
    from gsvc_amd import train as T
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    m = make_frame_model(256, 256, 2000, cuda, seed=3)
    gt = synthetic_gt(256, 256, 4, cuda)
    ws = T._workspace(cuda, 2000, 256, 256)
    ws.det_buf, ws.det_cap = None, 0
    monkeypatch.setattr(T, "DET_CAPACITY_PER_SPLAT", 1)
    return m, gt


def test_short_capacity_warns_under_warn_only(cuda, deterministic, monkeypatch):
    """a fused step whose pairs outnumber the slots is not bitwise
    reproducible -- warn_only mode says so, and the next step has room."""
    m, gt = _overflow_model(cuda, monkeypatch)
    with pytest.warns(UserWarning, match="not bitwise reproducible"):
        m.train_iter(gt, 1)
    assert m._bound_step.det_overflows == 1
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        m.train_iter(gt, 2)
    assert m._bound_step.det_overflows == 1


def test_short_capacity_raises_in_strict_mode(cuda, monkeypatch):
    prev = torch.are_deterministic_algorithms_enabled()
    prev_warn = torch.is_deterministic_algorithms_warn_only_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        m, gt = _overflow_model(cuda, monkeypatch)
        with pytest.raises(RuntimeError, match="not bitwise reproducible"):
            m.train_iter(gt, 1)
    finally:
        torch.use_deterministic_algorithms(prev, warn_only=prev_warn)


def test_op_path_short_capacity_repeats(cuda, deterministic, monkeypatch):
    """The op path's deterministic backward repeats a call whose pairs outnumber
    the slots, so its gradients are always the reproducible ones: a one-slot-
    per-splat start gives the bits of an ample capacity."""
    from gsvc_amd import ops
    from gsvc_amd.frame import synthetic_gt
    m, z = _state_model(cuda, fused=False)
    gt = synthetic_gt(H, W, int(z["gt_seed"]), "cpu").to(cuda)

    def grads():
        for p in m.parameters():
            p.grad = None
        img = m.forward()["render"]
        torch.nn.functional.mse_loss(img, gt).backward()
        return torch.cat([m._xyz.grad.flatten(), m._cholesky.grad.flatten(),
                          m._features_dc.grad.flatten()])

    ops._det_ws.clear()
    ref = grads()
    ops._det_ws.clear()
    monkeypatch.setattr(ops, "DET_PAIRS_PER_SPLAT", 1)
    assert torch.equal(grads(), ref)
