"""Device-side pruning (gsvc_prune_lowest, csrc/prune.hip) against the oracle
(oracle.prune_keep, pinned by the reference's removal_control /
adaptive_control in tests/golden/prune_controls.npz): bit-exact kept rows, in
order.  GaussianSplats_Represent.py:98-172."""
import numpy as np
import pytest
import torch

from conftest import load_golden

PARAMS = ("_xyz", "_cholesky", "_features_dc", "rgb_W")


def _prune(cuda, arrays, w, k):
    from gsvc_amd.prune import prune_lowest
    ts = [torch.from_numpy(np.ascontiguousarray(a)).to(cuda) for a in arrays]
    wt = torch.from_numpy(np.ascontiguousarray(w)).to(cuda)
    out = prune_lowest(wt, ts, k)
    torch.cuda.synchronize()
    return [o.cpu().numpy() for o in out]


@pytest.mark.gpu
def test_prune_kernel_matches_reference_fixture(cuda, oracle):
    d = load_golden("prune_controls")
    for ci in range(4):
        w = d[f"c{ci}_in_rgb_W"]
        k = w.shape[0] - d[f"c{ci}_out_rgb_W"].shape[0]
        got = _prune(cuda, [d[f"c{ci}_in_{p}"] for p in PARAMS], w, k)
        for p, g in zip(PARAMS, got):
            np.testing.assert_array_equal(g, d[f"c{ci}_out_{p}"], err_msg=f"case {ci} {p}")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["removal", "adaptive"])
def test_model_controls_match_reference_fixture(cuda, kind):
    """The frame model's removal_control / adaptive_control (host logic +
    kernel) on the fixture's parameters leave the reference's parameters."""
    from gsvc_amd.frame import GaussianVideoFrame
    d = load_golden("prune_controls")
    for ci in range(4):
        is_rm, it, n, mx = (int(x) for x in d[f"c{ci}_meta"])
        if (kind == "removal") != (is_rm == 0):
            continue
        m = GaussianVideoFrame(loss_type="L2", opt_type="adan", num_points=n, max_num_points=mx,
                               densification_interval=100, iterations=10, H=32, W=32, BLOCK_H=16,
                               BLOCK_W=16, device=cuda, lr=1e-3, quantize=False, removal_rate=0.1,
                               isdensity=kind == "adaptive", isremoval=kind == "removal").to(cuda)
        with torch.no_grad():
            for p in PARAMS:
                getattr(m, p).data = torch.from_numpy(d[f"c{ci}_in_{p}"]).to(cuda)
        (m.removal_control if kind == "removal" else m.adaptive_control)(it)
        for p in PARAMS:
            got = getattr(m, p)
            assert isinstance(got, torch.nn.Parameter)
            np.testing.assert_array_equal(got.detach().cpu().numpy(), d[f"c{ci}_out_{p}"],
                                          err_msg=f"case {ci} {p}")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 37, 1024, 1025, 5000, 110_000])
def test_prune_kernel_vs_oracle_ties_and_counts(cuda, oracle, n):
    """Heavy ties (8 distinct magnitudes, both signs), NaN, +-0, underflowing
    squares; counts 0, 1, inside a tie group, n-1, n, > n."""
    rng = np.random.default_rng(n)
    w = rng.choice(np.array([0.01, -0.01, 0.02, 0.005, -0.3, 0.7, 1e-25, 0.0], np.float32), n)
    if n > 10:
        w[rng.choice(n, 3, replace=False)] = np.array([np.nan, -0.0, 2e-20], np.float32)
    w = w.reshape(n, 1).astype(np.float32)
    xyz = rng.normal(size=(n, 2)).astype(np.float32)
    chol = rng.random((n, 3), dtype=np.float32)
    ks = sorted({0, 1, n // 3, n // 2, max(n - 1, 0), n, n + 5})
    for k in ks:
        keep = oracle.prune_keep(w, k)
        got = _prune(cuda, [xyz, chol, w], w, k)
        np.testing.assert_array_equal(got[0], xyz[keep], err_msg=f"k={k}")
        np.testing.assert_array_equal(got[1], chol[keep], err_msg=f"k={k}")
        np.testing.assert_array_equal(got[2], w[keep], err_msg=f"k={k}")


@pytest.mark.gpu
def test_prune_argument_errors(cuda):
    from gsvc_amd.prune import prune_lowest
    w = torch.ones(8, 1, device=cuda)
    with pytest.raises(RuntimeError, match="CUDA"):
        prune_lowest(w.cpu(), [w.cpu()], 1)
    with pytest.raises(ValueError):
        prune_lowest(w.view(8), [w], 1)
    with pytest.raises(ValueError):
        prune_lowest(w, [torch.ones(7, 2, device=cuda)], 1)
    with pytest.raises(RuntimeError, match="float32"):
        prune_lowest(w, [torch.ones(8, 2, device=cuda, dtype=torch.float64)], 1)
