"""The lane-group entry lists: each group of lanes walks
only the entries whose alpha >= 1/255 rectangle reaches its 4x4-pixel block.
Skipped pairs contribute nothing in the reference, so every variant must be
bit-identical: lists always on / the default threshold / never, the sparse
and banded composites, and the fused training step's forward with and
without its lists (A/B knobs 15 and 14), at random-init and trained-like
densities (3 to ~60 entries per tile)."""
import numpy as np
import pytest
import torch

from conftest import knobs

pytestmark = pytest.mark.gpu

H, W = 1080, 1920


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _tb(h, w):
    return ((w + 15) // 16, (h + 15) // 16, 1)


@pytest.mark.parametrize("n,chol", [(10000, 1.0), (50000, 1.0), (50000, 3.0), (20000, 8.0)])
def test_composite_lists_bit_identical(cuda, oracle, n, chol):
    from gsvc_amd.render import render_sum_frame
    means, L, colors, opac = oracle.synthetic_frame(n, seed=n + 17, rgb_w=2.0, chol_scale=chol)
    bg = torch.ones(3, device="cuda")
    outs = {}
    # mode 1 sparse / 2 banded; knob 15 = 1: lists on every chunk, 65: never
    for mode in (1, 2):
        for lists in (0, 1, 65):
            with knobs((0, mode), (15, lists)):
                outs[(mode, lists)] = render_sum_frame(T(means), T(L), T(colors), T(opac), H, W,
                                                       _tb(H, W), bg)
    ref = outs[(1, 65)]
    for key, out in outs.items():
        assert torch.equal(out, ref), key


def test_composite_lists_match_oracle_dense(cuda, oracle):
    """Trained-like density (~35 entries per tile, lists on by default) against
    the C oracle."""
    from gsvc_amd.render import render_sum_frame
    n = 30000
    means, L, colors, opac = oracle.synthetic_frame(n, seed=5, rgb_w=2.0, chol_scale=3.0)
    fast = render_sum_frame(T(means), T(L), T(colors), T(opac), H, W, _tb(H, W),
                            torch.ones(3, device="cuda"))
    ref = oracle.render_sum(means, L, colors, opac, H, W)["out"]
    ref = np.clip(ref, 0, 1).reshape(H, W, 3).transpose(2, 0, 1)[None]
    np.testing.assert_allclose(fast.cpu().numpy(), ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize("chol", [1.0, 4.0])
def test_train_forward_lists_bit_identical(cuda, chol):
    """The fused step's render with the band kernel's lists (default) and
    without (knob 14 = 1) is the same image; the gradients agree to the float
    atomics' summation order."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    gt = synthetic_gt(256, 384, 3, cuda)
    res = []
    for knob in (0, 1):
        model = make_frame_model(256, 384, 6000, cuda, seed=21)
        with torch.no_grad():
            model._cholesky.mul_(chol)
        with knobs((14, knob)):
            render = torch.empty(3, 256, 384, device=cuda)
            g = torch.empty(6000, 9, device=cuda)
            from gsvc_amd.train import train_step_sum
            losses = train_step_sum(model._xyz.data, model._cholesky.data, model._features_dc.data,
                                    model.rgb_W.data, False, model.cholesky_bound, model.background,
                                    gt.reshape(3, 256, 384).contiguous(), 256, 384, "L2", render_out=render, grads_out=g)
            torch.cuda.synchronize()
            res.append((render.clone(), g.clone(), losses.cpu().clone()))
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(res[0][2], res[1][2], rtol=0, atol=0)


def _bits(t):
    return t.contiguous().view(torch.int32)


@pytest.mark.parametrize("case", ["unit", "unit_dense", "mixed", "edge"])
def test_composite_sigma_cut_bit_identical(cuda, oracle, case):
    """The sparse render's sigma-threshold blend (chunks whose entries all have
    unit opacity, finite colour and bounded geometry; knob 19 = 1 turns it off)
    gives the same bits as the test as written -- including chunks that hold a
    NaN or infinite colour, an overflowing conic or a non-unit opacity, which
    must keep the written test (bitwise compare: NaN pixels included)."""
    from gsvc_amd.render import render_sum_frame
    n = 30000 if case == "unit_dense" else 8000
    means, L, colors, opac = oracle.synthetic_frame(
        n, seed=7, rgb_w=2.0, chol_scale=3.0 if case == "unit_dense" else 1.0)
    opac = np.ones_like(opac)
    if case == "mixed":
        opac[::7] = 0.5
    if case == "edge":
        colors = colors.copy()
        L = L.copy()
        colors[3] = np.nan
        colors[11, 1] = np.inf
        L[17] = [1e-19, 0.0, 1e-19]   # conic past the cut's bounds (or culled)
        L[23] = [40.0, 39.9, 1e-3]    # a needle: large, nearly singular conic
    bg = torch.ones(3, device="cuda")
    outs = []
    for knob in (0, 1):
        with knobs((0, 1), (19, knob)):
            outs.append(render_sum_frame(T(means), T(L), T(colors), T(opac), H, W, _tb(H, W), bg))
    assert torch.equal(_bits(outs[0]), _bits(outs[1])), case
    if case == "unit_dense":
        ref = oracle.render_sum(means, L, colors, opac, H, W)["out"]
        ref = np.clip(ref, 0, 1).reshape(H, W, 3).transpose(2, 0, 1)[None]
        np.testing.assert_allclose(outs[0].cpu().numpy(), ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize("want_idx", [False, True])
def test_sigma_cut_keeps_negative_zero_sigma(cuda, oracle, want_idx):
    """sigma = -0.0 passes the reference's test (!(sigma < 0), alpha = 1,
    forward.cu:598-606) while its bits fail the unsigned threshold compare of
    the sigma cut: an operator caller's conic with c = -0.0 and b < 0 gives it
    one pixel above the centre.  The cut must not take such an entry
    (cull.h geo_bounded: c/2 without sign bit), on the render instance
    (want_idx False, the cut) and the autograd one alike."""
    from gsvc_amd import ops
    H = W = 16
    xys = np.array([[8.0, 8.0], [3.0, 12.0]], np.float32)
    conics = np.array([[0.5, -1.0, -0.0], [0.3, 0.05, 0.4]], np.float32)
    colors = np.array([[0.25, 0.5, 0.75], [0.1, 0.2, 0.3]], np.float32)
    opac = np.ones((2, 1), np.float32)
    gids = np.array([0, 1], np.int32)
    bins = np.array([[0, 2]], np.int32)
    tb = (1, 1, 1)
    out, _ = ops.rasterize_sum_forward_ex(tb, (16, 16, 1), (W, H, 1), T(gids), T(bins), T(xys),
                                          T(conics), T(colors), T(opac),
                                          torch.ones(3, device=cuda), want_idx=want_idx)
    ref, _, _ = oracle.raster_sum_forward(tb, H, W, gids, bins, xys, conics, colors, opac)
    g = out.cpu().numpy()
    assert np.all(ref[7, 8] >= colors[0] - 1e-6)  # the sigma = -0 pixel (alpha 1) is in
    np.testing.assert_array_equal(np.isnan(g), np.isnan(ref))
    fin = np.isfinite(ref)
    np.testing.assert_allclose(g[fin], ref[fin], rtol=0, atol=1e-5)
