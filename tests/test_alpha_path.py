"""Alpha compositing (gsplat.rasterize_gaussians, the secondary composite of
SURVEY §8 a12: forward.cu:252-374, backward.cu:138-315) past the 32x48
fixture of test_gpu_parity:

* dense 32x32 fixtures made by the reference's own glue and its
  _torch_impl.rasterize_forward (tests/golden/make_golden.py ``alpha``):
  ``alpha_32x32_stop`` (opaque splats, ~400 entries per tile: the T <= 1e-4
  early stop fires on most pixels) and ``alpha_32x32_deep`` (faint splats:
  the compositing runs past entry 256 into the tile's second batch);
* 1920x1080 against the C oracle (oracle/oracle.c raster_forward /
  raster_backward, the restatement of the same kernels).

Tolerances: image / alpha 1e-5 abs (float32, same op order); gradients
1e-4 (float atomics in the backward); final_idx exact.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def T(a, dev="cuda"):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def _tb(H, W):
    return ((W + 15) // 16, (H + 15) // 16, 1)


def _forward_backward(z):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize import rasterize_gaussians
    H, W = int(z["H"]), int(z["W"])
    m = T(z["means2d"]).requires_grad_(True)
    l = T(z["L"]).requires_grad_(True)
    c = T(z["colors"]).requires_grad_(True)
    o = T(z["opacity"]).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, _tb(H, W))
    out, alpha = rasterize_gaussians(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                     background=T(z["background"]), return_alpha=True)
    ((out * T(z["v_out"])).sum() + (alpha * T(z["v_alpha"])).sum()).backward()
    return out, alpha, m, l, c, o


@pytest.mark.parametrize("name", ["alpha_32x32_stop", "alpha_32x32_deep"])
def test_alpha_dense_golden(cuda, name):
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    assert int(z["tile_count"].min()) > 256  # every tile needs a second batch
    out, alpha, m, l, c, o = _forward_backward(z)
    np.testing.assert_allclose(N(out), z["out_img"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(N(out), z["torch_impl_out_img"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(N(alpha), z["out_alpha"], rtol=1e-5, atol=1e-5)
    scale = max(H, W) / 2
    np.testing.assert_allclose(N(m.grad), z["v_means2d"], rtol=1e-4, atol=1e-4 * scale)
    np.testing.assert_allclose(N(l.grad), z["v_L"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(N(c.grad), z["v_colors"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(N(o.grad), z["v_opacity"], rtol=1e-4, atol=1e-4)
    # the kernel's own stop position per pixel
    tb = _tb(H, W)
    _, Ts, idx = ops.rasterize_forward(tb, (16, 16, 1), (W, H, 1), T(z["gaussian_ids_sorted"]),
                                       T(z["tile_bins"]), T(z["xys"]), T(z["conics"]),
                                       T(z["colors"]), T(z["opacity"]), T(z["background"]))
    np.testing.assert_array_equal(N(idx), z["final_idx"])
    np.testing.assert_allclose(N(Ts), z["final_Ts"], rtol=1e-5, atol=1e-7)
    reach = N(idx) - (z["final_idx"] - z["reach"])  # entry position reached in the tile
    count = z["tile_count"]
    if name.endswith("stop"):
        stopped = (reach < count - 1) & (N(Ts) < 1e-3)
        assert stopped.sum() > 0.9 * reach.size  # the T <= 1e-4 stop fired
        assert N(Ts).min() > 1e-4  # the entry that would cross it is skipped
    else:
        assert (reach >= 256).sum() > 0.5 * reach.size  # second 256-entry batch
        assert N(Ts).min() > 0.4


@pytest.mark.parametrize("n,chol", [(10000, 1.0), (30000, 4.0)])
def test_alpha_1080p_oracle(cuda, oracle, n, chol):
    """Full 1080p frame against the C restatement, forward and backward; the
    dense case (~40-60 entries per tile) walks the forward's lane-group lists."""
    from gsvc_amd import ops
    H, W = 1080, 1920
    tb = _tb(H, W)
    means, L, colors, _ = oracle.synthetic_frame(n, seed=n + 17, chol_scale=chol)
    opac = np.random.default_rng(n).uniform(0.2, 1.0, (n, 1)).astype(np.float32)
    bg = np.array([0.1, 0.4, 0.7], np.float32)
    ref = oracle.render_sum(means, L, colors, opac, H, W)  # projection + sorted bins
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(L), H, W, tb,
                                                                      0.01)
    gids, bins, _ = ops.bin_and_sort_tiles(n, ref["m"], xys, depths, radii, T(ref["cum"]), tb)
    np.testing.assert_array_equal(N(gids), ref["gids_sorted"])
    counts = ref["bins"][: tb[0] * tb[1], 1] - ref["bins"][: tb[0] * tb[1], 0]
    if chol > 1.0:
        assert (counts > 24).mean() > 0.5  # most tiles take the grouped lists
    out, Ts, idx = ops.rasterize_forward(tb, (16, 16, 1), (W, H, 1), gids, bins, xys, conics,
                                         T(colors), T(opac), T(bg))
    r_out, r_Ts, r_idx = oracle.raster_forward(tb, H, W, ref["gids_sorted"], ref["bins"], ref["xys"],
                                               ref["conics"], colors, opac, bg)
    np.testing.assert_allclose(N(out), r_out, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(N(Ts), r_Ts, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(N(idx), r_idx)
    g = np.random.default_rng(n + 1)
    v_out = g.standard_normal((H, W, 3)).astype(np.float32)
    v_alpha = g.standard_normal((H, W)).astype(np.float32)
    v = ops.rasterize_backward(H, W, 16, 16, gids, bins, xys, conics, T(colors), T(opac), T(bg),
                               Ts, idx, T(v_out), T(v_alpha))
    rv = oracle.raster_backward(tb, H, W, ref["gids_sorted"], ref["bins"], ref["xys"], ref["conics"],
                                colors, opac, bg, r_Ts, r_idx, v_out, v_alpha)
    for a, b in zip(v, rv):
        b = np.asarray(b, np.float32).reshape(N(a).shape)
        np.testing.assert_allclose(N(a), b, rtol=1e-4, atol=1e-4 * max(1.0, float(np.abs(b).max())))
