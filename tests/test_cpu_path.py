"""CPU suite: the CPU dispatch of the two drop-in operators (gsvc_amd/cpu.py,
csrc/cpu_ops.cpp; BASELINE configs[0]) -- project_gaussians_2d and
rasterize_gaussians_sum on CPU tensors, forward and backward -- against the
oracle and the reference-glue fixtures.  The product code is not the oracle:
the oracle only checks it.  HIP tensors never take this path (the operators
dispatch on the inputs' device) and the op table stays GPU-only."""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

SUM_CASES = golden_names("sum_")


def _tb(H, W):
    return ((W + 15) // 16, (H + 15) // 16, 1)


def _run(means, L, colors, opac, H, W, v_out=None, bg=None, return_alpha=False):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    m = torch.from_numpy(np.ascontiguousarray(means)).requires_grad_(True)
    l = torch.from_numpy(np.ascontiguousarray(L)).requires_grad_(True)
    c = torch.from_numpy(np.ascontiguousarray(colors)).requires_grad_(True)
    o = torch.from_numpy(np.ascontiguousarray(opac)).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, _tb(H, W))
    res = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                  background=torch.ones(3) if bg is None else bg,
                                  return_alpha=return_alpha)
    out = res[0] if return_alpha else res
    if v_out is not None:
        (out * torch.from_numpy(v_out)).sum().backward()
    return res, (xys, depths, radii, conics, nth), (m, l, c, o)


def test_config1_matches_oracle_bit_for_bit(oracle):
    """BASELINE configs[0]: 256x256, 1k splats.  Projection outputs, tile
    counts and the image are the oracle's bits (same op sequence and exp2f);
    gradients within 1e-5 of the largest (summation order)."""
    H = W = 256
    means, L, colors, opac = oracle.synthetic_frame(1000, seed=0)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    v_out = np.random.default_rng(1).standard_normal((H, W, 3)).astype(np.float32)
    out, (xys, _, radii, conics, nth), (m, l, c, o) = _run(means, L, colors, opac, H, W, v_out)
    np.testing.assert_array_equal(nth.numpy(), ref["nth"])
    np.testing.assert_array_equal(radii.numpy(), ref["radii"])
    np.testing.assert_array_equal(xys.detach().numpy(), ref["xys"])
    np.testing.assert_array_equal(conics.detach().numpy(), ref["conics"])
    np.testing.assert_array_equal(out.detach().numpy(), ref["out"])
    v_xy, v_conic, v_rgb, v_op = oracle.raster_sum_backward(
        ref["tb"], H, W, ref["gids_sorted"], ref["bins"], ref["xys"], ref["conics"], colors, opac,
        ref["final_idx"], v_out)
    _, v_mean, v_L = oracle.project_2d_backward(L, H, W, ref["radii"], ref["conics"],
                                                v_xy.astype(np.float32), v_conic.astype(np.float32))
    for g, r in ((c.grad, v_rgb), (m.grad, v_mean), (l.grad, v_L), (o.grad, v_op)):
        g = g.double().numpy()
        assert np.abs(g - r).max() <= 1e-5 * np.abs(r).max()


def test_binning_is_the_sorted_order(oracle):
    """Each tile's ids: the first 256 of the reference's stable sort of
    (tile << 32 | depth 0) keys, i.e. ascending ids (the oracle's glue)."""
    from gsvc_amd import cpu
    z = load_golden("sum_stress_48x48_n700")
    H, W = int(z["H"]), int(z["W"])
    tbx, tby = (W + 15) // 16, (H + 15) // 16
    xys = np.ascontiguousarray(z["xys"], np.float32)
    radii = np.ascontiguousarray(z["radii"], np.int32)
    ids = np.zeros(tbx * tby * 256, np.int32)
    bins = np.zeros((tbx * tby, 2), np.int32)
    m = cpu.lib().gsvc_cpu_bin_tiles(len(radii), xys.ctypes.data, radii.ctypes.data, tbx, tby,
                                     ids.ctypes.data, bins.ctypes.data)
    assert m == int(z["num_intersects"])
    gs, tb = z["gaussian_ids_sorted"], z["tile_bins"]
    overfull = 0
    for t in range(tbx * tby):
        want = gs[tb[t, 0]:tb[t, 1]][:256] if t < len(tb) else gs[:0]
        got = ids[bins[t, 0]:bins[t, 1]]
        np.testing.assert_array_equal(got, want)
        overfull += int(tb[t, 1] - tb[t, 0] > 256) if t < len(tb) else 0
    assert overfull > 0  # the stress case has tiles past 256 entries


@pytest.mark.parametrize("name", SUM_CASES)
def test_autograd_matches_reference_glue(name):
    """The reference's own autograd Functions run on the fixture (make_golden.py):
    the CPU dispatch's image and every gradient."""
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    out, _, (m, l, c, o) = _run(z["means2d"], z["L"], z["colors"], z["opacity"], H, W, z["v_out"])
    np.testing.assert_allclose(out.detach().numpy(), z["out_img"], rtol=1e-6, atol=1e-5)
    scale = max(H, W) / 2
    np.testing.assert_allclose(m.grad.numpy(), z["v_means2d"], rtol=1e-4, atol=1e-4 * scale)
    np.testing.assert_allclose(l.grad.numpy(), z["v_L"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(c.grad.numpy(), z["v_colors"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(o.grad.numpy(), z["v_opacity"], rtol=1e-4, atol=1e-4)


def test_background_branch_and_alpha(oracle):
    """rasterize_sum.py:121-127: no intersection -> the background, alpha 1,
    zero gradients; with intersections alpha = 1 - final_Ts = 0."""
    H, W = 32, 48
    means, L, colors, opac = oracle.synthetic_frame(50, seed=3)
    bg = torch.tensor([0.2, 0.4, 0.6])
    (out, alpha), _, (m, l, c, o) = _run(means + 40.0, L, colors, opac, H, W,
                                         bg=bg, return_alpha=True)
    assert torch.equal(out, bg.expand(H, W, 3)) and torch.all(alpha == 1.0)
    out.sum().backward()
    assert float(c.grad.abs().sum()) == 0.0 and float(m.grad.abs().sum()) == 0.0
    (out, alpha), _, _ = _run(means, L, colors, opac, H, W, bg=bg, return_alpha=True)
    assert torch.all(alpha == 0.0)


def test_mixed_devices_and_op_table_stay_gpu_only():
    """A CPU call takes CPU tensors only, and the `_C` op table (the reference's
    extension ops) has no CPU path: no GPU call can reach the CPU code."""
    from gsvc_amd import cpu, ops
    x = torch.zeros(4, 2)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        ops.project_gaussians_2d_forward(4, x, torch.ones(4, 3), 32, 32, (2, 2, 1), 0.01)
    with pytest.raises(RuntimeError, match="scalar type"):
        cpu.ProjectGaussians2dCPU.apply(x.double(), torch.ones(4, 3), 32, 32, (2, 2, 1), 0.01)
