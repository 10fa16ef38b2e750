"""GPU parity: the gfx950 ops (through the C ABI) against the oracle and the
golden fixtures.  Bars: indices, radii, tile counts, sort
order and bins bit-exact; projection floats bit-exact (same IEEE op
sequence); rasterized RGB within 1e-5 abs and gradients within 1e-4
(abs + rel), the only float difference in the forward being v_exp_f32 vs
libm exp2f (<= 1 ulp); final_idx exact except "borderline" pixels whose
candidate alpha lies within 1e-5 (relative) of 1/255.
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, knobs, load_golden

pytestmark = pytest.mark.gpu

SUM_CASES = golden_names("sum_")


def T(a, dev="cuda"):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def N(t):
    return t.detach().cpu().numpy()


def _tb(H, W):
    return ((W + 15) // 16, (H + 15) // 16, 1)


# --------------------------------------------------------------------------
# projection

@pytest.mark.parametrize("name", SUM_CASES)
def test_project_forward_bitexact(cuda, name):
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    n = z["means2d"].shape[0]
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(
        n, T(z["means2d"]), T(z["L"]), H, W, _tb(H, W), 0.01)
    np.testing.assert_array_equal(N(xys), z["xys"])
    np.testing.assert_array_equal(N(radii), z["radii"])
    np.testing.assert_array_equal(N(conics), z["conics"])
    np.testing.assert_array_equal(N(nth), z["num_tiles_hit"])
    assert (N(depths) == 0).all()


@pytest.mark.parametrize("name", ["sum_64x96_n300", "sum_trained_like_48x80_n200"])
def test_project_backward_bitexact(cuda, oracle, name):
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    n = z["means2d"].shape[0]
    rng = np.random.default_rng(3)
    v_xy = rng.standard_normal((n, 2)).astype(np.float32)
    v_conic = rng.standard_normal((n, 3)).astype(np.float32)
    g = ops.project_gaussians_2d_backward(n, T(z["means2d"]), T(z["L"]), H, W, T(z["radii"]),
                                          T(z["conics"]), T(v_xy), None, T(v_conic))
    ref = oracle.project_2d_backward(z["L"], H, W, z["radii"], z["conics"], v_xy, v_conic)
    for a, b in zip(g, ref):
        np.testing.assert_array_equal(N(a), b)


def test_cov2d_bounds_ref_tests(cuda, oracle):
    from gsvc_amd import utils
    z = load_golden("ref_tests_seed42")
    conics, radii = utils.compute_cov2d_bounds(T(z["covs2d"]))
    c_ref, r_ref = oracle.cov2d_bounds(z["covs2d"])
    np.testing.assert_array_equal(N(conics), c_ref)
    np.testing.assert_array_equal(N(radii), r_ref)
    m = z["cov2d_mask"]
    np.testing.assert_array_equal(N(radii)[m, 0], z["cov2d_radii"][m])


# --------------------------------------------------------------------------
# binning

@pytest.mark.parametrize("n", [1, 7, 2048, 2049, 5000, 70001])
def test_cumulative_intersects(cuda, n):
    from gsvc_amd import ops, utils
    rng = np.random.default_rng(n)
    nth = rng.integers(0, 9, n).astype(np.int32)
    nth[rng.random(n) < 0.3] = 0
    m, cum = utils.compute_cumulative_intersects(T(nth))
    np.testing.assert_array_equal(N(cum), np.cumsum(nth).astype(np.int32))
    assert m == int(nth.sum())
    depths = rng.random(n).astype(np.float32)
    _, meta = ops.cumulative_intersects(T(nth), T(depths))
    bits = depths.view(np.uint32)[nth > 0]
    meta = N(meta)
    assert meta[0] == int(nth.sum()) and meta[3] == int((nth > 0).sum())
    if bits.size:
        assert np.uint32(meta[1]) == np.bitwise_or.reduce(bits)
        assert np.uint32(meta[2]) == np.bitwise_and.reduce(bits)


@pytest.mark.parametrize("name", ["ref_tests_seed42"] + SUM_CASES)
def test_map_intersects_bitexact(cuda, oracle, name):
    from gsvc_amd import utils
    z = load_golden(name)
    if name.startswith("ref_tests"):
        tb = tuple(int(x) for x in z["tile_bounds"])
        xys, depths, radii, cum = z["xys"], z["depths"], z["radii"], z["cum_tiles_hit"]
    else:
        if int(z["num_intersects"]) < 1:
            pytest.skip("no intersections")
        tb = _tb(int(z["H"]), int(z["W"]))
        xys, radii, cum = z["xys"], z["radii"], z["cum_tiles_hit"]
        depths = np.zeros(len(xys), np.float32)
    m = int(cum[-1])
    isect, gids = utils.map_gaussian_to_intersects(len(xys), m, T(xys), T(depths), T(radii), T(cum), tb)
    ri, rg = oracle.map_intersects(xys, depths, radii, cum, tb, m)
    np.testing.assert_array_equal(N(isect), ri)
    np.testing.assert_array_equal(N(gids), rg)


def _sort_case(kind, n, rng):
    if kind == "ties":
        keys = (rng.integers(0, 37, n).astype(np.int64) << 32)
    elif kind == "signed":
        keys = rng.integers(-2**62, 2**62, n, dtype=np.int64)
        keys[rng.random(n) < 0.5] = 5
    else:  # tile | depth bits, like the reference 3D keys
        d = rng.standard_normal(n).astype(np.float32).view(np.int32).astype(np.int64)
        keys = (rng.integers(0, 8160, n).astype(np.int64) << 32) | d
    vals = np.arange(n, dtype=np.int32)
    return keys, vals


@pytest.mark.parametrize("kind", ["ties", "signed", "depth"])
@pytest.mark.parametrize("n", [1, 100, 2048, 5000, 124000])
def test_radix_sort_is_stable_torch_sort(cuda, oracle, kind, n):
    from gsvc_amd import ops
    keys, vals = _sort_case(kind, n, np.random.default_rng(n))
    ko, vo = ops.sort_isect_pairs(T(keys), T(vals))
    rk, rv = oracle.sort_pairs(keys, vals)
    np.testing.assert_array_equal(N(ko), rk)
    np.testing.assert_array_equal(N(vo), rv)


def test_sort_ref_tests_vector(cuda):
    from gsvc_amd import ops
    z = load_golden("ref_tests_seed42")
    ko, vo = ops.sort_isect_pairs(T(z["isect_ids"]), T(z["gaussian_ids"]))
    np.testing.assert_array_equal(N(ko), z["isect_ids_sorted"])
    np.testing.assert_array_equal(N(vo), z["gaussian_ids_sorted"])


def test_tile_bin_edges_ref_tests(cuda):
    from gsvc_amd import utils
    z = load_golden("ref_tests_seed42")
    bins = utils.get_tile_bin_edges(int(z["num_intersects"]), T(z["isect_ids_sorted"]))
    np.testing.assert_array_equal(N(bins), z["tile_bins"])


@pytest.mark.parametrize("name", SUM_CASES)
def test_bin_and_sort_matches_reference_glue(cuda, name):
    from gsvc_amd import ops, utils
    z = load_golden(name)
    m = int(z["num_intersects"])
    if m < 1:
        pytest.skip("no intersections")
    H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    n = len(z["xys"])
    depths = np.zeros(n, np.float32)
    # drop-in API (full int64 sort)
    isect, gids, isect_s, gids_s, bins = utils.bin_and_sort_gaussians(
        n, m, T(z["xys"]), T(depths), T(z["radii"]), T(z["cum_tiles_hit"]), tb)
    np.testing.assert_array_equal(N(isect), z["isect_ids"])
    np.testing.assert_array_equal(N(gids), z["gaussian_ids"])
    np.testing.assert_array_equal(N(isect_s), z["isect_ids_sorted"])
    np.testing.assert_array_equal(N(gids_s), z["gaussian_ids_sorted"])
    np.testing.assert_array_equal(N(bins)[: len(z["tile_bins"])], z["tile_bins"])
    # fused hot path (13-bit tile sort)
    g2, b2, i2 = ops.bin_and_sort_tiles(n, m, T(z["xys"]), T(depths), T(z["radii"]),
                                        T(z["cum_tiles_hit"]), tb, want_isect_ids=True)
    np.testing.assert_array_equal(N(g2), z["gaussian_ids_sorted"])
    np.testing.assert_array_equal(N(i2), z["isect_ids_sorted"])
    np.testing.assert_array_equal(N(b2), z["tile_bins"][: tb[0] * tb[1]])


# --------------------------------------------------------------------------
# sum rasterizer

def _check_final_idx(gpu_idx, ref_idx, margin):
    diff = gpu_idx != ref_idx
    borderline = margin < 1e-5
    assert not (diff & ~borderline).any(), int((diff & ~borderline).sum())
    return int(diff.sum())


@pytest.mark.parametrize("name", [c for c in SUM_CASES if "empty" not in c])
def test_raster_sum_forward_golden(cuda, name):
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    out, Ts, idx = ops.rasterize_sum_forward(
        _tb(H, W), (16, 16, 1), (W, H, 1), T(z["gaussian_ids_sorted"]), T(z["tile_bins"]),
        T(z["xys"]), T(z["conics"]), T(z["colors"]), T(z["opacity"]), T(np.ones(3, np.float32)))
    np.testing.assert_allclose(N(out), z["out_img"], rtol=1e-6, atol=1e-5)
    assert (N(Ts) == 1).all() and tuple(Ts.shape) == (H, W)
    _check_final_idx(N(idx), z["final_idx"], z["alpha_margin"])


@pytest.mark.parametrize("name", [c for c in SUM_CASES if "empty" not in c])
def test_raster_sum_forward_every_layout(cuda, name):
    """gsvc_rasterize_sum_forward_ex's three output layouts on every fixture:
    the [H, W, 3] image within 1e-5 of the golden output, the unclamped planes
    (2: the op path's GSVC_SLABS_PLANES image) its exact transpose, the
    clamped planes (1: the render's) exactly torch.clamp of it."""
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    args = (_tb(H, W), (16, 16, 1), (W, H, 1), T(z["gaussian_ids_sorted"]), T(z["tile_bins"]),
            T(z["xys"]), T(z["conics"]), T(z["colors"]), T(z["opacity"]), T(np.ones(3, np.float32)))
    hwc, _ = ops.rasterize_sum_forward_ex(*args, layout=ops.LAYOUT_HWC, want_idx=False)
    planes, _ = ops.rasterize_sum_forward_ex(*args, layout=ops.LAYOUT_CHW, want_idx=False)
    clamped, _ = ops.rasterize_sum_forward_ex(*args, layout=ops.LAYOUT_CHW_CLAMPED, want_idx=False)
    np.testing.assert_allclose(N(hwc), z["out_img"], rtol=1e-6, atol=1e-5)
    assert tuple(planes.shape) == (3, H, W)
    bits = lambda t: t.contiguous().view(torch.int32)  # noqa: E731 (NaN colours: bitwise)
    assert torch.equal(bits(planes), bits(hwc.permute(2, 0, 1)))
    ref = torch.clamp(hwc, 0, 1).permute(2, 0, 1)
    nan = torch.isnan(ref)
    assert torch.equal(torch.isnan(clamped), nan)
    assert torch.equal(clamped[~nan], ref[~nan])


@pytest.mark.parametrize("name", [c for c in SUM_CASES if "empty" not in c])
def test_raster_sum_backward_vs_oracle(cuda, oracle, name):
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    rng = np.random.default_rng(11)
    v_out = rng.standard_normal((H, W, 3)).astype(np.float32)
    g = ops.rasterize_sum_backward(H, W, 16, 16, T(z["gaussian_ids_sorted"]), T(z["tile_bins"]),
                                   T(z["xys"]), T(z["conics"]), T(z["colors"]), T(z["opacity"]),
                                   T(np.ones(3, np.float32)), None, T(z["final_idx"]), T(v_out),
                                   None)
    ref = oracle.raster_sum_backward(tb, H, W, z["gaussian_ids_sorted"], z["tile_bins"], z["xys"],
                                     z["conics"], z["colors"], z["opacity"], z["final_idx"], v_out)
    for a, b, nm in zip(g, ref, ("v_xy", "v_conic", "v_colors", "v_opacity")):
        np.testing.assert_allclose(N(a), b, rtol=1e-4, atol=1e-4, err_msg=nm)


def _lowered_final_idx(fi, bins, tbx, W, rng, share):
    """final_idx with a random ``share`` of the pixels lowered to a random
    index in [tile start - 1, final_idx] (share None: every pixel 0)."""
    fi = np.array(fi, np.int32)
    if share is None:
        return np.zeros_like(fi)
    H = fi.shape[0]
    ys, xs = np.nonzero(rng.random(fi.shape) < share)
    t = (ys // 16) * tbx + xs // 16
    lo = np.asarray(bins)[t, 0] - 1
    hi = fi[ys, xs]
    fi[ys, xs] = np.where(hi > lo, lo + (rng.random(ys.size) * (hi - lo + 1)).astype(np.int32), hi)
    return fi


@pytest.mark.parametrize("share", [0.1, None])
@pytest.mark.parametrize("name", [c for c in SUM_CASES if "empty" not in c] + ["1080p_n10000"])
def test_raster_sum_backward_honours_a_callers_final_idx(cuda, oracle, name, share):
    """the backward applies the reference's per-pixel skip of
    entries k > final_idx[p] (backward.cu:783-786) for a final_idx that is NOT
    the one this library's forward implies -- lowered on a random 10 % of the
    pixels, or 0 everywhere -- through the reference-named op and the zeroed
    C entry, each against oracle.raster_sum_backward on the same final_idx."""
    from gsvc_amd import _lib as L
    from gsvc_amd import ops
    if name.startswith("1080p"):
        H, W, n = 1080, 1920, 10000
        rng0 = np.random.default_rng(5)
        means = (2 * rng0.random((n, 2)) - 1).astype(np.float32)
        Lc = (rng0.random((n, 3)) + np.array([0.5, 0, 0.5])).astype(np.float32)
        cols = rng0.random((n, 3)).astype(np.float32)
        r = oracle.render_sum(means, Lc, cols, np.ones((n, 1), np.float32), H, W)
        z = dict(gaussian_ids_sorted=r["gids_sorted"], tile_bins=r["bins"], xys=r["xys"],
                 conics=r["conics"], colors=cols, opacity=np.ones((n, 1), np.float32),
                 final_idx=r["final_idx"])
    else:
        z = load_golden(name)
        H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    bins_t = ops._bins_for(T(np.asarray(z["tile_bins"], np.int32)), tb[0] * tb[1])[: tb[0] * tb[1]].contiguous()
    rng = np.random.default_rng(17)
    fi = _lowered_final_idx(z["final_idx"], N(bins_t), tb[0], W, rng, share)
    assert share is None or (fi != np.asarray(z["final_idx"])).mean() > 0.01
    v_out = rng.standard_normal((H, W, 3)).astype(np.float32)
    ref = oracle.raster_sum_backward(tb, H, W, z["gaussian_ids_sorted"], z["tile_bins"], z["xys"],
                                     z["conics"], z["colors"], z["opacity"], fi, v_out)
    g = ops.rasterize_sum_backward(H, W, 16, 16, T(z["gaussian_ids_sorted"]), T(z["tile_bins"]),
                                   T(z["xys"]), T(z["conics"]), T(z["colors"]), T(z["opacity"]),
                                   T(np.ones(3, np.float32)), None, T(fi), T(v_out), None)
    # the zeroed entry (the op path's), into a zeroed record
    nn = np.asarray(z["xys"]).shape[0]
    rec = torch.zeros((nn, 16), dtype=torch.float32, device=cuda)
    args = [T(z["gaussian_ids_sorted"]), bins_t, T(z["xys"]), T(z["conics"]), T(z["colors"]),
            T(z["opacity"]), T(fi), T(v_out)]
    L.call("gsvc_rasterize_sum_backward_zeroed", H, W, nn, *[L.ptr(a) for a in args],
           L.ptr(rec), L.stream(cuda))
    g2 = ops.split_grad_records(rec)
    for got in (g, g2):
        for a, b, nm in zip(got, ref, ("v_xy", "v_conic", "v_colors", "v_opacity")):
            scale = max(1.0, float(np.abs(b).max()))
            np.testing.assert_allclose(N(a), b, rtol=1e-4, atol=1e-4 * scale, err_msg=nm)
    if share is None:  # every entry skipped except sorted index 0
        others = np.ones(nn, bool)
        others[np.asarray(z["gaussian_ids_sorted"]).reshape(-1)[:1]] = False
        assert np.abs(N(g[2])[others]).max() == 0


@pytest.mark.parametrize("name", [c for c in SUM_CASES if "empty" not in c])
def test_raster_sum_backward_no_opacity_flag(cuda, oracle, name):
    """GSVC_BWD_NO_OPACITY (the C++ Function's backward when opacity takes no
    gradient, as GSVC's constant ones): v_xy, v_conic and v_colors as the oracle
    (1e-4), record word 8 untouched (still the zero the caller wrote)."""
    from gsvc_amd import _lib as L
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    rng = np.random.default_rng(23)
    v_out = rng.standard_normal((H, W, 3)).astype(np.float32)
    ref = oracle.raster_sum_backward(tb, H, W, z["gaussian_ids_sorted"], z["tile_bins"], z["xys"],
                                     z["conics"], z["colors"], z["opacity"], z["final_idx"], v_out)
    nn = np.asarray(z["xys"]).shape[0]
    bins_t = ops._bins_for(T(np.asarray(z["tile_bins"], np.int32)), tb[0] * tb[1])[: tb[0] * tb[1]].contiguous()
    vo = T(v_out)
    for flags in (1, 0):
        rec = torch.zeros((nn, 16), dtype=torch.float32, device=cuda)
        args = [T(z["gaussian_ids_sorted"]), bins_t, T(z["xys"]), T(z["conics"]), T(z["colors"]),
                T(z["opacity"]), T(np.asarray(z["final_idx"], np.int32)), vo]
        L.call("gsvc_rasterize_sum_backward_zeroed_strided_ex", H, W, nn, *[L.ptr(a) for a in args],
               3 * W, 3, 1, L.ptr(rec), L.stream(cuda), flags)
        got = ops.split_grad_records(rec)
        for a, b, nm in list(zip(got, ref, ("v_xy", "v_conic", "v_colors", "v_opacity")))[: 4 - flags]:
            scale = max(1.0, float(np.abs(b).max()))
            np.testing.assert_allclose(N(a), b, rtol=1e-4, atol=1e-4 * scale, err_msg=f"{nm} flags={flags}")
        if flags:
            assert float(rec[:, 8:].abs().max()) == 0.0


@pytest.mark.parametrize("name", SUM_CASES)
def test_autograd_end_to_end_matches_reference_glue(cuda, name):
    """gsplat.project_gaussians_2d -> rasterize_gaussians_sum -> backward, as
    GaussianSplats_Represent.forward calls them, vs the reference glue fixture."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    m = T(z["means2d"]).requires_grad_(True)
    l = T(z["L"]).requires_grad_(True)
    c = T(z["colors"]).requires_grad_(True)
    o = T(z["opacity"]).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, _tb(H, W))
    out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                  background=torch.ones(3, device="cuda"), return_alpha=False)
    np.testing.assert_allclose(N(out), z["out_img"], rtol=1e-6, atol=1e-5)
    (out * T(z["v_out"])).sum().backward()
    scale = max(H, W) / 2
    np.testing.assert_allclose(N(m.grad), z["v_means2d"], rtol=1e-4, atol=1e-4 * scale)
    np.testing.assert_allclose(N(l.grad), z["v_L"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(N(c.grad), z["v_colors"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(N(o.grad), z["v_opacity"], rtol=1e-4, atol=1e-4)


def test_return_alpha_and_empty_background(cuda):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    z = load_golden("sum_empty_32x32_n10")
    H, W = 32, 32
    m = T(z["means2d"]).requires_grad_(True)
    l = T(z["L"]).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, _tb(H, W))
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    out, alpha = rasterize_gaussians_sum(xys, depths, radii, conics, nth, T(z["colors"]),
                                         T(z["opacity"]), H, W, background=bg, return_alpha=True)
    np.testing.assert_array_equal(N(out), np.broadcast_to(N(bg), (H, W, 3)))
    assert (N(alpha) == 1).all()
    out.sum().backward()
    assert (N(m.grad) == 0).all() and (N(l.grad) == 0).all()


# --------------------------------------------------------------------------
# alpha compositing

def test_alpha_forward_backward_golden(cuda, oracle):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize import rasterize_gaussians
    z = load_golden("alpha_32x48_n40")
    H, W = int(z["H"]), int(z["W"])
    m = T(z["means2d"]).requires_grad_(True)
    l = T(z["L"]).requires_grad_(True)
    c = T(z["colors"]).requires_grad_(True)
    o = T(z["opacity"]).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, _tb(H, W))
    out, alpha = rasterize_gaussians(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                     background=T(z["background"]), return_alpha=True)
    np.testing.assert_allclose(N(out), z["out_img"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(N(out), z["torch_impl_out_img"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(N(alpha), z["out_alpha"], rtol=1e-5, atol=1e-5)
    ((out * T(z["v_out"])).sum() + (alpha * T(z["v_alpha"])).sum()).backward()
    scale = max(H, W) / 2
    np.testing.assert_allclose(N(m.grad), z["v_means2d"], rtol=1e-4, atol=1e-4 * scale)
    np.testing.assert_allclose(N(l.grad), z["v_L"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(N(c.grad), z["v_colors"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(N(o.grad), z["v_opacity"], rtol=1e-4, atol=1e-4)


# --------------------------------------------------------------------------
# full-size (BASELINE configs 2 and 3: 1920x1080, 10k / 50k splats)

@pytest.mark.parametrize("n", [10000, 50000])
def test_full_frame_1080p_parity(cuda, oracle, n):
    from gsvc_amd import ops
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    H, W = 1080, 1920
    means, L, colors, opac = oracle.synthetic_frame(n, seed=n)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    tb = _tb(H, W)
    xys, depths, radii, conics, nth = project_gaussians_2d(T(means), T(L), H, W, tb)
    np.testing.assert_array_equal(N(nth), ref["nth"])
    gids, bins, _ = ops.bin_and_sort_tiles(n, ref["m"], xys, depths, radii,
                                           T(ref["cum"]), tb)
    np.testing.assert_array_equal(N(gids), ref["gids_sorted"])
    np.testing.assert_array_equal(N(bins), ref["bins"][: tb[0] * tb[1]])
    out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, T(colors), T(opac), H, W)
    np.testing.assert_allclose(N(out), ref["out"], rtol=1e-6, atol=1e-5)
    _, _, idx = ops.rasterize_sum_forward(tb, (16, 16, 1), (W, H, 1), gids, bins, xys, conics,
                                          T(colors), T(opac), T(np.ones(3, np.float32)))
    margin = oracle.sum_min_margin(tb, H, W, ref["gids_sorted"], ref["bins"], ref["xys"],
                                   ref["conics"], opac)
    _check_final_idx(N(idx), ref["final_idx"], margin)
    # size-independent properties: linearity in colour, determinism
    out2 = rasterize_gaussians_sum(xys, depths, radii, conics, nth, 2 * T(colors), T(opac), H, W)
    assert torch.equal(out2, 2 * out)
    out3 = rasterize_gaussians_sum(xys, depths, radii, conics, nth, T(colors), T(opac), H, W)
    assert torch.equal(out3, out)


def test_full_frame_backward_properties(cuda):
    """At 1080p/50k the backward is checked by linearity in v_out and by the
    exact identity v_colors[g] = sum over its contributing pixels of alpha * v_out,
    which equals the forward rendered with v_out as colours (one channel)."""
    from gsvc_amd import ops
    import oracle as O
    H, W, n = 1080, 1920, 50000
    means, L, colors, opac = O.synthetic_frame(n, seed=7)
    from gsplat.project_gaussians_2d import project_gaussians_2d
    tb = _tb(H, W)
    xys, depths, radii, conics, nth = project_gaussians_2d(T(means), T(L), H, W, tb)
    from gsvc_amd.utils import bin_and_sort_for_raster
    m, gids, bins = bin_and_sort_for_raster(n, xys, depths, radii, nth, tb)
    bg = torch.ones(3, device="cuda")
    out, _, idx = ops.rasterize_sum_forward(tb, (16, 16, 1), (W, H, 1), gids, bins, xys, conics,
                                            T(colors), T(opac), bg)
    v = torch.randn((H, W, 3), device="cuda")
    g1 = ops.rasterize_sum_backward(H, W, 16, 16, gids, bins, xys, conics, T(colors), T(opac), bg,
                                    None, idx, v, None)
    g2 = ops.rasterize_sum_backward(H, W, 16, 16, gids, bins, xys, conics, T(colors), T(opac), bg,
                                    None, idx, 3 * v, None)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(b, 3 * a, rtol=1e-5, atol=1e-4)
    # <out, v> = sum_g <colors_g, v_colors_g>  (out is linear in colours)
    lhs = float((out.double() * v.double()).sum())
    rhs = float((T(colors).double() * g1[2].double()).sum())
    assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs))


def _nonfinite_colours(colors, rng):
    """inf, -inf and NaN in one channel of a few splats each."""
    c = colors.copy()
    n = len(c)
    pick = rng.choice(n, 12, replace=False)
    for j, s in enumerate(pick):
        c[s, j % 3] = (np.inf, -np.inf, np.nan)[j % 3]
    return c


@pytest.mark.parametrize("name", ["sum_64x96_n300", "sum_trained_like_48x80_n200"])
def test_raster_sum_forward_nonfinite_colours(cuda, oracle, name):
    """The reference skips a pair whose sigma < 0 or alpha < 1/255 before it
    touches the colour (forward.cu:600-609): an inf / NaN colour reaches only
    the pixels where its splat is valid.  The kernel selects the updates, so
    the non-finite footprint is the oracle's exactly (no c * 0 = NaN leaks)."""
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    colors = _nonfinite_colours(z["colors"], np.random.default_rng(5))
    out, _, idx = ops.rasterize_sum_forward(
        tb, (16, 16, 1), (W, H, 1), T(z["gaussian_ids_sorted"]), T(z["tile_bins"]),
        T(z["xys"]), T(z["conics"]), T(colors), T(z["opacity"]), T(np.ones(3, np.float32)))
    ref, _, ref_idx = oracle.raster_sum_forward(tb, H, W, z["gaussian_ids_sorted"], z["tile_bins"],
                                                z["xys"], z["conics"], colors, z["opacity"])
    g = N(out)
    assert (~np.isfinite(ref)).any()  # the case is not vacuous
    np.testing.assert_array_equal(np.isnan(g), np.isnan(ref))
    np.testing.assert_array_equal(np.isposinf(g), np.isposinf(ref))
    np.testing.assert_array_equal(np.isneginf(g), np.isneginf(ref))
    fin = np.isfinite(ref)
    np.testing.assert_allclose(g[fin], ref[fin], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("mode", [1, 2])
def test_render_frame_nonfinite_colours(cuda, oracle, mode):
    """The same through the frame path (both composite variants: 1 sparse,
    2 banded) with its fused clamp: torch.clamp keeps NaN, clamps +-inf."""
    from gsvc_amd.render import render_frame_sum
    z = load_golden("sum_64x96_n300")
    H, W = int(z["H"]), int(z["W"])
    colors = _nonfinite_colours(z["colors"], np.random.default_rng(6))
    # the fixture's means2d / L / colours as the frame inputs (no tanh, zero bound)
    bound = torch.zeros(3, device="cuda")
    with knobs((0, mode)):
        out = render_frame_sum(T(z["means2d"]), T(z["L"]), T(colors), H, W,
                               torch.ones(3, device="cuda"), xyz_tanh=False, cholesky_bound=bound)
    r = oracle.render_sum(z["means2d"], z["L"], colors, np.ones((len(colors), 1), np.float32), H, W)
    ref = np.clip(r["out"], 0, 1).transpose(2, 0, 1)[None]
    g = N(out)
    assert np.isnan(ref).any()
    np.testing.assert_array_equal(np.isnan(g), np.isnan(ref))
    fin = ~np.isnan(ref)
    np.testing.assert_allclose(g[fin], ref[fin], rtol=1e-6, atol=1e-5)


def test_raster_sum_backward_nonfinite_colours(cuda, oracle):
    """Backward with inf / NaN colours: a splat's gradients turn non-finite
    exactly where the oracle's do (valid pairs only, backward.cu:803-815);
    the finite ones stay within the usual tolerance."""
    from gsvc_amd import ops
    z = load_golden("sum_64x96_n300")
    H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    colors = _nonfinite_colours(z["colors"], np.random.default_rng(7))
    _, _, fidx = oracle.raster_sum_forward(tb, H, W, z["gaussian_ids_sorted"], z["tile_bins"],
                                           z["xys"], z["conics"], colors, z["opacity"])
    v_out = np.random.default_rng(12).standard_normal((H, W, 3)).astype(np.float32)
    g = ops.rasterize_sum_backward(H, W, 16, 16, T(z["gaussian_ids_sorted"]), T(z["tile_bins"]),
                                   T(z["xys"]), T(z["conics"]), T(colors), T(z["opacity"]),
                                   T(np.ones(3, np.float32)), None, T(fidx), T(v_out), None)
    ref = oracle.raster_sum_backward(tb, H, W, z["gaussian_ids_sorted"], z["tile_bins"], z["xys"],
                                     z["conics"], colors, z["opacity"], fidx, v_out)
    assert any((~np.isfinite(b)).any() for b in ref)
    for a, b, nm in zip(g, ref, ("v_xy", "v_conic", "v_colors", "v_opacity")):
        a = N(a)
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b), err_msg=nm)
        np.testing.assert_array_equal(np.isinf(a), np.isinf(b), err_msg=nm)
        fin = np.isfinite(b)
        np.testing.assert_allclose(a[fin], b[fin], rtol=1e-4, atol=1e-4, err_msg=nm)
