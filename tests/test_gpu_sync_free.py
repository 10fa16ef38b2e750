"""GPU parity of the sync-free hot path:

* gsvc_bin_tiles_counted (count -> scan -> fill -> per-tile segment sort) must
  give exactly the reference's sorted order -- gaussian_ids_sorted and
  tile_bins bit-exact against the oracle's stable sort and the golden
  fixtures -- including long segments (LDS-bitmap path), the 64/65 boundary
  between the two segment sorts, and an id span wider than one bitmap window;
* the rasterizer ops on that path (device-side M, background when M = 0,
  return_alpha) match the sized path and the fixtures;
* the render path (fused clamp + NCHW store, no final_idx) is bit-identical to
  GSVC's forward composed from the ops, in both kernel modes.
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


def _counted(n, xys, radii, tb):
    from gsvc_amd import ops
    cap = n * tb[0] * tb[1]
    gids, bins, meta = ops.bin_tiles_counted(n, xys, radii, tb, cap)
    m, ovf = (int(x) for x in meta.tolist())
    assert ovf == 0
    return m, gids[:m], bins


@pytest.mark.parametrize("name", SUM_CASES)
def test_counted_binning_golden(cuda, name):
    from gsvc_amd import ops
    z = load_golden(name)
    H, W = int(z["H"]), int(z["W"])
    tb = _tb(H, W)
    n = len(z["xys"])
    m, gids, bins = _counted(n, T(z["xys"]), T(z["radii"]), tb)
    assert m == int(z["num_intersects"])
    ref_bins = np.zeros((tb[0] * tb[1], 2), np.int32)
    if m > 0:
        np.testing.assert_array_equal(N(gids), z["gaussian_ids_sorted"])
        ref_bins = z["tile_bins"][: tb[0] * tb[1]]
    np.testing.assert_array_equal(N(bins), ref_bins)
    # deterministic despite the atomic fill
    m2, gids2, bins2 = _counted(n, T(z["xys"]), T(z["radii"]), tb)
    assert torch.equal(gids, gids2) and torch.equal(bins, bins2)
    del ops


@pytest.mark.parametrize("n,chol", [(10000, 1.0), (50000, 1.0), (20000, 8.0)])
def test_counted_binning_1080p(cuda, oracle, n, chol):
    """Full size, and large splats (chol x8: hundreds of entries per tile,
    LDS-bitmap segment sort)."""
    from gsvc_amd import ops
    H, W = 1080, 1920
    tb = _tb(H, W)
    means, L, colors, opac = oracle.synthetic_frame(n, seed=n + 3, chol_scale=chol)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(L), H, W, tb,
                                                                      0.01)
    m, gids, bins = _counted(n, xys, radii, tb)
    assert m == ref["m"]
    np.testing.assert_array_equal(N(gids), ref["gids_sorted"])
    np.testing.assert_array_equal(N(bins), ref["bins"][: tb[0] * tb[1]])
    counts = ref["bins"][:, 1] - ref["bins"][:, 0]
    if chol > 1:
        assert counts.max() > 64  # the bitmap path ran


def _clustered_frame(n, ids_on_tile, H=64, W=64):
    """Every splat far off-screen (no tiles) except ``ids_on_tile``, which all
    cover tile (1, 1) and its neighbours."""
    means = np.full((n, 2), 5.0, np.float32)
    L = np.tile(np.array([[1.0, 0.0, 1.0]], np.float32), (n, 1))
    rng = np.random.default_rng(0)
    sel = np.asarray(ids_on_tile)
    # pixel ~ (24, 24) +- 4: means2d in [-1, 1] maps to [0, W]
    means[sel, 0] = (24 + rng.uniform(-4, 4, len(sel))) / (W / 2) - 1
    means[sel, 1] = (24 + rng.uniform(-4, 4, len(sel))) / (H / 2) - 1
    L[sel] = np.array([3.0, 0.5, 2.0], np.float32)
    colors = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    opac = np.ones((n, 1), np.float32)
    return means, L, colors, opac, H, W


@pytest.mark.parametrize("count", [63, 64, 65, 130])
def test_segment_sort_boundaries(cuda, oracle, count):
    from gsvc_amd import ops
    n = 4000
    ids = np.random.default_rng(count).choice(n, count, replace=False)
    means, L, colors, opac, H, W = _clustered_frame(n, ids)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    tb = _tb(H, W)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(L), H, W, tb,
                                                                      0.01)
    m, gids, bins = _counted(n, xys, radii, tb)
    assert m == ref["m"]
    np.testing.assert_array_equal(N(gids), ref["gids_sorted"])
    np.testing.assert_array_equal(N(bins), ref["bins"][: tb[0] * tb[1]])
    assert (ref["bins"][:, 1] - ref["bins"][:, 0]).max() == count


def _capped_matches(n, xys, radii, tb, ref, keep=256):
    """bin_tiles_counted with tile_cap: every tile holds exactly the first
    min(count, keep) ids of the reference's sorted segment, M uncapped, and
    the buffers are tiles * min(n, keep) ints."""
    from gsvc_amd import ops
    ntiles = tb[0] * tb[1]
    cap = ntiles * min(n, keep)
    gids, bins, meta = ops.bin_tiles_counted(n, xys, radii, tb, cap, keep)
    m, ovf = (int(x) for x in meta.tolist())
    assert m == ref["m"] and ovf == 0 and gids.numel() == cap
    g, b = N(gids), N(bins)
    rb = ref["bins"][:ntiles]
    over = 0
    for t in range(ntiles):
        cnt = rb[t, 1] - rb[t, 0]
        want = ref["gids_sorted"][rb[t, 0]: rb[t, 0] + min(cnt, keep)] if cnt > 0 else []
        got = g[b[t, 0]: b[t, 1]] if b[t, 1] > b[t, 0] else []
        np.testing.assert_array_equal(np.asarray(got), np.asarray(want), err_msg=f"tile {t}")
        over += int(cnt > keep)
    return over


@pytest.mark.parametrize("count", [200, 300, 700])
def test_capped_binning_overflow_tile(cuda, oracle, count):
    """T*256 id buffers: a tile past 256 entries keeps its first 256 ids
    (rebuilt in id order from the bboxes)."""
    from gsvc_amd import ops
    n = 4000
    ids = np.random.default_rng(count).choice(n, count, replace=False)
    means, L, colors, opac, H, W = _clustered_frame(n, ids)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    tb = _tb(H, W)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(L), H, W, tb,
                                                                      0.01)
    over = _capped_matches(n, xys, radii, tb, ref)
    assert (over > 0) == (count > 256)


def test_capped_binning_1080p_dense(cuda, oracle):
    """1080p with large splats (20k, chol x24: hundreds of entries per tile):
    many tiles past 256 entries."""
    from gsvc_amd import ops
    H, W, n = 1080, 1920, 20000
    tb = _tb(H, W)
    means, L, colors, opac = oracle.synthetic_frame(n, seed=n + 3, chol_scale=24.0)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(L), H, W, tb,
                                                                      0.01)
    assert _capped_matches(n, xys, radii, tb, ref) > 0


def test_segment_sort_multi_window(cuda, oracle):
    """Splat ids spanning more than one 4096-word LDS bitmap (131072 ids)."""
    from gsvc_amd import ops
    n = 150000
    ids = np.unique(np.concatenate([np.linspace(0, n - 1, 150).astype(np.int64),
                                    [131071, 131072, 131073]]))
    means, L, colors, opac, H, W = _clustered_frame(n, ids)
    ref = oracle.render_sum(means, L, colors, opac, H, W)
    tb = _tb(H, W)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, T(means), T(L), H, W, tb,
                                                                      0.01)
    m, gids, bins = _counted(n, xys, radii, tb)
    np.testing.assert_array_equal(N(gids), ref["gids_sorted"])
    np.testing.assert_array_equal(N(bins), ref["bins"][: tb[0] * tb[1]])


def test_sized_fallback_same_as_sync_free(cuda):
    """Untagged depths (not known to be zero) take the host-sized sorted path;
    both paths give the same image and gradients."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    z = load_golden("sum_64x96_n300")
    H, W = int(z["H"]), int(z["W"])
    outs, grads = [], []
    for tagged in (True, False):
        m = T(z["means2d"]).requires_grad_(True)
        xys, depths, radii, conics, nth = project_gaussians_2d(m, T(z["L"]), H, W, _tb(H, W))
        if not tagged:
            depths = depths.clone()
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, T(z["colors"]),
                                      T(z["opacity"]), H, W)
        (out * T(z["v_out"])).sum().backward()
        outs.append(out.detach())
        grads.append(m.grad)
    assert torch.equal(outs[0], outs[1])
    # the backward accumulates per-tile records with float atomics: the
    # summation order (not the set of terms) varies between runs
    torch.testing.assert_close(grads[0], grads[1], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(N(outs[0]), z["out_img"], rtol=1e-6, atol=1e-5)


def _op_path_frame(means, L, colors, opac, H, W, bg):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, _tb(H, W))
    out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, colors, opac, H, W,
                                  background=bg)
    out = torch.clamp(out, 0, 1)
    return out.view(-1, H, W, 3).permute(0, 3, 1, 2).contiguous()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("case", ["sum_37x53_n120", "sum_stress_48x48_n700", "1080p_10k",
                                  "1080p_50k"])
def test_render_frame_matches_op_path(cuda, oracle, mode, case):
    from gsvc_amd.render import render_sum_frame
    if case.startswith("sum_"):
        z = load_golden(case)
        H, W = int(z["H"]), int(z["W"])
        means, L, colors, opac = z["means2d"], z["L"], z["colors"], z["opacity"]
    else:
        H, W = 1080, 1920
        n = 10000 if case.endswith("10k") else 50000
        means, L, colors, opac = oracle.synthetic_frame(n, seed=n + 1, rgb_w=2.0)
    bg = torch.ones(3, device="cuda")
    with knobs((0, mode)):
        fast = render_sum_frame(T(means), T(L), T(colors), T(opac), H, W, _tb(H, W), bg)
    with torch.no_grad():
        ref = _op_path_frame(T(means), T(L), T(colors), T(opac), H, W, bg)
    assert fast.shape == (1, 3, H, W) and fast.is_contiguous()
    assert torch.equal(fast, ref)


@pytest.mark.parametrize("case", ["sum_trained_like_48x80_n200", "1080p_50k", "1080p_50k_big"])
def test_render_frame_splat_order(cuda, oracle, case, monkeypatch):
    """The render with the training path's splat order (gsvc_render_frame_sum_ex:
    a refreshing call, then ordered calls with windowed slot atomics, large
    splats inserting directly) is bit-identical to the op path, call after call."""
    from gsvc_amd import train as Tr
    from gsvc_amd.render import render_sum_frame
    if case.startswith("sum_"):
        z = load_golden(case)
        H, W = int(z["H"]), int(z["W"])
        means, L, colors, opac = z["means2d"], z["L"], z["colors"], z["opacity"]
    else:
        H, W, n = 1080, 1920, 50000
        means, L, colors, opac = oracle.synthetic_frame(n, seed=n + 5, rgb_w=2.0,
                                                        chol_scale=6.0 if case.endswith("big") else 1.0)
    bg = torch.ones(3, device="cuda")
    with torch.no_grad():
        ref = _op_path_frame(T(means), T(L), T(colors), T(opac), H, W, bg)
    monkeypatch.setattr(Tr, "ORDER_REFRESH_EVERY", 3)
    for _ in range(7):  # refresh, ordered, ordered, refresh + ordered, ...
        fast = render_sum_frame(T(means), T(L), T(colors), T(opac), H, W, _tb(H, W), bg)
        assert torch.equal(fast, ref)


def test_render_frame_empty_is_background(cuda):
    from gsvc_amd.render import render_sum_frame
    z = load_golden("sum_empty_32x32_n10")
    bg = torch.tensor([0.25, 1.5, -0.5], device="cuda")
    fast = render_sum_frame(T(z["means2d"]), T(z["L"]), T(z["colors"]), T(z["opacity"]), 32, 32,
                            _tb(32, 32), bg)
    with torch.no_grad():
        ref = _op_path_frame(T(z["means2d"]), T(z["L"]), T(z["colors"]), T(z["opacity"]), 32, 32,
                             bg)
    assert torch.equal(fast, ref)
    np.testing.assert_array_equal(N(fast)[0, :, 0, 0], [0.25, 1.0, 0.0])


@pytest.mark.parametrize("H,W,n", [(72, 120, 500), (1080, 1920, 10000), (1080, 1920, 50000)])
def test_frame_model_forward_no_grad_matches_autograd(cuda, H, W, n):
    """The fused frame entry (tanh, + bound, * rgb_W in its kernel) against
    GaussianVideoFrame's op-by-op autograd forward, after some training so
    rgb_W and the Cholesky factors are not at their init values."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    model = make_frame_model(H, W, n, cuda, seed=3, isdensity=True)
    gt = synthetic_gt(H, W, 5, cuda)
    for it in range(1, 4):
        model.train_iter(gt, it)
    with torch.no_grad():
        fast = model()["render"]
        again = model()["render"]  # workspace reuse (counters left at zero)
    slow = model()["render"]
    assert slow.requires_grad
    assert torch.equal(fast, slow.detach())
    assert torch.equal(again, fast)


def test_frame_workspace_reuse_across_sizes(cuda):
    from gsvc_amd.frame import make_frame_model
    a = make_frame_model(72, 120, 300, cuda, seed=4)
    b = make_frame_model(40, 56, 200, cuda, seed=5)
    with torch.no_grad():
        ra = a()["render"]
        rb = b()["render"]
        ra2 = a()["render"]
        rb2 = b()["render"]
    assert torch.equal(ra, ra2) and torch.equal(rb, rb2)
    assert torch.equal(rb, b()["render"].detach())


def test_tanh_matches_torch(cuda):
    """The frame kernel's tanhf against torch.tanh, bit for bit, over a
    sweep of magnitudes (the activation of _xyz)."""
    from gsvc_amd.render import render_frame_sum
    x = torch.cat([torch.linspace(-12, 12, 20001), torch.randn(20000) * 3,
                   torch.tensor([0.0, -0.0, 1e-30, -1e-30, 1e-8, 20.0, -20.0])]).cuda()
    n = x.numel() // 2
    xyz = x[: 2 * n].view(n, 2)
    # render a 16x16 frame: means2d only matter through xys; compare xys via
    # the op path instead -- tanh is checked on the projected centres
    from gsvc_amd import ops
    ref = ops.project_gaussians_2d_forward(n, torch.tanh(xyz), torch.ones(n, 3, device="cuda"),
                                           16, 16, (1, 1, 1), 0.01)[0]
    out = render_frame_sum(xyz, torch.ones(n, 3, device="cuda"), torch.zeros(n, 3, device="cuda"),
                           16, 16, torch.zeros(3, device="cuda"))
    assert out.shape == (1, 3, 16, 16)
    from gsvc_amd.render import _workspaces
    fw = _workspaces[(0, torch.cuda.current_stream().cuda_stream)]
    # counts + M slots (256-aligned), then one tile's slab region: the 8-record
    # head and the 256-record body (frame.h slab_frame_f4), then its overflow
    # ids (768 ints: slots 256 .. 1023), each 256-aligned
    off = 256 + ((8 + 256) * 48 + 255) // 256 * 256 + (768 * 4 + 255) // 256 * 256
    xys = fw.buf[off: off + 8 * n].view(torch.float32).view(n, 2)
    assert torch.equal(xys, ref)


@pytest.mark.parametrize("n,count", [(4000, 64), (4000, 65), (4000, 300), (150000, 150),
                                     (150000, 600)])
def test_render_frame_in_kernel_sort(cuda, oracle, n, count):
    """The frame path leaves each tile's ids in fill order and the rasterizer
    sorts them (shuffle ranks <= 64 entries, LDS bitmap in 16384-id windows
    above, stopping at 256): clustered tiles with ids spread over 150k splats
    against the op path (sorted by the separate segment sort)."""
    from gsvc_amd.render import render_sum_frame
    ids = np.unique(np.random.default_rng(count).choice(n, count, replace=False))
    means, L, colors, opac, H, W = _clustered_frame(n, ids)
    bg = torch.ones(3, device="cuda")
    fast = render_sum_frame(T(means), T(L), T(colors), T(opac), H, W, _tb(H, W), bg)
    with torch.no_grad():
        ref = _op_path_frame(T(means), T(L), T(colors), T(opac), H, W, bg)
    assert torch.equal(fast, ref)
    # and against the oracle image (clamped, planar)
    o = oracle.render_sum(means, L, colors, opac, H, W)["out"]
    np.testing.assert_allclose(N(fast)[0], np.clip(o, 0, 1).transpose(2, 0, 1), rtol=1e-6,
                               atol=1e-5)


def _frame_models(sizes, H, W, seed, cluster_frame=None):
    g = torch.Generator().manual_seed(seed)
    xyz, chol, feat = [], [], []
    for b, n in enumerate(sizes):
        x = torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5) * 0.999)
        c = torch.rand(n, 3, generator=g)
        if b == 1 and n:  # a frame whose splats are all degenerate: M = 0, background
            c = -torch.tensor([0.5, 0.0, 0.5]).expand(n, 3).clone()
        if b == cluster_frame:  # > 256 entries on the tiles around one spot
            k = n // 2
            x[:k] = torch.atanh(torch.full((k, 2), -0.3) + 0.02 * torch.rand(k, 2, generator=g))
            c[:k] = torch.tensor([2.0, 0.2, 1.5])
        xyz.append(x)
        chol.append(c)
        feat.append(torch.rand(n, 3, generator=g))
    return torch.cat(xyz).cuda(), torch.cat(chol).cuda(), torch.cat(feat).cuda()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("H,W,sizes,cluster", [
    (72, 120, [300, 200, 0, 1200, 50], 3),
    (1080, 1920, [10000] * 8, None),
])
def test_render_frames_batch_matches_single(cuda, mode, H, W, sizes, cluster):
    """gsvc_render_frames_sum: every frame of the batch bit-identical to its
    own one-frame render -- empty frames, an all-background frame, tiles past
    256 entries (the id-range brute rebuild of the frame's own splats)."""
    from gsvc_amd.render import render_frame_sum, render_frames_sum
    xyz, chol, feat = _frame_models(sizes, H, W, seed=len(sizes) + H, cluster_frame=cluster)
    bound = torch.tensor([0.5, 0.0, 0.5], device="cuda")
    rgbw = torch.rand(sum(sizes), 1, device="cuda") + 0.5
    bg = torch.tensor([0.3, 0.6, 0.9], device="cuda")
    with knobs((0, mode)):
        outs = [render_frames_sum(xyz, chol, feat, sizes, H, W, bg, cholesky_bound=bound,
                                  rgb_w=rgbw) for _ in range(3)]  # parity slots reused
        off = 0
        for b, n in enumerate(sizes):
            sl = slice(off, off + n)
            one = render_frame_sum(xyz[sl], chol[sl], feat[sl], H, W, bg, cholesky_bound=bound,
                                   rgb_w=rgbw[sl])
            for o in outs:
                assert torch.equal(o[b], one[0]), (b, n)
            off += n
    if sizes[2] == 0:  # a frame without splats is the background
        assert torch.equal(outs[0][2], bg.view(3, 1, 1).expand(3, H, W))
