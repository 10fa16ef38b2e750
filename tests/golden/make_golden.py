"""Generate the golden fixtures under tests/golden/ (run in the build container only).

    python tests/golden/make_golden.py

This script imports the reference Python from /root/reference (read-only) and
is never run by the tests or on the GPU box; only its outputs (.npz data) are
committed.  Five kinds of fixtures are produced:

1. ``sum_*.npz`` / ``alpha_*.npz``: the reference's own autograd glue
   (gsplat/project_gaussians_2d.py:59-141, rasterize_sum.py:14-254,
   rasterize.py:14-253, utils.py:12-167, including torch.cumsum / .item() /
   torch.sort / torch.gather and the M<1 background branch) executed on CPU with
   the oracle (oracle/oracle.c) injected as ``gsplat.cuda._backend._C``.  This
   pins the glue semantics; the kernel arithmetic is the oracle's.
2. ``ref_tests_*.npz``: known-answer vectors of the reference's own tests
   (gsplat/tests/test_map_gaussians.py, test_get_tile_bin_edges.py,
   test_cov2d_bounds.py), i.e. the pure-torch ``_torch_impl`` outputs on the
   tests' seed-42 inputs.  These pin the oracle's map/bins/cov2d code.
   ``alpha_*`` additionally stores ``_torch_impl.rasterize_forward`` (the only
   reference-authored CPU rasterizer, per-pixel Python loops) for out_img/final_Ts.
3. ``train_iter_*.npz``: one and two ``GaussianVideo_frame.train_iter`` steps
   (GaussianSplats_Represent.py:191-207, L2 loss, Adan optimizer.py:39-362) of
   the reference model on CPU, oracle injected.
4. ``train_state_1080p_n50k.npz`` (``make_golden.py trained STATE.npz``): the
   state bench.py times -- its 1080p / 50k frame after 2020 training
   iterations, trained on the CPU by the oracle (tests/analysis/train_oracle_state.py)
   -- and the reference's own forward / backward / three train_iter steps
   from it (make_trained_state_case).
5. ``prune_controls.npz``: ``removal_control`` / ``adaptive_control``
   (GaussianSplats_Represent.py:98-172) of the reference model on CPU with a
   stable torch.sort, on rgb_W with tie groups, NaN, +-0 and underflowing
   squares (``python tests/golden/make_golden.py prune`` remakes only this).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden")
REF = "/root/reference"

sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402


def _install_stubs():
    jt = types.ModuleType("jaxtyping")

    class _Ann:
        def __class_getitem__(cls, item):
            return cls

    jt.Float = _Ann
    jt.Int = _Ann
    sys.modules["jaxtyping"] = jt
    # modules imported by the reference's top-level utils.py / drivers that are
    # absent here; none of them is on the L2 train_iter path.
    msssim = types.ModuleType("pytorch_msssim")
    msssim.ms_ssim = msssim.ssim = lambda *a, **k: (_ for _ in ()).throw(RuntimeError("no msssim"))
    sys.modules["pytorch_msssim"] = msssim
    sys.modules["cv2"] = types.ModuleType("cv2")


def _np(t):
    return t.detach().cpu().numpy()


class OracleC:
    """Stand-in for the reference's compiled ``gsplat.csrc`` module: each op
    has the reference binding's signature (bindings.cu) and runs the oracle."""

    @staticmethod
    def project_gaussians_2d_forward(num_points, means2d, L, img_h, img_w, tile_bounds, clip):
        xys, depths, radii, conics, nth = O.project_2d_forward(_np(means2d), _np(L), img_h, img_w, tile_bounds)
        return tuple(torch.from_numpy(a) for a in (xys, depths, radii, conics, nth))

    @staticmethod
    def project_gaussians_2d_backward(num_points, means2d, L, img_h, img_w, radii, conics,
                                      v_xy, v_depth, v_conic):
        v_cov2d, v_mean2d, v_L = O.project_2d_backward(_np(L), img_h, img_w, _np(radii), _np(conics),
                                                       _np(v_xy), _np(v_conic))
        return torch.from_numpy(v_cov2d), torch.from_numpy(v_mean2d), torch.from_numpy(v_L)

    @staticmethod
    def map_gaussian_to_intersects(num_points, num_intersects, xys, depths, radii, cum, tile_bounds):
        isect, gids = O.map_intersects(_np(xys), _np(depths), _np(radii), _np(cum), tile_bounds,
                                       num_intersects)
        return torch.from_numpy(isect), torch.from_numpy(gids)

    @staticmethod
    def get_tile_bin_edges(num_intersects, isect_sorted):
        s = _np(isect_sorted)
        rows = max(num_intersects, int((s >> 32).max()) + 1 if s.size else 0)
        return torch.from_numpy(O.tile_bin_edges(s, rows))

    @staticmethod
    def compute_cov2d_bounds(num_pts, covs):
        c, r = O.cov2d_bounds(_np(covs))
        return torch.from_numpy(c), torch.from_numpy(r)

    @staticmethod
    def _pad_bins(bins, tb):
        b = _np(bins)
        t = tb[0] * tb[1]
        if b.shape[0] < t:
            b = np.concatenate([b, np.zeros((t - b.shape[0], 2), np.int32)])
        return b

    @classmethod
    def rasterize_sum_forward(cls, tile_bounds, block, img_size, gids, bins, xys, conics, colors,
                              opac, bg):
        out, Ts, idx = O.raster_sum_forward(tile_bounds, img_size[1], img_size[0], _np(gids),
                                            cls._pad_bins(bins, tile_bounds), _np(xys), _np(conics),
                                            _np(colors), _np(opac))
        return torch.from_numpy(out), torch.from_numpy(Ts), torch.from_numpy(idx)

    @classmethod
    def rasterize_sum_backward(cls, img_h, img_w, bh, bw, gids, bins, xys, conics, colors, opac, bg,
                               final_Ts, final_idx, v_out, v_out_alpha):
        tb = ((img_w + bw - 1) // bw, (img_h + bh - 1) // bh, 1)
        v = O.raster_sum_backward(tb, img_h, img_w, _np(gids), cls._pad_bins(bins, tb), _np(xys),
                                  _np(conics), _np(colors), _np(opac), _np(final_idx),
                                  _np(v_out.contiguous()))
        return tuple(torch.from_numpy(a.astype(np.float32)) for a in v)

    @classmethod
    def rasterize_forward(cls, tile_bounds, block, img_size, gids, bins, xys, conics, colors, opac, bg):
        out, Ts, idx = O.raster_forward(tile_bounds, img_size[1], img_size[0], _np(gids),
                                        cls._pad_bins(bins, tile_bounds), _np(xys), _np(conics),
                                        _np(colors), _np(opac), _np(bg))
        return torch.from_numpy(out), torch.from_numpy(Ts), torch.from_numpy(idx)

    @classmethod
    def rasterize_backward(cls, img_h, img_w, bh, bw, gids, bins, xys, conics, colors, opac, bg,
                           final_Ts, final_idx, v_out, v_out_alpha):
        tb = ((img_w + bw - 1) // bw, (img_h + bh - 1) // bh, 1)
        v = O.raster_backward(tb, img_h, img_w, _np(gids), cls._pad_bins(bins, tb), _np(xys),
                              _np(conics), _np(colors), _np(opac), _np(bg), _np(final_Ts),
                              _np(final_idx), _np(v_out.contiguous()), _np(v_out_alpha.contiguous()))
        return tuple(torch.from_numpy(a.astype(np.float32)) for a in v)


def _import_reference():
    _install_stubs()
    # the reference package must win over this repo's own drop-in ``gsplat``
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != REPO]
    sys.path.insert(0, os.path.join(REF, "gsplat"))
    import gsplat  # noqa: F401
    import gsplat.cuda._backend as backend
    assert os.path.abspath(gsplat.__file__).startswith(REF), gsplat.__file__
    backend._C = OracleC()
    # torch.sort(int64) is NOT stable on CPU in this torch build (equal keys get
    # permuted).  The reference ran it on CUDA, where torch.sort of more than 32
    # elements uses stable merge / radix sorts (WarpMergeSort, MediumRadixSort,
    # cub segmented radix sort), so the reference's tie order is input order.
    # Emulate that inside the reference's gsplat.utils (utils.py:164).
    import gsplat.utils as gu

    class _StableTorch(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

        @staticmethod
        def sort(x, *a, **k):
            k.setdefault("stable", True)
            return torch.sort(x, *a, **k)

    gu.torch = _StableTorch("torch_stable_sort")
    return gsplat


def make_sum_case(gs, name, H, W, means, L, colors, opac, seed):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    tb = O.tile_bounds(H, W)
    m = torch.from_numpy(means).requires_grad_(True)
    l = torch.from_numpy(L).requires_grad_(True)
    c = torch.from_numpy(colors).requires_grad_(True)
    o = torch.from_numpy(opac).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
    xys.retain_grad()
    conics.retain_grad()
    out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                  background=torch.ones(3), return_alpha=False)
    g = torch.Generator().manual_seed(seed + 2)
    v_out = torch.randn(out.shape, generator=g)
    (out * v_out).sum().backward()
    rec = dict(H=H, W=W, means2d=means, L=L, colors=colors, opacity=opac, v_out=_np(v_out),
               xys=_np(xys), depths=_np(depths), radii=_np(radii), conics=_np(conics),
               num_tiles_hit=_np(nth), out_img=_np(out),
               v_xy=_np(xys.grad) if xys.grad is not None else np.zeros_like(_np(xys)),
               v_conic=_np(conics.grad) if conics.grad is not None else np.zeros_like(_np(conics)),
               v_means2d=_np(m.grad), v_L=_np(l.grad), v_colors=_np(c.grad), v_opacity=_np(o.grad))
    # binning intermediates through the reference glue (utils.py:99-167)
    from gsplat.utils import bin_and_sort_gaussians, compute_cumulative_intersects
    M, cum = compute_cumulative_intersects(nth.detach())
    rec["num_intersects"] = np.int64(M)
    rec["cum_tiles_hit"] = _np(cum)
    if M >= 1:
        isect, gids, isect_s, gids_s, bins = bin_and_sort_gaussians(
            m.shape[0], M, xys.detach(), depths.detach(), radii.detach(), cum, tb)
        rec.update(isect_ids=_np(isect), gaussian_ids=_np(gids), isect_ids_sorted=_np(isect_s),
                   gaussian_ids_sorted=_np(gids_s))
        b = OracleC._pad_bins(bins, tb)
        rec["tile_bins"] = b
        _, Ts, idx = O.raster_sum_forward(tb, H, W, _np(gids_s), b, _np(xys), _np(conics), colors, opac)
        rec["final_idx"] = idx
        rec["alpha_margin"] = O.sum_min_margin(tb, H, W, _np(gids_s), b, _np(xys), _np(conics), opac)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    print(f"{name}: N={means.shape[0]} M={M} out[{H}x{W}] sum={float(out.sum()):.4f}")


def make_alpha_case(gs, name, H, W, means, L, colors, opac, seed):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize import rasterize_gaussians
    from gsplat import _torch_impl
    from gsplat.utils import bin_and_sort_gaussians, compute_cumulative_intersects
    tb = O.tile_bounds(H, W)
    bg = np.array([0.2, 0.5, 0.9], np.float32)
    m = torch.from_numpy(means).requires_grad_(True)
    l = torch.from_numpy(L).requires_grad_(True)
    c = torch.from_numpy(colors).requires_grad_(True)
    o = torch.from_numpy(opac).requires_grad_(True)
    xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
    xys.retain_grad()
    conics.retain_grad()
    out, alpha = rasterize_gaussians(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                     background=torch.from_numpy(bg), return_alpha=True)
    g = torch.Generator().manual_seed(seed + 2)
    v_out = torch.randn(out.shape, generator=g)
    v_alpha = torch.randn(alpha.shape, generator=g)
    ((out * v_out).sum() + (alpha * v_alpha).sum()).backward()
    M, cum = compute_cumulative_intersects(nth.detach())
    isect, gids, isect_s, gids_s, bins = bin_and_sort_gaussians(
        m.shape[0], M, xys.detach(), depths.detach(), radii.detach(), cum, tb)
    b = OracleC._pad_bins(bins, tb)
    # reference-authored CPU rasterizer (per-pixel Python loops)
    t_out, t_Ts, _ = _torch_impl.rasterize_forward(
        tb, (16, 16, 1), (W, H, 1), gids_s, torch.from_numpy(b), xys.detach(), conics.detach(),
        c.detach(), o.detach(), torch.from_numpy(bg))
    _, Ts, idx = O.raster_forward(tb, H, W, _np(gids_s), b, _np(xys), _np(conics), colors, opac, bg)
    rec = dict(H=H, W=W, means2d=means, L=L, colors=colors, opacity=opac, background=bg,
               v_out=_np(v_out), v_alpha=_np(v_alpha), xys=_np(xys), conics=_np(conics),
               radii=_np(radii), num_tiles_hit=_np(nth), gaussian_ids_sorted=_np(gids_s),
               tile_bins=b, out_img=_np(out), out_alpha=_np(alpha), final_Ts=Ts, final_idx=idx,
               torch_impl_out_img=_np(t_out), torch_impl_final_Ts=_np(t_Ts),
               v_xy=_np(xys.grad), v_conic=_np(conics.grad), v_means2d=_np(m.grad), v_L=_np(l.grad),
               v_colors=_np(c.grad), v_opacity=_np(o.grad))
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    err = float(np.abs(_np(t_out) - _np(out)).max())
    print(f"{name}: N={means.shape[0]} M={M} |oracle - _torch_impl| max = {err:.3e}")


def make_alpha_dense_cases(gs):
    """Alpha compositing past one 256-entry batch (forward.cu:252-374 loops over
    every batch of the tile) and with the T <= 1e-4 early stop firing: 400
    large splats over a 32x32 frame (4 tiles, ~400 entries each).
    ``alpha_32x32_stop``: opaque splats, most pixels stop within a few
    entries; ``alpha_32x32_deep``: faint splats, T stays above 1e-4 past entry
    256.  Each fixture stores the per-pixel entry position the compositing
    reached (final_idx - tile start) and whether it stopped early."""
    rng = np.random.default_rng(21)
    n = 400
    for name, lo, hi in (("alpha_32x32_stop", 0.6, 1.0), ("alpha_32x32_deep", 0.004, 0.012)):
        means = rng.uniform(-0.6, 0.6, (n, 2)).astype(np.float32)
        L = (rng.random((n, 3), dtype=np.float32) * np.array([2, 0.5, 2], np.float32)
             + np.array([4.0, 0, 4.0], np.float32)).astype(np.float32)
        colors = rng.random((n, 3), dtype=np.float32)
        opac = rng.uniform(lo, hi, (n, 1)).astype(np.float32)
        make_alpha_case(gs, name, 32, 32, means, L, colors, opac, 21)
        z = dict(np.load(os.path.join(OUT, name + ".npz")))
        tb = O.tile_bounds(32, 32)
        b = z["tile_bins"]
        ty, tx = np.meshgrid(np.arange(32) // 16, np.arange(32) // 16, indexing="ij")
        tile = ty * tb[0] + tx
        start = b[tile, 0]
        count = b[tile, 1] - b[tile, 0]
        z["reach"] = (z["final_idx"] - start).astype(np.int32)
        z["tile_count"] = count.astype(np.int32)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **z)
        print(f"{name}: entries/tile {count.min()}..{count.max()}, reach max {z['reach'].max()}, "
              f"final_Ts min {z['final_Ts'].min():.2e}")


def make_ref_tests_case():
    """Inputs and expected outputs of gsplat/tests/test_map_gaussians.py:8-73,
    test_get_tile_bin_edges.py:9-81 and test_cov2d_bounds.py:8-35 (seed 42)."""
    from gsplat import _torch_impl
    torch.manual_seed(42)
    num_points = 100
    means3d = torch.randn((num_points, 3))
    scales = torch.randn((num_points, 3))
    glob_scale = 0.3
    quats = torch.randn((num_points, 4))
    quats /= torch.linalg.norm(quats, dim=-1, keepdim=True)
    viewmat = torch.eye(4)
    projmat = torch.eye(4)
    fx, fy = 3.0, 3.0
    H, W = 512, 512
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    (_cov3d, xys, depths, radii, conics, nth, masks) = _torch_impl.project_gaussians_forward(
        means3d, scales, glob_scale, quats, viewmat, projmat, fx, fy, (H, W), tb, 0.01)
    xys, depths, radii, nth = xys[masks], depths[masks], radii[masks], nth[masks]
    n = int(masks.sum())
    cum = torch.cumsum(nth, dim=0, dtype=torch.int32)
    M = int(cum[-1])
    isect, gids = _torch_impl.map_gaussian_to_intersects(n, xys, depths.contiguous(), radii, cum, tb)
    isect_s, order = torch.sort(isect, stable=True)
    gids_s = torch.gather(gids, 0, order)
    bins = _torch_impl.get_tile_bin_edges(M, isect_s)
    # _torch_impl.get_tile_bin_edges breaks at k=M-1 before the tile-change
    # check (_torch_impl.py:341-343); flag whether that quirk is exercised.
    last_change = bool(M > 1 and int(isect_s[-1] >> 32) != int(isect_s[-2] >> 32))
    torch.manual_seed(42)
    _covs2d = torch.rand((100, 2, 2), dtype=torch.float32)
    covs2d = torch.stack([torch.triu(_covs2d)[:, 0, 0], torch.triu(_covs2d)[:, 0, 1],
                          torch.triu(_covs2d)[:, 1, 1]], dim=-1)
    _conic, _radii, _mask = _torch_impl.compute_cov2d_bounds(_covs2d)
    rec = dict(tile_bounds=np.array(tb, np.int32), num_points=np.int64(n), num_intersects=np.int64(M),
               xys=_np(xys).astype(np.float32), depths=_np(depths).astype(np.float32),
               radii=_np(radii).astype(np.int32), cum_tiles_hit=_np(cum),
               isect_ids=_np(isect), gaussian_ids=_np(gids), isect_ids_sorted=_np(isect_s),
               gaussian_ids_sorted=_np(gids_s), tile_bins=_np(bins),
               bins_last_change_quirk=np.bool_(last_change),
               covs2d=_np(covs2d), cov2d_conic=_np(_conic), cov2d_radii=_np(_radii),
               cov2d_mask=_np(_mask))
    np.savez_compressed(os.path.join(OUT, "ref_tests_seed42.npz"), **rec)
    print(f"ref_tests_seed42: n={n} M={M} last-entry tile change: {last_change}")


def make_train_iter_case(name, H, W, n, seed, isremoval=False):
    sys.path.insert(0, REF)
    import GaussianSplats_Represent as GR
    torch.manual_seed(seed)
    model = GR.GaussianVideo_frame(
        loss_type="L2", opt_type="adan", num_points=n, max_num_points=n, densification_interval=100,
        iterations=10, H=H, W=W, BLOCK_H=16, BLOCK_W=16, device=torch.device("cpu"), lr=1e-3,
        quantize=False, removal_rate=0.1, isdensity=False, isremoval=isremoval)
    init = {k: _np(v).copy() for k, v in model.state_dict().items()}
    yy, xx = np.meshgrid(np.linspace(0, 1, H, dtype=np.float32), np.linspace(0, 1, W, dtype=np.float32),
                         indexing="ij")
    gt = np.stack([0.5 + 0.4 * np.sin(6.0 * xx + 1.0), 0.5 + 0.4 * np.cos(5.0 * yy),
                   0.5 + 0.3 * np.sin(4.0 * (xx + yy))])[None].astype(np.float32)
    gt_t = torch.from_numpy(gt)
    # gradients of one forward/backward (the part of train_iter before Adan)
    img = model.forward()["render"]
    loss0 = GR.loss_fn(img.squeeze(0), gt_t.squeeze(0), "L2", lambda_value=0)
    loss0.backward()
    grads = {k: _np(p.grad).copy() for k, p in model.named_parameters() if p.grad is not None}
    model.optimizer.zero_grad(set_to_none=True)
    rec = dict(H=H, W=W, gt=gt, render0=_np(img), loss0=np.float64(loss0.item()))
    for k, v in init.items():
        rec["init_" + k] = v
    for k, v in grads.items():
        rec["grad_" + k] = v
    losses, psnrs = [], []
    for it in (1, 2):
        loss, psnr = model.train_iter(gt_t, it)
        losses.append(float(loss.item()))
        psnrs.append(float(psnr))
        for k, v in model.state_dict().items():
            rec[f"step{it}_" + k] = _np(v).copy()
    rec["losses"] = np.array(losses)
    rec["psnrs"] = np.array(psnrs)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    print(f"{name}: losses={losses} psnrs={psnrs}")


def synthetic_gt_np(H, W, seed):
    """The bench's target frame (gsvc_amd/frame.py ``synthetic_gt``, CPU torch
    ops, so the same bits on any host with this torch): a sum of 8 seeded
    sinusoids per channel.  Restated here because this script must import the
    reference's ``gsplat``, not the repo's; the fixture stores a checksum that
    tests/test_train_trajectory.py compares with the repo's function."""
    g = torch.Generator().manual_seed(int(seed))
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    chans = []
    for _ in range(3):
        acc = torch.zeros(H, W)
        for _ in range(8):
            fx, fy, ph = (torch.rand(3, generator=g) * torch.tensor([12.0, 12.0, 6.28])).tolist()
            acc += torch.sin(fx * xx + fy * yy + ph)
        chans.append(0.5 + 0.5 * acc / 8)
    return torch.stack(chans)[None].clamp(0, 1)


def make_train_trajectory_case(name, H, W, n, seed, gt_seed, iters, keep=4096):
    """BASELINE configs[2] at full size: ``iters`` reference
    GaussianVideo_frame.train_iter steps (GaussianSplats_Represent.py:191-207:
    forward, L2, backward, PSNR, Adan, StepLR) at H x W with n splats, oracle
    injected, torch.sort stable.  Records per-iteration loss / PSNR, the
    parameters of the first ``keep`` splats after the last step and float64
    checksums of every parameter (the whole 50k-splat state would be 1.8 MB)."""
    import time
    sys.path.insert(0, REF)
    import GaussianSplats_Represent as GR
    torch.manual_seed(seed)
    model = GR.GaussianVideo_frame(
        loss_type="L2", opt_type="adan", num_points=n, max_num_points=n, densification_interval=100,
        iterations=30000, H=H, W=W, BLOCK_H=16, BLOCK_W=16, device=torch.device("cpu"), lr=1e-3,
        quantize=False, removal_rate=0.1, isdensity=False, isremoval=False)
    gt = synthetic_gt_np(H, W, gt_seed)
    losses, psnrs = [], []
    t0 = time.time()
    for it in range(1, iters + 1):
        loss, psnr = model.train_iter(gt, it)
        losses.append(float(loss.item()))
        psnrs.append(float(psnr))
    rec = dict(H=H, W=W, n=n, seed=seed, gt_seed=gt_seed, iters=iters,
               gt_sum=np.float64(gt.double().sum()), gt_sq=np.float64((gt.double() ** 2).sum()),
               losses=np.array(losses), psnrs=np.array(psnrs))
    for k, v in model.state_dict().items():
        a = _np(v)
        if a.ndim == 2 and a.shape[0] == n:
            rec["final_" + k] = a[:keep].copy()
            rec["sum_" + k] = np.float64(a.astype(np.float64).sum())
            rec["abssum_" + k] = np.float64(np.abs(a.astype(np.float64)).sum())
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    print(f"{name}: {iters} iters in {time.time() - t0:.1f} s, psnrs={[round(p, 4) for p in psnrs]}")


TRAINED_CROPS = ((0, 0), (512, 960), (1064, 1904), (300, 1500), (777, 123))


def make_trained_state_case(state_path, name="train_state_1080p_n50k", steps=3, keep=4096):
    """BASELINE configs[2] at the state bench.py times: the bench's 1080p / 50k
    frame (seed 1000, target seed 8) after its settle + warmup iterations
    (trained density, M ~ 230-240k), trained on the CPU by the oracle's
    train_iter_sum (tests/analysis/train_oracle_state.py), loaded here into the
    reference model.  Records, from the reference's own Python with the oracle
    injected (GaussianSplats_Represent.py:83-90,191-207, fresh Adan):

    * the forward's image checksums and five 16x16-aligned crops, M, and the
      L2 loss / PSNR;
    * the parameter gradients of that loss (the part of train_iter before Adan);
    * ``steps`` train_iter steps: loss and PSNR per step, the first ``keep``
      splats' parameters after the last step, float64 sums of all of them."""
    import time
    sys.path.insert(0, REF)
    import GaussianSplats_Represent as GR
    st = np.load(state_path)
    n = int(st["_xyz"].shape[0])
    H, W = 1080, 1920
    torch.manual_seed(0)
    model = GR.GaussianVideo_frame(
        loss_type="L2", opt_type="adan", num_points=n, max_num_points=n, densification_interval=100,
        iterations=30000, H=H, W=W, BLOCK_H=16, BLOCK_W=16, device=torch.device("cpu"), lr=1e-3,
        quantize=False, removal_rate=0.1, isdensity=False, isremoval=False)
    with torch.no_grad():
        for k in ("_xyz", "_cholesky", "_features_dc"):
            getattr(model, k).copy_(torch.from_numpy(st[k]))
        assert np.all(st["rgb_W"] == 1.0)
    gt_seed = int(st["gt_seed"])
    gt = synthetic_gt_np(H, W, gt_seed)
    t0 = time.time()
    img = model.forward()["render"]
    loss0 = GR.loss_fn(img.squeeze(0), gt.squeeze(0), "L2", lambda_value=0)
    loss0.backward()
    grads = {k: _np(p.grad).copy() for k, p in model.named_parameters() if p.grad is not None}
    model.optimizer.zero_grad(set_to_none=True)
    im = _np(img)[0].astype(np.float64)
    from gsplat.utils import compute_cumulative_intersects
    with torch.no_grad():
        _, _, _, _, nth = GR.project_gaussians_2d(model.get_xyz, model.get_cholesky_elements, H, W,
                                                  model.tile_bounds)
        M, _ = compute_cumulative_intersects(nth)
    rec = dict(H=H, W=W, n=n, gt_seed=gt_seed, iters=int(st["iters"]), seed=int(st["seed"]),
               M=np.int64(M), loss0=np.float64(loss0.item()),
               render_sum=im.sum(axis=(1, 2)), render_sq=(im ** 2).sum(axis=(1, 2)),
               crops=np.array(TRAINED_CROPS, np.int32),
               render_crops=np.stack([_np(img)[0][:, y:y + 16, x:x + 16] for y, x in TRAINED_CROPS]),
               gt_sum=np.float64(gt.double().sum()))
    for k in ("_xyz", "_cholesky", "_features_dc"):
        rec["state_" + k] = st[k]
        rec["grad_" + k] = grads[k]
    losses, psnrs = [], []
    for it in range(int(st["iters"]) + 1, int(st["iters"]) + 1 + steps):
        loss, psnr = model.train_iter(gt, it)
        losses.append(float(loss.item()))
        psnrs.append(float(psnr))
    rec["losses"] = np.array(losses)
    rec["psnrs"] = np.array(psnrs)
    for k in ("_xyz", "_cholesky", "_features_dc"):
        a = _np(getattr(model, k))
        rec["final_" + k] = a[:keep].copy()
        rec["sum_" + k] = np.float64(a.astype(np.float64).sum())
        rec["abssum_" + k] = np.float64(np.abs(a.astype(np.float64)).sum())
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
    print(f"{name}: N={n} M={M} loss0={float(loss0):.6g} psnrs={psnrs} ({time.time() - t0:.1f} s)")


def make_prune_cases():
    """removal_control / adaptive_control (GaussianSplats_Represent.py:98-172)
    of the reference model on CPU, torch.sort made stable (the GPU's radix
    sort; CPU torch.sort permutes ties).  rgb_W holds tie groups straddling the
    cut (+-0.01: densified splats start at 0.01), a NaN, +-0 and values whose
    square underflows.  Records the parameters before and after."""
    sys.path.insert(0, REF)
    import GaussianSplats_Represent as GR

    class _StableTorch(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

        @staticmethod
        def sort(x, *a, **k):
            k.setdefault("stable", True)
            return torch.sort(x, *a, **k)

    GR.torch = _StableTorch("torch_stable_sort")
    rec = {}
    cases = [("removal", 100, 4000, 4000), ("removal", 4000, 3800, 4000),
             ("adaptive", 600, 4400, 4000), ("adaptive", 1000, 4100, 4000)]
    for ci, (kind, it, n, mx) in enumerate(cases):
        torch.manual_seed(100 + ci)
        model = GR.GaussianVideo_frame(
            loss_type="L2", opt_type="adan", num_points=n, max_num_points=mx,
            densification_interval=100, iterations=10, H=32, W=32, BLOCK_H=16, BLOCK_W=16,
            device=torch.device("cpu"), lr=1e-3, quantize=False, removal_rate=0.1,
            isdensity=kind == "adaptive", isremoval=kind == "removal")
        rng = np.random.default_rng(200 + ci)
        w = rng.choice(np.array([-0.03, -0.01, 0.01, 0.02, 0.5, 1.0], np.float32), n)
        w = w + (rng.random(n) < 0.5) * rng.normal(0, 0.2, n).astype(np.float32)
        w[rng.choice(n, 6, replace=False)] = np.array([np.nan, 0.0, -0.0, 3e-25, 1e-25, 2e-20],
                                                      np.float32)
        with torch.no_grad():
            model.rgb_W.data = torch.from_numpy(w.astype(np.float32)).reshape(n, 1)
        for k, v in model.state_dict().items():
            rec[f"c{ci}_in_{k}"] = _np(v).copy()
        rec[f"c{ci}_in_rgb_W"] = _np(model.rgb_W).copy()
        (model.removal_control if kind == "removal" else model.adaptive_control)(it)
        rec[f"c{ci}_out_rgb_W"] = _np(model.rgb_W).copy()
        for k, v in model.state_dict().items():
            rec[f"c{ci}_out_{k}"] = _np(v).copy()
        rec[f"c{ci}_meta"] = np.array([0 if kind == "removal" else 1, it, n, mx])
        print(f"prune case {ci}: {kind} iter {it}: {n} -> {model._xyz.shape[0]}")
    np.savez_compressed(os.path.join(OUT, "prune_controls.npz"), **rec)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "prune":
        _import_reference()
        make_prune_cases()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "alpha":
        gs = _import_reference()
        make_alpha_dense_cases(gs)
        return
    if len(sys.argv) > 2 and sys.argv[1] == "trained":
        _import_reference()
        make_trained_state_case(sys.argv[2])
        return
    if len(sys.argv) > 1 and sys.argv[1] == "trajectory":
        _import_reference()
        make_train_trajectory_case("train_traj_1080p_n50k", 1080, 1920, 50000, 7, 8, 40)
        return
    gs = _import_reference()
    os.makedirs(OUT, exist_ok=True)
    make_ref_tests_case()
    cases = [
        ("sum_64x96_n300", 64, 96, 300, 0, 1.0, 1.0),
        ("sum_37x53_n120", 37, 53, 120, 1, 1.0, 1.0),
        ("sum_256x256_n1000", 256, 256, 1000, 2, 1.0, 1.0),
        ("sum_trained_like_48x80_n200", 48, 80, 200, 3, 1.0, 8.0),
    ]
    for name, H, W, n, seed, rgbw, chol in cases:
        means, L, colors, opac = O.synthetic_frame(n, seed, rgb_w=rgbw, chol_scale=chol)
        make_sum_case(gs, name, H, W, means, L, colors, opac, seed)
    # >256 splats in one tile: the sum path renders only the first 256
    rng = np.random.default_rng(7)
    n = 700
    means = np.concatenate([rng.uniform(-0.15, 0.05, (600, 2)), rng.uniform(-1, 1, (100, 2))]).astype(np.float32)
    L = (rng.random((n, 3), dtype=np.float32) + np.array([0.5, 0, 0.5], np.float32)).astype(np.float32)
    colors = rng.random((n, 3), dtype=np.float32)
    opac = rng.uniform(0.3, 1.0, (n, 1)).astype(np.float32)
    make_sum_case(gs, "sum_stress_48x48_n700", 48, 48, means, L, colors, opac, 7)
    # M < 1: every splat degenerate (det == 0) -> background branch
    z = np.zeros((10, 3), np.float32)
    make_sum_case(gs, "sum_empty_32x32_n10", 32, 32, np.zeros((10, 2), np.float32), z,
                  np.ones((10, 3), np.float32), np.ones((10, 1), np.float32), 9)
    means, L, colors, opac = O.synthetic_frame(40, 11)
    opac = np.random.default_rng(11).uniform(0.2, 1.0, (40, 1)).astype(np.float32)
    make_alpha_case(gs, "alpha_32x48_n40", 32, 48, means, (L * 3).astype(np.float32), colors, opac, 11)
    make_train_iter_case("train_iter_64x64_n200", 64, 64, 200, 5)
    make_prune_cases()


if __name__ == "__main__":
    main()
