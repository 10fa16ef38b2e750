"""ctypes/numpy wrapper around oracle/liboracle.so.

TEST INFRASTRUCTURE ONLY: the parity checker for the HIP path.  Only tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import it.

Every function mirrors one reference operator (paths relative to
/root/reference/gsplat/gsplat):
  project_2d_forward / backward   project_gaussians_2d.py:63-141 -> cuda/csrc/foward2d.cu, backward2d.cu
  cumulative_intersects           utils.py:99-118
  map_intersects                  utils.py:12-50 -> cuda/csrc/forward.cu:100-136
  sort_pairs                      utils.py:164-165 (torch.sort + gather)
  tile_bin_edges                  utils.py:53-74 -> cuda/csrc/forward.cu:141-163
  bin_and_sort                    utils.py:121-167
  raster_sum_forward / backward   rasterize_sum.py:92-254 -> forward.cu:512-627, backward.cu:696-862
  raster_forward / backward       rasterize.py:89-253 -> forward.cu:252-374, backward.cu:138-315
  prune_keep                      /root/reference/GaussianSplats_Represent.py:101-125, 149-166
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

F32 = np.float32
I32 = np.int32
I64 = np.int64
F64 = np.float64


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))
        ):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.oracle_set_threads(1)  # single-threaded unless a caller asks for more
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the per-tile oracle loops (sum forward); results do
    not depend on it.  Returns the count in effect."""
    return int(lib().oracle_set_threads(int(n)))


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def tile_bounds(img_h: int, img_w: int, block: int = 16):
    return ((img_w + block - 1) // block, (img_h + block - 1) // block, 1)


def project_2d_forward(means2d, L, img_h, img_w, tb):
    means2d = _c(means2d, F32)
    L = _c(L, F32)
    n = means2d.shape[0]
    xys = np.zeros((n, 2), F32)
    depths = np.zeros((n,), F32)
    radii = np.zeros((n,), I32)
    conics = np.zeros((n, 3), F32)
    nth = np.zeros((n,), I32)
    lib().oracle_project_2d_forward(
        ctypes.c_int(n), _p(means2d), _p(L), ctypes.c_int(img_h), ctypes.c_int(img_w),
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]),
        _p(xys), _p(depths), _p(radii), _p(conics), _p(nth))
    return xys, depths, radii, conics, nth


def project_2d_backward(L, img_h, img_w, radii, conics, v_xy, v_conic):
    L = _c(L, F32)
    radii = _c(radii, I32)
    conics = _c(conics, F32)
    v_xy = _c(v_xy, F32)
    v_conic = _c(v_conic, F32)
    n = L.shape[0]
    v_cov2d = np.zeros((n, 3), F32)
    v_mean2d = np.zeros((n, 2), F32)
    v_L = np.zeros((n, 3), F32)
    lib().oracle_project_2d_backward(
        ctypes.c_int(n), _p(L), ctypes.c_int(img_h), ctypes.c_int(img_w), _p(radii), _p(conics),
        _p(v_xy), _p(v_conic), _p(v_cov2d), _p(v_mean2d), _p(v_L))
    return v_cov2d, v_mean2d, v_L


def cov2d_bounds(covs):
    covs = _c(covs, F32)
    n = covs.shape[0]
    conics = np.zeros((n, 3), F32)
    radii = np.zeros((n, 1), F32)
    lib().oracle_cov2d_bounds(ctypes.c_int(n), _p(covs), _p(conics), _p(radii))
    return conics, radii


def cumulative_intersects(num_tiles_hit):
    """utils.py:99-118: int32 inclusive cumsum and its last element."""
    cum = np.cumsum(np.asarray(num_tiles_hit, dtype=np.int64)).astype(I32)
    m = int(cum[-1]) if cum.size else 0
    return m, cum


def map_intersects(xys, depths, radii, cum, tb, m):
    xys = _c(xys, F32)
    depths = _c(depths, F32)
    radii = _c(radii, I32)
    cum = _c(cum, I32)
    n = xys.shape[0]
    isect = np.zeros((m,), I64)
    gids = np.zeros((m,), I32)
    lib().oracle_map_intersects(
        ctypes.c_int(n), _p(xys), _p(depths), _p(radii), _p(cum),
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]), _p(isect), _p(gids))
    return isect, gids


def sort_pairs(keys, vals):
    keys = _c(keys, I64)
    vals = _c(vals, I32)
    m = keys.shape[0]
    ko = np.zeros((m,), I64)
    vo = np.zeros((m,), I32)
    lib().oracle_sort_pairs(ctypes.c_int(m), _p(keys), _p(vals), _p(ko), _p(vo))
    return ko, vo


def tile_bin_edges(isect_sorted, rows):
    isect_sorted = _c(isect_sorted, I64)
    bins = np.zeros((rows, 2), I32)
    lib().oracle_tile_bin_edges(ctypes.c_int(isect_sorted.shape[0]), _p(isect_sorted), _p(bins),
                                ctypes.c_int(rows))
    return bins


def bin_and_sort(xys, depths, radii, cum, tb, m):
    """utils.py:121-167.  tile_bins gets max(M, num_tiles) rows."""
    isect, gids = map_intersects(xys, depths, radii, cum, tb, m)
    isect_sorted, gids_sorted = sort_pairs(isect, gids)
    rows = max(m, tb[0] * tb[1])
    bins = tile_bin_edges(isect_sorted, rows)
    return isect, gids, isect_sorted, gids_sorted, bins


def raster_sum_forward(tb, img_h, img_w, gids_sorted, bins, xys, conics, colors, opac):
    out = np.zeros((img_h, img_w, 3), F32)
    Ts = np.zeros((img_h, img_w), F32)
    idx = np.zeros((img_h, img_w), I32)
    args = [_c(gids_sorted, I32), _c(bins, I32), _c(xys, F32), _c(conics, F32),
            _c(colors, F32), _c(opac, F32)]
    lib().oracle_raster_sum_forward(
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]), ctypes.c_int(img_w), ctypes.c_int(img_h),
        *[_p(a) for a in args], _p(out), _p(Ts), _p(idx))
    return out, Ts, idx


def raster_sum_backward(tb, img_h, img_w, gids_sorted, bins, xys, conics, colors, opac,
                        final_idx, v_out):
    n = np.asarray(xys).shape[0]
    v_xy = np.zeros((n, 2), F64)
    v_conic = np.zeros((n, 3), F64)
    v_rgb = np.zeros((n, 3), F64)
    v_opac = np.zeros((n, 1), F64)
    args = [_c(gids_sorted, I32), _c(bins, I32), _c(xys, F32), _c(conics, F32),
            _c(colors, F32), _c(opac, F32), _c(final_idx, I32), _c(v_out, F32)]
    lib().oracle_raster_sum_backward(
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]), ctypes.c_int(img_w), ctypes.c_int(img_h),
        ctypes.c_int(n), *[_p(a) for a in args], _p(v_xy), _p(v_conic), _p(v_rgb), _p(v_opac))
    return v_xy, v_conic, v_rgb, v_opac


def raster_forward(tb, img_h, img_w, gids_sorted, bins, xys, conics, colors, opac, bg):
    out = np.zeros((img_h, img_w, 3), F32)
    Ts = np.zeros((img_h, img_w), F32)
    idx = np.zeros((img_h, img_w), I32)
    args = [_c(gids_sorted, I32), _c(bins, I32), _c(xys, F32), _c(conics, F32),
            _c(colors, F32), _c(opac, F32), _c(bg, F32)]
    lib().oracle_raster_forward(
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]), ctypes.c_int(img_w), ctypes.c_int(img_h),
        *[_p(a) for a in args], _p(out), _p(Ts), _p(idx))
    return out, Ts, idx


def raster_backward(tb, img_h, img_w, gids_sorted, bins, xys, conics, colors, opac, bg,
                    final_Ts, final_idx, v_out, v_out_alpha):
    n = np.asarray(xys).shape[0]
    v_xy = np.zeros((n, 2), F64)
    v_conic = np.zeros((n, 3), F64)
    v_rgb = np.zeros((n, 3), F64)
    v_opac = np.zeros((n, 1), F64)
    args = [_c(gids_sorted, I32), _c(bins, I32), _c(xys, F32), _c(conics, F32),
            _c(colors, F32), _c(opac, F32), _c(bg, F32), _c(final_Ts, F32), _c(final_idx, I32),
            _c(v_out, F32), _c(v_out_alpha, F32)]
    lib().oracle_raster_backward(
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]), ctypes.c_int(img_w), ctypes.c_int(img_h),
        ctypes.c_int(n), *[_p(a) for a in args], _p(v_xy), _p(v_conic), _p(v_rgb), _p(v_opac))
    return v_xy, v_conic, v_rgb, v_opac


def sum_min_margin(tb, img_h, img_w, gids_sorted, bins, xys, conics, opac):
    margin = np.full((img_h, img_w), np.inf, F32)
    args = [_c(gids_sorted, I32), _c(bins, I32), _c(xys, F32), _c(conics, F32), _c(opac, F32)]
    lib().oracle_sum_min_margin(
        ctypes.c_int(tb[0]), ctypes.c_int(tb[1]), ctypes.c_int(img_w), ctypes.c_int(img_h),
        *[_p(a) for a in args], _p(margin))
    return margin


def render_sum(means2d, L, colors, opac, img_h, img_w):
    """The whole sum-path forward of GaussianSplats_Represent.py:83-90 (minus
    clamp/permute): project -> cumsum -> bin/sort -> sum-rasterize."""
    tb = tile_bounds(img_h, img_w)
    xys, depths, radii, conics, nth = project_2d_forward(means2d, L, img_h, img_w, tb)
    m, cum = cumulative_intersects(nth)
    if m < 1:
        return dict(out=np.ones((img_h, img_w, 3), F32), m=0, xys=xys, radii=radii,
                    conics=conics, nth=nth)
    isect, gids, isect_sorted, gids_sorted, bins = bin_and_sort(xys, depths, radii, cum, tb, m)
    out, Ts, idx = raster_sum_forward(tb, img_h, img_w, gids_sorted, bins, xys, conics, colors, opac)
    return dict(out=out, final_Ts=Ts, final_idx=idx, m=m, cum=cum, xys=xys, depths=depths,
                radii=radii, conics=conics, nth=nth, isect=isect, gids=gids,
                isect_sorted=isect_sorted, gids_sorted=gids_sorted, bins=bins, tb=tb)


def synthetic_frame(n: int, seed: int, rgb_w: float = 1.0, chol_scale: float = 1.0):
    """Reference init distributions (GaussianSplats_Represent.py:28-38,57-70) on a
    seeded numpy RNG: means = tanh(atanh(2(u-.5))) = 2u-1, L = rand + [.5,0,.5],
    colors = rand * rgb_W, opacity = 1."""
    rng = np.random.default_rng(seed)
    u = rng.random((n, 2), dtype=np.float32)
    means = np.tanh(np.arctanh(2.0 * (u - 0.5))).astype(F32)
    chol = (rng.random((n, 3), dtype=np.float32) * chol_scale
            + np.array([0.5, 0.0, 0.5], F32) * chol_scale).astype(F32)
    colors = (rng.random((n, 3), dtype=np.float32) * np.float32(rgb_w)).astype(F32)
    opac = np.ones((n, 1), F32)
    return means, chol, colors, opac


def i420_to_rgb(yuv: np.ndarray, h: int, w: int) -> np.ndarray:
    """OpenCV's COLOR_YUV2RGB_I420 (fixed-point ITU-R BT.601, 20-bit, as in
    utils.py:153 ``cv2.cvtColor``) then ToTensor's / 255: [3, h, w] float32.
    Restated from OpenCV's published constants; cv2 itself is absent here, so
    this is parity-unpinned against it."""
    CY, CUB, CUG, CVG, CVR, SH = 1220542, 2116026, -409993, -852492, 1673527, 20
    yuv = np.asarray(yuv, np.uint8).reshape(-1)
    Y = yuv[: h * w].reshape(h, w).astype(np.int64)
    U = yuv[h * w: h * w + (h // 2) * (w // 2)].reshape(h // 2, w // 2).astype(np.int64) - 128
    V = yuv[h * w + (h // 2) * (w // 2):].reshape(h // 2, w // 2).astype(np.int64) - 128
    U = np.repeat(np.repeat(U, 2, 0), 2, 1)
    V = np.repeat(np.repeat(V, 2, 0), 2, 1)
    y = np.maximum(0, Y - 16) * CY
    half = 1 << (SH - 1)
    r = (y + half + CVR * V) >> SH
    g = (y + half + CVG * V + CUG * U) >> SH
    b = (y + half + CUB * U) >> SH
    rgb = np.clip(np.stack([r, g, b]), 0, 255).astype(np.float32)
    return (rgb / np.float32(255.0)).astype(np.float32)


# ---------------------------------------------------------------- SSIM / MS-SSIM
# pytorch_msssim's published algorithm (ssim, ms_ssim, _ssim, gaussian_filter,
# _fspecial_gauss_1d), the package GSVC calls at utils.py:29-40 and
# train_video_Represent.py:145.  It is unpinned (requirements.txt:5) and not
# installed here, so this float64 restatement is the checker: parity unpinned
# against the package itself.

def gauss_window(size: int, sigma: float) -> np.ndarray:
    """_fspecial_gauss_1d: exp(-(c^2) / (2 sigma^2)) at c = t - size//2, normalised."""
    c = np.arange(size, dtype=F64) - size // 2
    g = np.exp(-(c ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def _filter(x: np.ndarray, g: np.ndarray) -> np.ndarray:
    """gaussian_filter: valid correlation along H, then W; a dimension shorter
    than the window is left unfiltered.  x: [..., H, W]."""
    k = g.shape[0]
    out = x
    for axis in (-2, -1):
        if out.shape[axis] >= k:
            win = np.lib.stride_tricks.sliding_window_view(out, k, axis=axis)
            out = win @ g
    return out


def _ssim_terms(X, Y, g, C1, C2):
    mu1, mu2 = _filter(X, g), _filter(Y, g)
    s1 = _filter(X * X, g) - mu1 * mu1
    s2 = _filter(Y * Y, g) - mu2 * mu2
    s12 = _filter(X * Y, g) - mu1 * mu2
    cs_map = (2 * s12 + C2) / (s1 + s2 + C2)
    ssim_map = ((2 * mu1 * mu2 + C1) / (mu1 * mu1 + mu2 * mu2 + C1)) * cs_map
    return ssim_map.mean(axis=(-2, -1)), cs_map.mean(axis=(-2, -1))  # [B, C]


def ssim(X, Y, data_range=255.0, size_average=True, win_size=11, win_sigma=1.5,
         K=(0.01, 0.03), nonnegative_ssim=False):
    """X, Y: [B, C, H, W] -> scalar (size_average) or [B]."""
    X = np.asarray(X, F64)
    Y = np.asarray(Y, F64)
    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    s, _ = _ssim_terms(X, Y, gauss_window(win_size, win_sigma), C1, C2)
    if nonnegative_ssim:
        s = np.maximum(s, 0.0)
    return s.mean() if size_average else s.mean(axis=1)


def avg_pool2(x: np.ndarray) -> np.ndarray:
    """F.avg_pool2d(kernel 2, stride 2, padding (H % 2, W % 2)), pads counted."""
    H, W = x.shape[-2:]
    ph, pw = H % 2, W % 2
    xp = np.pad(x, [(0, 0)] * (x.ndim - 2) + [(ph, ph), (pw, pw)])
    Ho, Wo = (H + 2 * ph - 2) // 2 + 1, (W + 2 * pw - 2) // 2 + 1
    xp = xp[..., :2 * Ho, :2 * Wo]
    return (xp[..., 0::2, 0::2] + xp[..., 0::2, 1::2] + xp[..., 1::2, 0::2] +
            xp[..., 1::2, 1::2]) / 4.0


MS_SSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def ms_ssim(X, Y, data_range=255.0, size_average=True, win_size=11, win_sigma=1.5,
            weights=None, K=(0.01, 0.03)):
    X = np.asarray(X, F64)
    Y = np.asarray(Y, F64)
    w = np.asarray(MS_SSIM_WEIGHTS if weights is None else weights, F64)
    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    g = gauss_window(win_size, win_sigma)
    mcs = []
    for i in range(len(w)):
        s, cs = _ssim_terms(X, Y, g, C1, C2)
        if i < len(w) - 1:
            mcs.append(np.maximum(cs, 0.0))
            X, Y = avg_pool2(X), avg_pool2(Y)
    stack = np.stack(mcs + [np.maximum(s, 0.0)], axis=0)  # [levels, B, C]
    val = np.prod(stack ** w[:, None, None], axis=0)
    return val.mean() if size_average else val.mean(axis=1)


def prune_keep(rgb_w: np.ndarray, remove_count: int) -> np.ndarray:
    """GaussianSplats_Represent.py:101-125 / 149-166: keep mask after removing
    the ``remove_count`` smallest ``torch.norm(rgb_W, dim=1)`` -- float32
    sqrt(w*w) per row ([N, 1]), ordered as the GPU's stable torch.sort
    (ties by index, NaN last; numpy's stable argsort does the same)."""
    w = np.ascontiguousarray(rgb_w, dtype=F32).reshape(-1)
    norms = np.sqrt(w * w).astype(F32)
    order = np.argsort(norms, kind="stable")
    keep = np.ones(w.shape[0], dtype=bool)
    keep[order[:max(int(remove_count), 0)]] = False
    return keep



# ---------------------------------------------------------------- Adan + train_iter
# The checker for the fused training step and the CPU baseline of bench.py's
# headline (BASELINE configs[2]).  Adan: reference optimizer.py:296-362
# (``_multi_tensor_adan``) with the bias corrections of :171-173,211, restated
# per element in float32 numpy in the foreach op order (each foreach op rounds
# its result to fp32; Python-float scalars enter as fp32 for fp32 tensors).

def adan_scalars(step, lr=1e-3, betas=(0.98, 0.92, 0.99), eps=1e-8, weight_decay=0.0):
    b1, b2, b3 = betas
    return dict(b1=b1, b2=b2, b3=b3, bc1=1.0 - b1 ** step, bc2=1.0 - b2 ** step,
                bc3_sqrt=math.sqrt(1.0 - b3 ** step), lr=lr, wd=weight_decay, eps=eps)


def adan_step(p, grad, st, step, lr=1e-3, betas=(0.98, 0.92, 0.99), eps=1e-8, weight_decay=0.0,
              no_prox=False, clip=1.0):
    """One Adan update of parameter ``p`` (float32 array, updated in place) with
    gradient ``grad`` and state dict ``st`` (exp_avg, exp_avg_sq, exp_avg_diff,
    neg_pre_grad; created on the first call as the reference does at
    optimizer.py:181-189).  Returns ``p``."""
    f = np.float32
    S = adan_scalars(step, lr, betas, eps, weight_decay)
    g = (np.asarray(grad, F32) * f(clip)).astype(F32)
    if not st:
        st["exp_avg"] = np.zeros_like(p)
        st["exp_avg_sq"] = np.zeros_like(p)
        st["exp_avg_diff"] = np.zeros_like(p)
    if "neg_pre_grad" not in st or step == 1:
        st["neg_pre_grad"] = (g * f(-1.0)).astype(F32)
    m, v, df, npg = st["exp_avg"], st["exp_avg_sq"], st["exp_avg_diff"], st["neg_pre_grad"]
    npg += g                                                          # :313
    m *= f(S["b1"]); m += f(1 - S["b1"]) * g                          # :315-316
    df *= f(S["b2"]); df += f(1 - S["b2"]) * npg                      # :318-319
    npg *= f(S["b2"]); npg += g                                       # :321-322
    v *= f(S["b3"]); v += f(1 - S["b3"]) * (npg * npg)                # :323-324
    den = (np.sqrt(v) / f(S["bc3_sqrt"])).astype(F32) + f(S["eps"])   # :326-328
    step_size = f(S["lr"] / S["bc1"])
    step_diff = f(S["lr"] * S["b2"] / S["bc2"])
    if no_prox:
        p *= f(1 - S["lr"] * S["wd"])
        p += (-step_size) * (m / den)
        p += (-step_diff) * (df / den)
    else:
        p += (-step_size) * (m / den)
        p += (-step_diff) * (df / den)
        p /= f(1 + S["lr"] * S["wd"])
    npg[...] = -g                                                     # :361-362
    return p


def train_grads_sum(means, L, colors, gt, H, W):
    """The part of GaussianVideo_frame.train_iter (GaussianSplats_Represent.py:
    191-195) before Adan, from ACTIVATED inputs (means2d = tanh(_xyz), L,
    colors; opacity 1): the sum-path forward, clamp, F.mse_loss against ``gt``
    [3, H, W], its gradient through the clamp (torch clamp passes where 0 <=
    out <= 1), the rasterizer and projection VJPs.  Returns (loss, render
    [3, H, W] clamped, v_means2d [N,2], v_L [N,3], v_colors [N,3]) in float32
    (loss float64)."""
    n = means.shape[0]
    opac = np.ones((n, 1), F32)
    r = render_sum(means, L, colors, opac, H, W)
    out = r["out"]
    img = np.clip(out, 0.0, 1.0).transpose(2, 0, 1)
    gt = np.asarray(gt, F32).reshape(3, H, W)
    d = (img - gt).astype(F32)
    numel = 3 * H * W
    loss = float(np.mean(d.astype(F64) ** 2))
    if r["m"] < 1:
        z2, z3 = np.zeros((n, 2), F32), np.zeros((n, 3), F32)
        return loss, img, z2, z3, z3.copy()
    v_img = (np.float32(2.0 / numel) * d).astype(F32)
    v_img[(img < 0.0) | (img > 1.0)] = 0.0  # (never: img is clamped; kept for the rule)
    o_chw = out.transpose(2, 0, 1)
    v_img[(o_chw < 0.0) | (o_chw > 1.0)] = 0.0
    v_out = np.ascontiguousarray(v_img.transpose(1, 2, 0))
    tb = r["tb"]
    v_xy, v_conic, v_rgb, _ = raster_sum_backward(tb, H, W, r["gids_sorted"], r["bins"], r["xys"],
                                                  r["conics"], colors, opac, r["final_idx"], v_out)
    _, v_mean2d, v_L = project_2d_backward(L, H, W, r["radii"], r["conics"], v_xy.astype(F32),
                                           v_conic.astype(F32))
    return loss, img, v_mean2d, v_L.astype(F32), v_rgb.astype(F32)


def train_iter_sum(params, gt, H, W, state, step, lr=1e-3):
    """GaussianVideo_frame.train_iter (GaussianSplats_Represent.py:191-207) for
    the L2 loss, no prune / densify, on CPU: activations (:57-70),
    train_grads_sum, the activation VJPs and one Adan step of _xyz, _cholesky,
    _features_dc (rgb_W fixed at ones).  ``params``: dict of float32 arrays
    ``_xyz`` [N,2], ``_cholesky`` [N,3], ``_features_dc`` [N,3], updated in
    place; ``state``: dict of per-parameter Adan state dicts; ``step``: the
    optimizer's own step count (1 for a fresh Adan, as optimizer.py:171-173
    counts it -- not the training iteration).  Returns (loss, psnr)."""
    xyz, chol, feat = params["_xyz"], params["_cholesky"], params["_features_dc"]
    means = np.tanh(xyz).astype(F32)
    L = (chol + np.array([0.5, 0.0, 0.5], F32)).astype(F32)
    loss, _, v_mean2d, v_L, v_rgb = train_grads_sum(means, L, feat.astype(F32), gt, H, W)
    d_xyz = (v_mean2d * (1.0 - means * means)).astype(F32)
    grads = [d_xyz, v_L, v_rgb]
    for name, p, g in zip(("_xyz", "_cholesky", "_features_dc"), (xyz, chol, feat), grads):
        adan_step(p, g, state.setdefault(name, {}), step, lr=lr)
    return loss, 10.0 * math.log10(1.0 / loss)
