"""Native op table: the MI355X replacement of the reference's ``gsplat.cuda``.

Each function keeps the name, positional signature, dtypes and return tuple of
the op the reference bound in gsplat/gsplat/cuda/csrc/ext.cpp:6-23 (wrappers
in bindings.cu) and exposed lazily through gsplat/gsplat/cuda/__init__.py:14-30,
and calls the gfx950 C ABI (include/gsvc_amd.h) on the tensors' device and
current stream.  Outputs are fresh tensors from the PyTorch caching allocator,
as with the reference's ``torch::zeros`` (bindings.cu:808-817 etc.).

Differences from the reference, all documented in DESIGN.md §3:
  * ``rasterize_sum_forward`` returns ``final_Ts`` as an expanded constant 1
    view (the sum kernel never changes T, forward.cu:579,617);
  * the rasterizer backward ops return the four gradients as strided views of
    one [N, 16] record tensor (one 64-byte atomic record per splat);
  * ``get_tile_bin_edges`` returns max(M, last tile + 1) rows instead of M
    (the reference wrote past its M-row allocation when M < #tiles);
  * ``nd_rasterize_*`` (C != 3) are not provided: out of scope, and the
    reference did not export ``nd_rasterize_sum_*`` either (AttributeError).
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib as L

TILE = 16

# Optional live timing of the composite kernels (bench.py): when a list is
# installed here, each rasterizer launch is bracketed by HIP events recorded on
# the stream the kernel is launched on (torch's current stream).
_kernel_events = None


_timing_every = 1
_timing_calls = 0


def enable_kernel_timing(on: bool = True, every: int = 1):
    """Start (or stop) recording (name, start_event, end_event) around the
    rasterizer launches -- every ``every``-th call, so that the event records
    do not slow the loop being measured."""
    global _kernel_events, _timing_every, _timing_calls
    _kernel_events = [] if on else None
    _timing_every = max(1, int(every))
    _timing_calls = 0
    return _kernel_events


def composite_timing(on: bool, max_launches: int = 4096, every: int = 1, dispatch: bool = False):
    """C-side HIP-event timing of the sum-forward kernel launches (every
    entry point, including the fused frame render); see gsvc_timing_enable.
    ``dispatch``: the timed launch carries the events itself (the kernel's own
    start / end) instead of events recorded around it."""
    L.call("gsvc_timing_enable", int(max_launches) if on else 0, int(every), 1 if dispatch else 0)


def composite_times_ms(max_launches: int = 4096):
    import ctypes
    buf = (ctypes.c_float * max_launches)()
    cnt = ctypes.c_int(0)
    L.call("gsvc_timing_collect", ctypes.addressof(buf), max_launches, ctypes.addressof(cnt))
    return list(buf[: cnt.value])


TIMING_CHANNELS = {"composite": 0, "train_tile": 1, "project": 2, "train_splat": 3,
                   "sum_bwd": 4, "alpha_fwd": 5, "alpha_bwd": 6}


def channel_timing(channel: str, on: bool, max_launches: int = 4096, every: int = 1,
                   dispatch: bool = True):
    """HIP-event timing of one kernel's launches (gsvc_timing_enable_channel):
    ``channel`` is one of TIMING_CHANNELS; ``dispatch`` as composite_timing."""
    L.call("gsvc_timing_enable_channel", TIMING_CHANNELS[channel], int(max_launches) if on else 0,
           int(every), 1 if dispatch else 0)


def channel_times_ms(channel: str, max_launches: int = 4096):
    import ctypes
    buf = (ctypes.c_float * max_launches)()
    cnt = ctypes.c_int(0)
    L.call("gsvc_timing_collect_channel", TIMING_CHANNELS[channel], ctypes.addressof(buf),
           max_launches, ctypes.addressof(cnt))
    return list(buf[: cnt.value])


def kernel_times_ms(name: str):
    """Durations in ms of the recorded launches of ``name`` (synchronizes)."""
    if not _kernel_events:
        return []
    torch.cuda.synchronize()
    return [s.elapsed_time(e) for n, s, e in _kernel_events if n == name]


def _timed_call(sym, *args):
    global _timing_calls
    if _kernel_events is None:
        L.call(sym, *args)
        return
    _timing_calls += 1
    if (_timing_calls - 1) % _timing_every:
        L.call(sym, *args)
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    L.call(sym, *args)
    e.record()
    _kernel_events.append((sym, s, e))


def _dev(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} must be a CUDA tensor (gsvc_amd has no CPU path)")


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    _dev(t, name)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name}: expected scalar type Float but found {t.dtype}")
    return t.contiguous()


def _i32(t: torch.Tensor, name: str) -> torch.Tensor:
    _dev(t, name)
    if t.dtype != torch.int32:
        raise RuntimeError(f"{name}: expected scalar type Int but found {t.dtype}")
    return t.contiguous()


def _i64(t: torch.Tensor, name: str) -> torch.Tensor:
    _dev(t, name)
    if t.dtype != torch.int64:
        raise RuntimeError(f"{name}: expected scalar type Long but found {t.dtype}")
    return t.contiguous()


def _tb(tile_bounds) -> Tuple[int, int, int]:
    tb = tuple(int(x) for x in tile_bounds)
    if len(tb) != 3:
        raise ValueError("tile_bounds must be a (x, y, z) tuple")
    return tb


# ---------------------------------------------------------------------------
# 2D projection (bindings.cu:781-839, 902-949)

def project_gaussians_2d_forward(num_points, means2d, L_elements, img_height, img_width,
                                 tile_bounds, clip_thresh):
    means2d = _f32(means2d, "means2d")
    L_elements = _f32(L_elements, "L_elements")
    n = int(num_points)
    dev = means2d.device
    tb = _tb(tile_bounds)
    # separate tensors: carved views of one block made the autograd backward of
    # the two ops 144 us slower (view tracking of outputs that carry gradients)
    xys = torch.empty((n, 2), dtype=torch.float32, device=dev)
    depths = torch.empty((n,), dtype=torch.float32, device=dev)
    radii = torch.empty((n,), dtype=torch.int32, device=dev)
    conics = torch.empty((n, 3), dtype=torch.float32, device=dev)
    nth = torch.empty((n,), dtype=torch.int32, device=dev)
    L.call("gsvc_project_gaussians_2d_forward", n, L.ptr(means2d), L.ptr(L_elements),
           int(img_height), int(img_width), tb[0], tb[1], tb[2], float(clip_thresh),
           L.ptr(xys), L.ptr(depths), L.ptr(radii), L.ptr(conics), L.ptr(nth), L.stream(dev))
    # the 2D projection writes depth 0 for every splat (foward2d.cu:67,122):
    # tag it for utils.depths_known_zero (cleared by any in-place change)
    depths._gsvc_zero_version = depths._version
    return xys, depths, radii, conics, nth


def project_gaussians_2d_backward(num_points, means2d, L_elements, img_height, img_width, radii,
                                  conics, v_xy, v_depth, v_conic):
    L_elements = _f32(L_elements, "L_elements")
    radii = _i32(radii, "radii")
    conics = _f32(conics, "conics")
    v_xy = _f32(v_xy, "v_xy")
    v_conic = _f32(v_conic, "v_conic")
    n = int(num_points)
    dev = L_elements.device
    v_cov2d = torch.empty((n, 3), dtype=torch.float32, device=dev)
    v_mean2d = torch.empty((n, 2), dtype=torch.float32, device=dev)
    v_L = torch.empty((n, 3), dtype=torch.float32, device=dev)
    L.call("gsvc_project_gaussians_2d_backward", n, L.ptr(means2d), L.ptr(L_elements),
           int(img_height), int(img_width), L.ptr(radii), L.ptr(conics), L.ptr(v_xy), None,
           L.ptr(v_conic), L.ptr(v_cov2d), L.ptr(v_mean2d), L.ptr(v_L), L.stream(dev))
    return v_cov2d, v_mean2d, v_L


def compute_cov2d_bounds(num_pts, covs2d):
    covs2d = _f32(covs2d, "covs2d")
    n = int(num_pts)
    dev = covs2d.device
    conics = torch.empty((n, 3), dtype=torch.float32, device=dev)
    radii = torch.empty((n, 1), dtype=torch.float32, device=dev)
    L.call("gsvc_compute_cov2d_bounds", n, L.ptr(covs2d), L.ptr(conics), L.ptr(radii), L.stream(dev))
    return conics, radii


# ---------------------------------------------------------------------------
# Binning (bindings.cu:274-330 and the torch glue of utils.py:99-167)

def cumulative_intersects(num_tiles_hit, depths=None):
    """int32 inclusive cumsum (utils.py:116) and a device int32[4] meta record
    {M, OR of depth bits, AND of depth bits, #emitting splats}."""
    num_tiles_hit = _i32(num_tiles_hit, "num_tiles_hit")
    n = num_tiles_hit.numel()
    dev = num_tiles_hit.device
    if depths is not None:
        depths = _f32(depths, "depths")
    cum = torch.empty((n,), dtype=torch.int32, device=dev)
    meta = torch.empty((4,), dtype=torch.int32, device=dev)
    ws = torch.empty((L.size("gsvc_cumsum_workspace_bytes", n),), dtype=torch.uint8, device=dev)
    L.call("gsvc_compute_cumulative_intersects", n, L.ptr(num_tiles_hit), L.ptr(depths), L.ptr(cum),
           L.ptr(meta), L.ptr(ws), ws.numel(), L.stream(dev))
    return cum, meta


def map_gaussian_to_intersects(num_points, num_intersects, xys, depths, radii, cum_tiles_hit,
                               tile_bounds):
    xys = _f32(xys, "xys")
    depths = _f32(depths, "depths")
    radii = _i32(radii, "radii")
    cum_tiles_hit = _i32(cum_tiles_hit, "cum_tiles_hit")
    tb = _tb(tile_bounds)
    m = int(num_intersects)
    dev = xys.device
    isect = torch.empty((m,), dtype=torch.int64, device=dev)
    gids = torch.empty((m,), dtype=torch.int32, device=dev)
    L.call("gsvc_map_gaussian_to_intersects", int(num_points), m, L.ptr(xys), L.ptr(depths),
           L.ptr(radii), L.ptr(cum_tiles_hit), tb[0], tb[1], tb[2], L.ptr(isect), L.ptr(gids),
           L.stream(dev))
    return isect, gids


def sort_isect_pairs(isect_ids, gaussian_ids, begin_bit=0, end_bit=64):
    """torch.sort(isect_ids) + torch.gather(gaussian_ids) (utils.py:164-165) as
    one stable radix sort; ties keep input order."""
    isect_ids = _i64(isect_ids, "isect_ids")
    gaussian_ids = _i32(gaussian_ids, "gaussian_ids")
    m = isect_ids.numel()
    dev = isect_ids.device
    ko = torch.empty_like(isect_ids)
    vo = torch.empty_like(gaussian_ids)
    ws = torch.empty((L.size("gsvc_sort_pairs_workspace_bytes", m),), dtype=torch.uint8, device=dev)
    L.call("gsvc_sort_isect_pairs", m, L.ptr(isect_ids), L.ptr(gaussian_ids), L.ptr(ko), L.ptr(vo),
           int(begin_bit), int(end_bit), L.ptr(ws), ws.numel(), L.stream(dev))
    return ko, vo


def get_tile_bin_edges(num_intersects, isect_ids_sorted, num_rows=None):
    isect_ids_sorted = _i64(isect_ids_sorted, "isect_ids_sorted")
    m = int(num_intersects)
    dev = isect_ids_sorted.device
    if num_rows is None:
        last_tile = int(isect_ids_sorted[m - 1].item() >> 32) if m > 0 else -1
        num_rows = max(m, last_tile + 1)
    bins = torch.empty((int(num_rows), 2), dtype=torch.int32, device=dev)
    L.call("gsvc_get_tile_bin_edges", m, L.ptr(isect_ids_sorted), L.ptr(bins), int(num_rows),
           L.stream(dev))
    return bins


def bin_and_sort_tiles(num_points, num_intersects, xys, depths, radii, cum_tiles_hit, tile_bounds,
                       want_isect_ids=False):
    """Fused hot-path binning (valid when all emitting splats share their depth
    bits): returns (gaussian_ids_sorted, tile_bins[#tiles, 2], isect_ids_sorted|None)."""
    xys = _f32(xys, "xys")
    radii = _i32(radii, "radii")
    cum_tiles_hit = _i32(cum_tiles_hit, "cum_tiles_hit")
    depths = _f32(depths, "depths") if depths is not None else None
    tb = _tb(tile_bounds)
    n, m = int(num_points), int(num_intersects)
    ntiles = tb[0] * tb[1]
    dev = xys.device
    gids = torch.empty((m,), dtype=torch.int32, device=dev)
    bins = torch.empty((ntiles, 2), dtype=torch.int32, device=dev)
    isect = torch.empty((m,), dtype=torch.int64, device=dev) if want_isect_ids else None
    ws = torch.empty((L.size("gsvc_bin_tiles_workspace_bytes", n, m, ntiles),), dtype=torch.uint8,
                     device=dev)
    L.call("gsvc_bin_and_sort_tiles", n, m, L.ptr(xys), L.ptr(depths), L.ptr(radii),
           L.ptr(cum_tiles_hit), tb[0], tb[1], L.ptr(gids), L.ptr(bins), ntiles, L.ptr(isect),
           L.ptr(ws), ws.numel(), L.stream(dev))
    return gids, bins, isect


def bin_tiles_counted(num_points, xys, radii, tile_bounds, capacity, tile_cap=0):
    """Sync-free tile binning (gsvc_bin_tiles_counted): returns
    (gaussian_ids_sorted [capacity], tile_bins [#tiles, 2], meta [2] = {M,
    overflow}) with M only on the device.  Valid when every emitting splat has
    the same depth bits (the order is (tile, splat id)).  tile_cap = 256 keeps
    each tile's first 256 entries only (the rasterizers read no more,
    forward.cu:569-571,613); 0 keeps all.  Other caps raise ValueError."""
    if int(tile_cap) not in (0, 256):
        raise ValueError(f"bin_tiles_counted: tile_cap must be 0 or 256, got {tile_cap}")
    xys = _f32(xys, "xys")
    radii = _i32(radii, "radii")
    tb = _tb(tile_bounds)
    n, cap = int(num_points), int(capacity)
    ntiles = tb[0] * tb[1]
    dev = xys.device
    scratch = torch.empty((cap,), dtype=torch.int32, device=dev)
    gids = torch.empty((cap,), dtype=torch.int32, device=dev)
    bins = torch.empty((ntiles, 2), dtype=torch.int32, device=dev)
    meta = torch.empty((2,), dtype=torch.int32, device=dev)
    ws = torch.empty((L.size("gsvc_bin_tiles_counted_workspace_bytes", ntiles) // 4 + 1,),
                     dtype=torch.int32, device=dev)
    L.call("gsvc_bin_tiles_counted", n, L.ptr(xys), L.ptr(radii), tb[0], tb[1], cap, int(tile_cap),
           L.ptr(scratch), L.ptr(gids), L.ptr(bins), L.ptr(meta), L.ptr(ws), 4 * ws.numel(),
           L.stream(dev))
    return gids, bins, meta


# ---------------------------------------------------------------------------
# Rasterizers (bindings.cu:332-469, 631-779)

def _bins_for(tile_bins: torch.Tensor, ntiles: int) -> torch.Tensor:
    tile_bins = _i32(tile_bins, "tile_bins")
    if tile_bins.dim() != 2 or tile_bins.shape[1] != 2:
        raise RuntimeError("tile_bins must have shape (rows, 2)")
    if tile_bins.shape[0] < ntiles:  # reference-style M-row table: pad with empty tiles
        pad = torch.zeros((ntiles - tile_bins.shape[0], 2), dtype=torch.int32, device=tile_bins.device)
        tile_bins = torch.cat([tile_bins, pad])
    return tile_bins


def _raster_inputs(tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys, conics,
                   colors, opacities, background):
    tb = _tb(tile_bounds)
    blk = _tb(block)
    img_w, img_h, img_d = (int(x) for x in img_size)
    gids = _i32(gaussian_ids_sorted, "gaussian_ids_sorted")
    xys = _f32(xys, "xys")
    conics = _f32(conics, "conics")
    colors = _f32(colors, "colors")
    opacities = _f32(opacities, "opacities")
    background = _f32(background, "background")
    if colors.dim() != 2 or colors.shape[1] != 3:
        raise RuntimeError("colors must have shape (N, 3)")
    bins = _bins_for(tile_bins, tb[0] * tb[1])
    return tb, blk, (img_w, img_h, img_d), gids, bins, xys, conics, colors, opacities, background


def _raster_fwd(sym, tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys, conics,
                colors, opacities, background, want_Ts):
    tb, blk, (img_w, img_h, img_d), gids, bins, xys, conics, colors, opacities, background = \
        _raster_inputs(tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys, conics,
                       colors, opacities, background)
    dev = xys.device
    out = torch.empty((img_h, img_w, 3), dtype=torch.float32, device=dev)
    idx = torch.empty((img_h, img_w), dtype=torch.int32, device=dev)
    Ts = torch.empty((img_h, img_w), dtype=torch.float32, device=dev) if want_Ts else None
    _timed_call(sym, tb[0], tb[1], tb[2], blk[0], blk[1], blk[2], img_w, img_h, img_d,
                L.ptr(gids), L.ptr(bins), L.ptr(xys), L.ptr(conics), L.ptr(colors),
                L.ptr(opacities), L.ptr(background), L.ptr(out), L.ptr(Ts), L.ptr(idx),
                L.stream(dev))
    return out, Ts, idx


def rasterize_sum_forward(tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys,
                          conics, colors, opacities, background):
    out, _, idx = _raster_fwd("gsvc_rasterize_sum_forward", tile_bounds, block, img_size,
                              gaussian_ids_sorted, tile_bins, xys, conics, colors, opacities,
                              background, want_Ts=False)
    final_Ts = torch.ones((1, 1), dtype=torch.float32, device=out.device).expand(out.shape[0],
                                                                              out.shape[1])
    return out, final_Ts, idx


LAYOUT_HWC = 0
LAYOUT_CHW_CLAMPED = 1
LAYOUT_CHW = 2  # channel planes, unclamped (the op path's GSVC_SLABS_PLANES image)


def rasterize_sum_forward_ex(tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys,
                             conics, colors, opacities, background, num_intersects_dev=None,
                             density_hint=0, layout=LAYOUT_HWC, want_idx=True, out=None):
    """Sum forward with the hot path's knobs (gsvc_rasterize_sum_forward_ex):
    a device-side M (background when 0), a density hint for the kernel choice,
    the fused clamp + [3,H,W] layout, and final_idx optional.  Returns
    (out_img, final_idx | None); out_img is [H,W,3] or [3,H,W] (``out`` may
    supply it)."""
    tb, blk, (img_w, img_h, img_d), gids, bins, xys, conics, colors, opacities, background = \
        _raster_inputs(tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys, conics,
                       colors, opacities, background)
    dev = xys.device
    shape = (img_h, img_w, 3) if layout == LAYOUT_HWC else (3, img_h, img_w)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=dev)
    elif out.numel() != img_h * img_w * 3 or not out.is_contiguous() or out.dtype != torch.float32:
        raise RuntimeError("out must be a contiguous float32 tensor of H*W*3 elements")
    idx = torch.empty((img_h, img_w), dtype=torch.int32, device=dev) if want_idx else None
    m_dev = None
    if num_intersects_dev is not None:
        m_dev = _i32(num_intersects_dev, "num_intersects_dev")
    _timed_call("gsvc_rasterize_sum_forward_ex", tb[0], tb[1], tb[2], blk[0], blk[1], blk[2], img_w,
                img_h, img_d, L.ptr(gids), L.ptr(bins), L.ptr(xys), L.ptr(conics), L.ptr(colors),
                L.ptr(opacities), L.ptr(background), L.ptr(m_dev), int(density_hint), int(layout),
                L.ptr(out), None, L.ptr(idx), L.stream(dev))
    return out, idx


def rasterize_forward(tile_bounds, block, img_size, gaussian_ids_sorted, tile_bins, xys, conics,
                      colors, opacities, background):
    return _raster_fwd("gsvc_rasterize_forward", tile_bounds, block, img_size, gaussian_ids_sorted,
                       tile_bins, xys, conics, colors, opacities, background, want_Ts=True)


def split_grad_records(rec: torch.Tensor):
    """(v_xy [N,2], v_conic [N,3], v_colors [N,3], v_opacity [N,1]) views."""
    return rec[:, 0:2], rec[:, 2:5], rec[:, 5:8], rec[:, 8:9]


def _raster_bwd(sym, img_height, img_width, BLOCK_H, BLOCK_W, gaussian_ids_sorted, tile_bins, xys,
                conics, colors, opacities, background, final_Ts, final_idx, v_output,
                v_output_alpha):
    xys = _f32(xys, "xys")
    colors = _f32(colors, "colors")
    if xys.dim() != 2 or xys.shape[1] != 2:
        raise RuntimeError("xys must have dimensions (num_points, 2)")
    if colors.dim() != 2 or colors.shape[1] != 3:
        raise RuntimeError("colors must have 2 dimensions")
    h, w = int(img_height), int(img_width)
    tb = ((w + int(BLOCK_W) - 1) // int(BLOCK_W), (h + int(BLOCK_H) - 1) // int(BLOCK_H))
    gids = _i32(gaussian_ids_sorted, "gaussian_ids_sorted")
    bins = _bins_for(tile_bins, tb[0] * tb[1])
    conics = _f32(conics, "conics")
    opacities = _f32(opacities, "opacities")
    background = _f32(background, "background")
    final_idx = _i32(final_idx, "final_idx")
    v_output = _f32(v_output, "v_output")
    Ts = _f32(final_Ts, "final_Ts") if sym == "gsvc_rasterize_backward" else None
    v_alpha = (_f32(v_output_alpha, "v_output_alpha")
               if sym == "gsvc_rasterize_backward" else None)
    n = xys.shape[0]
    rec = torch.empty((n, 16), dtype=torch.float32, device=xys.device)
    _timed_call(sym, h, w, int(BLOCK_H), int(BLOCK_W), n, L.ptr(gids), L.ptr(bins), L.ptr(xys),
           L.ptr(conics), L.ptr(colors), L.ptr(opacities), L.ptr(background), L.ptr(Ts),
           L.ptr(final_idx), L.ptr(v_output), L.ptr(v_alpha), L.ptr(rec), L.stream(xys.device))
    return split_grad_records(rec)


def rasterize_sum_backward(img_height, img_width, BLOCK_H, BLOCK_W, gaussian_ids_sorted, tile_bins,
                           xys, conics, colors, opacities, background, final_Ts, final_idx,
                           v_output, v_output_alpha, radii=None):
    """bindings.cu:706-779.  Under torch.use_deterministic_algorithms(True)
    and with the splats' ``radii`` (the autograd Function passes them), the
    bitwise reproducible variant (gsvc_rasterize_sum_backward_det)."""
    if radii is not None and torch.are_deterministic_algorithms_enabled():
        return _raster_sum_bwd_det(img_height, img_width, BLOCK_H, BLOCK_W, gaussian_ids_sorted,
                                   tile_bins, xys, conics, colors, opacities, radii, final_idx,
                                   v_output)
    return _raster_bwd("gsvc_rasterize_sum_backward", img_height, img_width, BLOCK_H, BLOCK_W,
                       gaussian_ids_sorted, tile_bins, xys, conics, colors, opacities, background,
                       final_Ts, final_idx, v_output, v_output_alpha)


DET_PAIRS_PER_SPLAT = 16  # the deterministic backward's first slot capacity per splat
# (device index, stream) -> [workspace, capacity, pair count of the last call (device int)]
_det_ws = {}


def _raster_sum_bwd_det(img_height, img_width, BLOCK_H, BLOCK_W, gaussian_ids_sorted, tile_bins,
                        xys, conics, colors, opacities, radii, final_idx, v_output):
    """The bitwise reproducible backward: one slot per (splat, tile) pair,
    summed in a fixed order.  If the pairs outnumber the slots (the excess
    would fall back to float atomics) the call is repeated with room for all
    of them, so the result is always the reproducible one; the capacity is
    kept for later calls (keyed by device and stream)."""
    xys = _f32(xys, "xys")
    colors = _f32(colors, "colors")
    if xys.dim() != 2 or xys.shape[1] != 2:
        raise RuntimeError("xys must have dimensions (num_points, 2)")
    if colors.dim() != 2 or colors.shape[1] != 3:
        raise RuntimeError("colors must have 2 dimensions")
    h, w = int(img_height), int(img_width)
    tb = ((w + int(BLOCK_W) - 1) // int(BLOCK_W), (h + int(BLOCK_H) - 1) // int(BLOCK_H))
    gids = _i32(gaussian_ids_sorted, "gaussian_ids_sorted")
    bins = _bins_for(tile_bins, tb[0] * tb[1])
    conics = _f32(conics, "conics")
    opacities = _f32(opacities, "opacities")
    radii = _i32(radii, "radii")
    final_idx = _i32(final_idx, "final_idx")
    v_output = _f32(v_output, "v_output")
    n = xys.shape[0]
    dev = xys.device
    key = (dev.index, L._raw_stream(dev.index))
    st = _det_ws.get(key)
    cap = max(DET_PAIRS_PER_SPLAT * n, st[1] if st is not None else 0)
    rec = torch.empty((n, 16), dtype=torch.float32, device=dev)
    for _ in range(2):
        need = L.size("gsvc_rasterize_sum_backward_det_workspace_bytes", n, cap)
        if st is None or st[0].numel() < need or st[1] != cap:
            st = _det_ws[key] = [torch.empty((need,), dtype=torch.uint8, device=dev), cap,
                                 torch.zeros((1,), dtype=torch.int32, device=dev)]
        _timed_call("gsvc_rasterize_sum_backward_det", h, w, int(BLOCK_H), int(BLOCK_W), n,
                    L.ptr(gids), L.ptr(bins), L.ptr(xys), L.ptr(conics), L.ptr(colors),
                    L.ptr(opacities), L.ptr(radii), L.ptr(final_idx), L.ptr(v_output), L.ptr(rec),
                    L.ptr(st[0]), st[0].numel(), cap, L.ptr(st[2]), L.stream(dev))
        pairs = int(st[2].item())
        if pairs <= cap:
            break
        cap = pairs + pairs // 2  # short: every slot again, with room to spare
    return split_grad_records(rec)


def rasterize_backward(img_height, img_width, BLOCK_H, BLOCK_W, gaussian_ids_sorted, tile_bins,
                       xys, conics, colors, opacities, background, final_Ts, final_idx, v_output,
                       v_output_alpha):
    return _raster_bwd("gsvc_rasterize_backward", img_height, img_width, BLOCK_H, BLOCK_W,
                       gaussian_ids_sorted, tile_bins, xys, conics, colors, opacities, background,
                       final_Ts, final_idx, v_output, v_output_alpha)


__all__ = [
    "project_gaussians_2d_forward", "project_gaussians_2d_backward", "compute_cov2d_bounds",
    "map_gaussian_to_intersects", "get_tile_bin_edges", "rasterize_sum_forward",
    "rasterize_sum_backward", "rasterize_forward", "rasterize_backward",
]


# ---------------------------------------------------------------------------
# Fused Adan (optimizer.py:296-362)

def adan_step(params, grads, exp_avgs, exp_avg_sqs, exp_avg_diffs, neg_pre_grads, *, beta1,
              beta2, beta3, bias_correction1, bias_correction2, bias_correction3_sqrt, lr,
              weight_decay, eps, no_prox, clip_global_grad_norm):
    """One fused Adan update of every tensor (gsvc_adan_step); same keyword
    arguments as _multi_tensor_adan.  Tensors must be contiguous fp32 CUDA."""
    import ctypes
    lists = (params, grads, exp_avgs, exp_avg_sqs, exp_avg_diffs, neg_pre_grads)
    n = len(params)
    if n == 0:
        return
    if any(len(x) != n for x in lists):
        raise RuntimeError("adan_step: tensor lists differ in length")
    for group in lists:
        for t in group:
            if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError("adan_step: tensors must be contiguous float32 CUDA tensors")
    for i in range(n):
        if any(x[i].numel() != params[i].numel() for x in lists):
            raise RuntimeError("adan_step: tensor sizes differ")
    P = ctypes.c_void_p * n
    arrs = [P(*[t.data_ptr() for t in group]) for group in lists]
    numels = (ctypes.c_longlong * n)(*[t.numel() for t in params])
    clip = float(clip_global_grad_norm)
    L.call("gsvc_adan_step", n, numels, *arrs, float(beta1), float(beta2), float(beta3),
           float(bias_correction1), float(bias_correction2), float(bias_correction3_sqrt),
           float(lr), float(weight_decay), float(eps), 1 if no_prox else 0, clip,
           L.stream(params[0].device))
