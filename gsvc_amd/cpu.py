"""CPU dispatch of the two drop-in operators (BASELINE configs[0]).

``project_gaussians_2d`` and ``rasterize_gaussians_sum`` called with CPU
tensors run here: autograd Functions over ``libgsvc_amd_cpu.so``
(csrc/cpu_ops.cpp, host C++ with OpenMP, the gfx950 kernels' op sequence).
HIP tensors never come here -- the operators dispatch on the inputs' device,
as torch's own ops do, and a GPU call that cannot run raises instead of
falling back.  Semantics are the GPU Functions' (project_gaussians_2d.py:
59-141, rasterize_sum.py:89-254): the M < 1 background branch, each tile's
first 256 entries in (tile, splat id) order, final_idx, gradients for xys,
conics, colours and opacity, the projection VJP with the reference's doubled
cross term.  Only depth-0 inputs (project_gaussians_2d's output) are binned
here; others raise, as the sorted path is GPU-only.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch
from torch.autograd import Function

_HERE = os.path.dirname(os.path.abspath(__file__))
CPU_LIB_PATH = os.path.join(_HERE, "lib", "libgsvc_amd_cpu.so")
TILE_KEEP = 256

_P, _I, _U = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint
_SIGS = {
    "gsvc_cpu_abi_version": ([], _I),
    "gsvc_cpu_set_threads": ([_I], _I),
    "gsvc_cpu_project_gaussians_2d_forward": ([_I, _P, _P, _U, _U, _I, _I, _P, _P, _P, _P, _P],
                                              ctypes.c_longlong),
    "gsvc_cpu_project_gaussians_2d_backward": ([_I, _P, _U, _U, _P, _P, _P, _P, _P, _P, _P], None),
    "gsvc_cpu_bin_tiles": ([_I, _P, _P, _I, _I, _P, _P], ctypes.c_longlong),
    "gsvc_cpu_rasterize_sum_forward": ([_I, _I, _U, _U, _P, _P, _P, _P, _P, _P, _P, _P], None),
    "gsvc_cpu_rasterize_sum_backward": ([_U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P], None),
}
_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(CPU_LIB_PATH):
                    raise RuntimeError(f"gsvc_amd: {CPU_LIB_PATH} not found; build it with "
                                       "`python -m gsvc_amd.build`")
                h = ctypes.CDLL(CPU_LIB_PATH)
                for name, (args, res) in _SIGS.items():
                    fn = getattr(h, name)
                    fn.argtypes = args
                    fn.restype = res
                _lib = h
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the CPU dispatch (results do not depend on it)."""
    return int(lib().gsvc_cpu_set_threads(int(n)))


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _cpu(t, name, dtype=torch.float32):
    if t.device.type != "cpu":
        raise RuntimeError(f"{name}: all inputs of a CPU call must be CPU tensors")
    if t.dtype != dtype:
        raise RuntimeError(f"{name}: expected scalar type {dtype} but found {t.dtype}")
    return t.contiguous()


class ProjectGaussians2dCPU(Function):
    @staticmethod
    def forward(ctx, means2d, L_elements, img_height, img_width, tile_bounds, clip_thresh=0.01):
        means2d = _cpu(means2d, "means2d")
        L_elements = _cpu(L_elements, "L_elements")
        n = means2d.shape[-2]
        xys = torch.empty((n, 2))
        depths = torch.empty((n,))
        radii = torch.empty((n,), dtype=torch.int32)
        conics = torch.empty((n, 3))
        nth = torch.empty((n,), dtype=torch.int32)
        lib().gsvc_cpu_project_gaussians_2d_forward(
            n, _p(means2d), _p(L_elements), int(img_height), int(img_width), int(tile_bounds[0]),
            int(tile_bounds[1]), _p(xys), _p(depths), _p(radii), _p(conics), _p(nth))
        ctx.img_height, ctx.img_width = int(img_height), int(img_width)
        ctx.save_for_backward(L_elements, radii, conics)
        ctx.mark_non_differentiable(radii, nth)
        ctx.set_materialize_grads(False)  # depths' gradient: None, not zeros
        return xys, depths, radii, conics, nth

    @staticmethod
    def backward(ctx, v_xys, v_depths, v_radii, v_conics, v_nth):
        L_elements, radii, conics = ctx.saved_tensors
        n = L_elements.shape[0]
        v_xys = torch.zeros((n, 2)) if v_xys is None else _cpu(v_xys, "v_xy")
        v_conics = torch.zeros((n, 3)) if v_conics is None else _cpu(v_conics, "v_conic")
        v_cov2d, v_mean2d, v_L = torch.empty((n, 3)), torch.empty((n, 2)), torch.empty((n, 3))
        lib().gsvc_cpu_project_gaussians_2d_backward(
            n, _p(L_elements), ctx.img_height, ctx.img_width, _p(radii), _p(conics), _p(v_xys),
            _p(v_conics), _p(v_cov2d), _p(v_mean2d), _p(v_L))
        return v_mean2d, v_L, None, None, None, None


class RasterizeGaussiansSumCPU(Function):
    @staticmethod
    def forward(ctx, xys, radii, conics, colors, opacity, background, img_height, img_width):
        xys = _cpu(xys, "xys")
        radii = _cpu(radii, "radii", torch.int32)
        conics = _cpu(conics, "conics")
        colors = _cpu(colors, "colors")
        opacity = _cpu(opacity, "opacity")
        background = _cpu(background, "background")
        H, W = int(img_height), int(img_width)
        n = xys.shape[0]
        tbx, tby = (W + 15) // 16, (H + 15) // 16
        ids = torch.empty((tbx * tby * TILE_KEEP,), dtype=torch.int32)
        bins = torch.empty((tbx * tby, 2), dtype=torch.int32)
        m = lib().gsvc_cpu_bin_tiles(n, _p(xys), _p(radii), tbx, tby, _p(ids), _p(bins))
        ctx.img_height, ctx.img_width, ctx.m = H, W, int(m)
        if m < 1:  # rasterize_sum.py:121-127
            out = torch.ones(H, W, 3) * background
            ctx.save_for_backward(xys, conics, colors, opacity)
            return out
        out = torch.empty((H, W, 3))
        idx = torch.empty((H, W), dtype=torch.int32)
        lib().gsvc_cpu_rasterize_sum_forward(tbx, tby, W, H, _p(ids), _p(bins), _p(xys), _p(conics),
                                             _p(colors), _p(opacity), _p(out), _p(idx))
        ctx.save_for_backward(xys, conics, colors, opacity, ids, bins, idx)
        return out

    @staticmethod
    def backward(ctx, v_out):
        saved = ctx.saved_tensors
        xys, conics, colors, opacity = saved[:4]
        if ctx.m < 1:
            return (torch.zeros_like(xys), None, torch.zeros_like(conics), torch.zeros_like(colors),
                    torch.zeros_like(opacity), None, None, None)
        ids, bins, idx = saved[4:]
        v_out = _cpu(v_out, "v_output")
        n = xys.shape[0]
        rec = torch.empty((n, 16))
        lib().gsvc_cpu_rasterize_sum_backward(ctx.img_height, ctx.img_width, n, _p(ids), _p(bins),
                                              _p(xys), _p(conics), _p(colors), _p(opacity), _p(idx),
                                              _p(v_out), _p(rec))
        v_opac = rec[:, 8:9]
        if opacity.dim() != 2:
            v_opac = v_opac.reshape(opacity.shape)
        return rec[:, 0:2], None, rec[:, 2:5], rec[:, 5:8], v_opac, None, None, None


def project_gaussians_2d(means2d, L_elements, img_height, img_width, tile_bounds, clip_thresh=0.01):
    xys, depths, radii, conics, nth = ProjectGaussians2dCPU.apply(
        means2d, L_elements, img_height, img_width, tile_bounds, clip_thresh)
    depths._gsvc_zero_version = depths._version
    return xys, depths, radii, conics, nth


def rasterize_gaussians_sum(xys, depths, radii, conics, num_tiles_hit, colors, opacity, img_height,
                            img_width, background, return_alpha):
    from .utils import depths_known_zero
    if not depths_known_zero(depths) and bool((depths != depths.flatten()[:1]).any()):
        raise RuntimeError("rasterize_gaussians_sum on CPU tensors bins depth-0 splats only "
                           "(project_gaussians_2d's output); the sorted path is GPU-only")
    out = RasterizeGaussiansSumCPU.apply(xys, radii, conics, colors, opacity, background,
                                         img_height, img_width)
    if return_alpha:
        m = int((num_tiles_hit.to(torch.int64)).sum())
        return out, torch.full((int(img_height), int(img_width)), 0.0 if m > 0 else 1.0)
    return out
