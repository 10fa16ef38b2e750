"""ctypes binding of the C ABI in include/gsvc_amd.h (libgsvc_amd.so).

This is the MI355X counterpart of the reference's backend loader
(gsplat/gsplat/cuda/_backend.py:54-98), which imported the compiled torch
extension or JIT-compiled it with nvcc and otherwise set ``_C = None``.  Here
the library is prebuilt in-tree for gfx950 (gsvc_amd/build.py).  There is no
CPU fallback: if the library is missing, or a tensor is not on a HIP device,
the call raises.

Two builds of the same sources exist: the product library (libgsvc_amd.so,
include/gsvc_amd.h) and the diagnostic one (libgsvc_amd_diag.so, -DGSVC_DIAG:
the A/B knobs and timestamped / ablation kernel variants of
include/gsvc_amd_diag.h).  ``load()`` returns the product library unless the
process runs with GSVC_DIAG=1 (tools/) or inside ``with diagnostic():`` (the
variant-comparison tests), which switches every op of this package to the
diagnostic library for its duration.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

import torch  # noqa: F401  (loads torch's libamdhip64 first; the library reuses it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libgsvc_amd.so")
# GSVC_DIAG_LIB: another build of the diagnostic library (tools' A/B of two builds)
DIAG_LIB_PATH = os.environ.get("GSVC_DIAG_LIB") or os.path.join(_HERE, "lib", "libgsvc_amd_diag.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_U = ctypes.c_uint
_F = ctypes.c_float
_SZ = ctypes.c_size_t
_LL = ctypes.c_longlong

# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS = {
    "gsvc_abi_version": [],
    "gsvc_last_error": [],
    "gsvc_alpha_cut_bits": [],
    "gsvc_alpha_cut_scan": [_P, _P],
    "gsvc_stream_sync": [_P],
    "gsvc_host_alloc": [_SZ],
    "gsvc_host_free": [_P],
    "gsvc_wait_host_seq": [_P, _U, _P, _I],
    "gsvc_timing_enable": [_I, _I, _I],
    "gsvc_timing_collect": [_P, _I, _P],
    "gsvc_timing_enable_channel": [_I, _I, _I, _I],
    "gsvc_timing_collect_channel": [_I, _P, _I, _P],
    "gsvc_prune_workspace_bytes": [_I],
    "gsvc_prune_lowest": [_I, _I, _P, _I, _P, _P, _P, _P, _SZ, _P],
    "gsvc_project_gaussians_2d_forward": [_I, _P, _P, _U, _U, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P],
    "gsvc_project_gaussians_2d_backward": [_I, _P, _P, _U, _U, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "gsvc_project_gaussians_2d_backward_strided": [_I, _P, _U, _U, _P, _P, _P, _I, _P, _I, _P, _P,
                                                   _P, _P],
    "gsvc_rasterize_sum_slabs_workspace_bytes": [_I],
    "gsvc_rasterize_sum_forward_slabs": [_I, _P, _P, _P, _P, _P, _P, _U, _U, _I, _I, _P, _SZ, _P,
                                         _P, _P, _P, _P, _P, _P],
    "gsvc_rasterize_sum_order_workspace_bytes": [_I],
    "gsvc_rasterize_sum_forward_slabs_ordered": [_I, _P, _P, _P, _P, _P, _P, _U, _U, _I, _I, _P, _SZ,
                                                 _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _I],
    "gsvc_rasterize_sum_backward_zeroed": [_U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "gsvc_rasterize_sum_backward_zeroed_strided": [_U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P, _LL,
                                                   _LL, _LL, _P, _P],
    "gsvc_rasterize_sum_backward_zeroed_strided_ex": [_U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                                      _LL, _LL, _LL, _P, _P, _I],
    "gsvc_compute_cov2d_bounds": [_I, _P, _P, _P, _P],
    "gsvc_cumsum_workspace_bytes": [_I],
    "gsvc_compute_cumulative_intersects": [_I, _P, _P, _P, _P, _P, _SZ, _P],
    "gsvc_map_gaussian_to_intersects": [_I, _I, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P],
    "gsvc_sort_pairs_workspace_bytes": [_I],
    "gsvc_sort_isect_pairs": [_I, _P, _P, _P, _P, _I, _I, _P, _SZ, _P],
    "gsvc_get_tile_bin_edges": [_I, _P, _P, _I, _P],
    "gsvc_bin_tiles_workspace_bytes": [_I, _I, _I],
    "gsvc_bin_tiles_counted_workspace_bytes": [_I],
    "gsvc_bin_tiles_counted": [_I, _P, _P, _I, _I, ctypes.c_longlong, _I, _P, _P, _P, _P, _P, _SZ,
                               _P],
    "gsvc_bin_and_sort_tiles": [_I, _I, _P, _P, _P, _P, _I, _I, _P, _P, _I, _P, _P, _SZ, _P],
    "gsvc_rasterize_sum_forward": [_I, _I, _I, _I, _I, _I, _U, _U, _U, _P, _P, _P, _P, _P, _P, _P,
                                   _P, _P, _P, _P],
    "gsvc_rasterize_sum_forward_ex": [_I, _I, _I, _I, _I, _I, _U, _U, _U, _P, _P, _P, _P, _P, _P,
                                      _P, _P, _I, _I, _P, _P, _P, _P],
    "gsvc_render_frame_workspace_bytes": [_I, _U, _U],
    "gsvc_render_frame_zeroed_bytes": [_U, _U],
    "gsvc_render_frame_sum": [_I, _P, _I, _P, _P, _P, _P, _P, _P, _U, _U, _I, _I, _P, _P, _SZ, _P,
                              _P],
    "gsvc_render_frame_sum_ex": [_I, _P, _I, _P, _P, _P, _P, _P, _P, _U, _U, _I, _I, _P, _P, _SZ,
                                 _P, _P, _I],
    "gsvc_train_step_workspace_bytes": [_I, _U, _U],
    "gsvc_train_step_det_workspace_bytes": [_I, ctypes.c_longlong],
    "gsvc_rasterize_sum_backward_det_workspace_bytes": [_I, ctypes.c_longlong],
    "gsvc_rasterize_sum_backward_det": [_U, _U, _U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                        _P, _P, _SZ, ctypes.c_longlong, _P, _P],
    "gsvc_train_step_sum_args": [_P],
    "gsvc_train_step_sum": [_I, _P, _P, _P, _P, _P, _I, _P, _P, _U, _U, _I, _I, _P, _P, _I, _P, _P,
                            _P, _P, _SZ, _P],
    "gsvc_i420_to_rgb": [_P, _I, _I, _P, _P],
    "gsvc_ssim_workspace_bytes": [_I, _I, _I, _I, _I],
    "gsvc_ssim_forward": [_I, _I, _I, _I, _P, _P, _I, _F, _F, _F, _I, _P, _I, _P, _P, _SZ, _P],
    "gsvc_ssim_backward_scratch_bytes": [_I, _I, _I, _I, _I],
    "gsvc_ssim_backward": [_I, _I, _I, _I, _P, _P, _I, _F, _F, _F, _I, _I, _P, _P, _P, _P, _SZ,
                           _P, _SZ, _P],
    "gsvc_render_frames_workspace_bytes": [_I, _I, _U, _U],
    "gsvc_render_frames_zeroed_bytes": [_I, _U, _U],
    "gsvc_render_frames_sum": [_I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _U, _U, _I, _I, _P, _P,
                               _SZ, _P, _P],
    "gsvc_adan_step": [_I, _P, _P, _P, _P, _P, _P, _P] + [ctypes.c_double] * 9 +
                      [_I, ctypes.c_double, _P],
    "gsvc_rasterize_sum_backward": [_U, _U, _U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                    _P, _P],
    "gsvc_rasterize_forward": [_I, _I, _I, _I, _I, _I, _U, _U, _U, _P, _P, _P, _P, _P, _P, _P,
                               _P, _P, _P, _P],
    "gsvc_rasterize_backward": [_U, _U, _U, _U, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                _P, _P],
}
# include/gsvc_amd_diag.h: the diagnostic library's extra entry points
_DIAG_SIGS = {
    "gsvc_debug_set": [_I, _I],
    "gsvc_debug_set_ptr": [_P],
}
_RESTYPE = {
    "gsvc_debug_set_ptr": None,
    "gsvc_alpha_cut_bits": _U,
    "gsvc_host_alloc": _P,
    "gsvc_last_error": ctypes.c_char_p,
    "gsvc_cumsum_workspace_bytes": _SZ,
    "gsvc_prune_workspace_bytes": _SZ,
    "gsvc_sort_pairs_workspace_bytes": _SZ,
    "gsvc_bin_tiles_workspace_bytes": _SZ,
    "gsvc_bin_tiles_counted_workspace_bytes": _SZ,
    "gsvc_render_frame_workspace_bytes": _SZ,
    "gsvc_rasterize_sum_slabs_workspace_bytes": _SZ,
    "gsvc_rasterize_sum_order_workspace_bytes": _SZ,
    "gsvc_render_frame_zeroed_bytes": _SZ,
    "gsvc_train_step_workspace_bytes": _SZ,
    "gsvc_train_step_det_workspace_bytes": _SZ,
    "gsvc_rasterize_sum_backward_det_workspace_bytes": _SZ,
    "gsvc_render_frames_workspace_bytes": _SZ,
    "gsvc_render_frames_zeroed_bytes": _SZ,
    "gsvc_ssim_workspace_bytes": _SZ,
    "gsvc_ssim_backward_scratch_bytes": _SZ,
}

ABI_VERSION = 2

_libs = {}       # path -> loaded CDLL
_active = None   # the library ops call (load())
_lock = threading.Lock()


def symbols(diag: bool = False):
    """Names of every entry point declared in include/gsvc_amd.h (with
    ``diag``: also include/gsvc_amd_diag.h)."""
    return list(_SIGS) + (list(_DIAG_SIGS) if diag else [])


def _open(path: str, diag: bool):
    lib = _libs.get(path)
    if lib is not None:
        return lib
    with _lock:
        lib = _libs.get(path)
        if lib is None:
            if not os.path.exists(path):
                raise RuntimeError(
                    f"gsvc_amd: {path} not found; build it with `python -m gsvc_amd.build` "
                    "(there is no CPU fallback)")
            lib = ctypes.CDLL(path)
            for name, args in list(_SIGS.items()) + (list(_DIAG_SIGS.items()) if diag else []):
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, _I)
            v = lib.gsvc_abi_version()
            if v != ABI_VERSION:
                raise RuntimeError(f"gsvc_amd: ABI version {v} != {ABI_VERSION}; rebuild the library")
            _libs[path] = lib
    return lib


def load():
    """The library the ops call: libgsvc_amd.so, or the diagnostic build when
    GSVC_DIAG=1 or inside ``diagnostic()`` (raises if it has not been built)."""
    global _active
    if _active is None:
        if os.environ.get("GSVC_DIAG") == "1":
            _active = _open(DIAG_LIB_PATH, True)
        else:
            _active = _open(LIB_PATH, False)
    return _active


def load_product():
    """libgsvc_amd.so itself, whatever library is active."""
    return _open(LIB_PATH, False)


TORCH_EXT_PATH = os.path.join(_HERE, "lib", "_torch_ops.so")
_ext = None


def torch_ops():
    """The C++ autograd Functions of the drop-in operators (csrc/torch_ops.cpp,
    a torch extension module over libgsvc_amd.so); raises if it has not been
    built -- there is no silent fallback."""
    global _ext
    if _ext is None:
        with _lock:
            if _ext is None:
                if not os.path.exists(TORCH_EXT_PATH):
                    raise RuntimeError(f"gsvc_amd: {TORCH_EXT_PATH} not found; build it with "
                                       "`python -m gsvc_amd.build`")
                import importlib.util
                spec = importlib.util.spec_from_file_location("_torch_ops", TORCH_EXT_PATH)
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                if mod.abi_version() != ABI_VERSION:
                    raise RuntimeError("gsvc_amd: _torch_ops.so was built for another ABI; rebuild")
                _ext = mod
    return _ext


def product_active() -> bool:
    """Whether the ops run on the product library (not inside diagnostic())."""
    return load() is _libs.get(LIB_PATH)


@contextlib.contextmanager
def diagnostic():
    """Run this package's ops on libgsvc_amd_diag.so for the block (its A/B
    knobs: gsvc_debug_set); yields that library.  Objects that bound a
    library function before the block (BoundStep, BoundRender) keep theirs."""
    global _active
    prev = load()
    lib = _open(DIAG_LIB_PATH, True)
    _active = lib
    try:
        yield lib
    finally:
        _active = prev


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        msg = load().gsvc_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")


def size(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


_raw_stream = torch._C._cuda_getCurrentRawStream  # the handle, without a Stream object


def stream(device) -> ctypes.c_void_p:
    index = device.index if device.index is not None else torch.cuda.current_device()
    return ctypes.c_void_p(_raw_stream(index))
