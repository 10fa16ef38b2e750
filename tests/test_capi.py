"""CPU: the C-ABI library loads, exports every symbol include/gsvc_amd.h
declares, shares torch's HIP runtime, and the HIP op table refuses CPU tensors
(no GPU call falls back to the CPU; CPU tensors have their own dispatch,
tests/test_cpu_path.py)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import REPO

HEADER = os.path.join(REPO, "include", "gsvc_amd.h")
DIAG_HEADER = os.path.join(REPO, "include", "gsvc_amd_diag.h")


def _declared(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gsvc_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    assert "gsvc_rasterize_sum_forward" in names and "gsvc_project_gaussians_2d_forward" in names
    assert len(names) >= 15


def test_library_exports_all_symbols():
    from gsvc_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes signature table covers exactly the declared ABI
    assert sorted(_lib.symbols()) == _declared()


def test_product_library_has_no_diagnostics():
    """the A/B knobs and diagnostic kernel variants live only in
    libgsvc_amd_diag.so (include/gsvc_amd_diag.h); the product library exports
    none of its entry points and carries none of its kernel variants."""
    import subprocess
    from gsvc_amd import _lib
    diag = _declared(DIAG_HEADER)
    assert diag == ["gsvc_debug_set", "gsvc_debug_set_ptr"]
    prod = ctypes.CDLL(_lib.LIB_PATH)
    assert not [n for n in diag if hasattr(prod, n)]
    dlib = ctypes.CDLL(_lib.DIAG_LIB_PATH)
    assert not [n for n in _declared() + diag if not hasattr(dlib, n)]
    assert sorted(_lib.symbols(diag=True)) == sorted(_declared() + diag)

    # the timestamped / ablation / A/B variants are diagnostic-only symbols
    names = subprocess.run(["nm", "-C", _lib.LIB_PATH], capture_output=True, text=True).stdout
    dnames = subprocess.run(["nm", "-C", _lib.DIAG_LIB_PATH], capture_output=True, text=True).stdout
    for variant in ("raster_sum_fwd_kernel<7,", "raster_sum_fwd_kernel<3,", "train_tile_kernel<",
                    "train_tile_band_kernel<true", "frame_project_kernel<1, true>",
                    "train_splat_kernel<true"):
        assert variant not in names, variant
        assert variant in dnames, variant


def test_abi_version_and_queries():
    from gsvc_amd import _lib
    lib = _lib.load()
    assert lib.gsvc_abi_version() == _lib.ABI_VERSION
    assert lib.gsvc_cumsum_workspace_bytes(50000) > 0
    assert lib.gsvc_sort_pairs_workspace_bytes(124000) >= 124000 * 12
    assert lib.gsvc_bin_tiles_workspace_bytes(50000, 124000, 8160) >= 124000 * 20


def test_argument_errors_are_reported_without_launch():
    from gsvc_amd import _lib
    lib = _lib.load()
    rc = lib.gsvc_rasterize_sum_forward(8, 8, 1, 8, 8, 1, 128, 128, 1, *([None] * 10), None)
    assert rc == 1
    assert b"16x16" in lib.gsvc_last_error()


def test_bin_tiles_counted_rejects_partial_caps():
    """The overflow rebuild writes 256 ids per overfull tile, so the only caps
    are 0 (keep all) and 256 (what the rasterizers read); anything else is an
    argument error before any HIP call (C ABI) or a ValueError (ops)."""
    from gsvc_amd import _lib, ops
    lib = _lib.load()
    for cap in (1, 100, 255, 257, 1024):
        rc = lib.gsvc_bin_tiles_counted(10, None, None, 2, 2, 1024, cap, None, None, None, None,
                                        None, 0, None)
        assert rc == 1 and b"tile_cap" in lib.gsvc_last_error(), cap
        with pytest.raises(ValueError, match="tile_cap"):
            ops.bin_tiles_counted(10, torch.zeros(10, 2), torch.zeros(10, dtype=torch.int32),
                                  (2, 2, 1), 1024, cap)


def test_prune_and_timing_argument_errors():
    """gsvc_prune_lowest / gsvc_timing_enable check their arguments before any
    HIP call; a prune that keeps nothing launches nothing."""
    from gsvc_amd import _lib
    lib = _lib.load()
    assert lib.gsvc_prune_workspace_bytes(100000) >= 8 * 98
    assert lib.gsvc_prune_lowest(10, -1, None, 0, None, None, None, None, 0, None) == 1
    assert lib.gsvc_prune_lowest(10, 2, None, 9, None, None, None, None, 0, None) == 1
    assert lib.gsvc_prune_lowest(10, 2, None, 0, None, None, None, None, 0, None) == 1
    assert b"rgb_w" in lib.gsvc_last_error()
    assert lib.gsvc_prune_lowest(10, 10, None, 0, None, None, None, None, 0, None) == 0
    w = ctypes.c_void_p(16)  # never dereferenced: the workspace check fails first
    assert lib.gsvc_prune_lowest(10, 2, w, 0, None, None, None, None, 0, None) == 2
    assert lib.gsvc_timing_enable(4, 1, 2) == 1
    assert b"how" in lib.gsvc_last_error()
    assert lib.gsvc_timing_enable(0, 0, 0) == 0
    from gsvc_amd.prune import prune_lowest
    with pytest.raises(RuntimeError, match="CUDA"):
        prune_lowest(torch.ones(4, 1), [torch.ones(4, 2)], 1)


def test_single_hip_runtime_loaded():
    from gsvc_amd import _lib
    _lib.load()
    maps = open("/proc/self/maps").read()
    libs = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(libs) == 1, libs


def test_product_path_rejects_cpu_tensors():
    """The HIP op table (the reference's `_C` ops) takes device tensors only;
    the two operators dispatch CPU tensors to the CPU library (test_cpu_path)."""
    from gsvc_amd import ops
    means = torch.zeros(4, 2)
    L = torch.ones(4, 3)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        ops.project_gaussians_2d_forward(4, means, L, 32, 32, (2, 2, 1), 0.01)


def test_dropin_package_surface():
    import gsplat
    import gsplat.cuda as C
    for name in ("project_gaussians_2d", "rasterize_gaussians_sum", "rasterize_gaussians",
                 "bin_and_sort_gaussians", "compute_cumulative_intersects", "compute_cov2d_bounds",
                 "get_tile_bin_edges", "map_gaussian_to_intersects", "RasterizeGaussiansSum"):
        assert hasattr(gsplat, name)
    for op in ("project_gaussians_2d_forward", "project_gaussians_2d_backward",
               "rasterize_sum_forward", "rasterize_sum_backward", "map_gaussian_to_intersects",
               "get_tile_bin_edges", "compute_cov2d_bounds"):
        assert callable(getattr(C, op))
    with pytest.raises(AttributeError):
        C.nd_rasterize_sum_forward  # noqa: B018  (not exported by the reference either)
    with pytest.raises(NotImplementedError):
        gsplat.project_gaussians()


def test_train_step_args_struct_layout(tmp_path):
    """gsvc_amd.train._StepArgs mirrors include/gsvc_amd.h gsvc_train_step_args
    field by field (offsets from the C compiler)."""
    import shutil
    import subprocess
    from gsvc_amd.train import _StepArgs
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    names = [f[0] for f in _StepArgs._fields_]
    body = "".join(f'printf("%zu ", offsetof(gsvc_train_step_args, {n}));' for n in names)
    src = tmp_path / "off.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\nint main(void){%s'
                   'printf("%%zu\\n", sizeof(gsvc_train_step_args));return 0;}\n' % (HEADER, body))
    exe = tmp_path / "off"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert got[:-1] == [getattr(_StepArgs, n).offset for n in names]
    assert got[-1] == ctypes.sizeof(_StepArgs)


def test_host_seq_wait_without_gpu_work():
    """gsvc_wait_host_seq returns at once when the word already holds the
    sequence (coherent host memory needs a HIP runtime; skip without one)."""
    from gsvc_amd import _lib
    lib = _lib.load()
    rc = lib.gsvc_wait_host_seq(None, 1, None, 10)
    assert rc != 0 and b"null" in lib.gsvc_last_error()
    buf = (ctypes.c_uint * 4)(0, 0, 0x80000005, 0)
    assert lib.gsvc_wait_host_seq(ctypes.addressof(buf) + 8, 0x80000005, None, 10) == 0


def test_train_step_ahead_flag_errors_without_launch():
    """The tile-kernel-ahead flags (GSVC_TRAIN_TILES_NEXT / TILED / REBUILD_NEXT)
    are checked before any HIP call: they need the carried bins of a projected
    frame and the Adan update; REBUILD_NEXT needs TILES_NEXT."""
    from gsvc_amd import _lib
    from gsvc_amd import train as T
    lib = _lib.load()
    dummy = 16  # never dereferenced: the flag checks fail first
    state = (ctypes.c_void_p * 16)(*([dummy] * 16))
    hp = (ctypes.c_double * 10)()
    a = T._StepArgs()
    a.num_points = 10
    a.xyz = a.cholesky = a.features = a.rgb_w = a.background = a.gt = a.loss = dummy
    a.img_height, a.img_width = 32, 32
    a.adan_state, a.adan_hparams = ctypes.addressof(state), ctypes.addressof(hp)
    a.workspace, a.workspace_bytes = dummy, 1 << 40
    base = T.TRAIN_PROJECTED | T.TRAIN_CARRY
    cases = [
        (T.TRAIN_PROJECTED | T.TRAIN_TILED, b"TILED"),  # no carried bins
        (T.TRAIN_CARRY | T.TRAIN_TILES_NEXT, b"TILED"),  # not projected
        (base | T.TRAIN_REBUILD_NEXT, b"REBUILD_NEXT"),
    ]
    for flags, msg in cases:
        a.adan_flags = flags
        assert lib.gsvc_train_step_sum_args(ctypes.byref(a)) == 1, hex(flags)
        assert msg in lib.gsvc_last_error(), (hex(flags), lib.gsvc_last_error())
    # the gradient-only test hook has no update to run the next tile kernel behind
    a.adan_flags, a.grads_out = base | T.TRAIN_TILES_NEXT, dummy
    assert lib.gsvc_train_step_sum_args(ctypes.byref(a)) == 1
    assert b"Adan update" in lib.gsvc_last_error()


def test_slabs_ordered_argument_errors_without_launch():
    """gsvc_rasterize_sum_forward_slabs_ordered checks its order flags and
    workspaces before any HIP call; the order workspace grows with the splat
    count and has room for the sort's counters."""
    from gsvc_amd import _lib
    lib = _lib.load()
    assert lib.gsvc_rasterize_sum_order_workspace_bytes(50000) >= 6 * 4 * 50000
    assert lib.gsvc_rasterize_sum_order_workspace_bytes(1) > 0
    args = [10, None, None, None, None, None, None, 64, 64, 0, 0, None, 0, None, None, None, None,
            None, None, None]
    assert lib.gsvc_rasterize_sum_forward_slabs_ordered(*args, None, 0, 0x1) == 1
    assert b"unknown flags" in lib.gsvc_last_error()
    assert lib.gsvc_rasterize_sum_forward_slabs_ordered(*args, None, 0, 0x200) == 2
    assert b"order workspace" in lib.gsvc_last_error()
    w = ctypes.c_void_p(16)  # never dereferenced: the slab workspace check fails first
    assert lib.gsvc_rasterize_sum_forward_slabs_ordered(*args, w, 16, 0x200) == 2
