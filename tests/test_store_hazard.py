"""The gfx940+ store-data hazard behind round 5's lost tile rows.

CPU: tools/store_hazard_scan.py finds no VALU write to a >64-bit store's data
VGPRs within two wait states in the product and diagnostic libraries, and the
scanner itself flags the round-5 code shape (a synthetic disassembly of the
exact sequence) while passing its padded form.

GPU: a 1080p frame through every image store layout the library has -- the
render's CHW planes (sparse kernel: 16-byte write-through rows; banded:
8-byte), the op path's HWC rows (C++ Function over id slabs; the Python
Function with final_idx; the banded kernel) -- each held to the C oracle at
every pixel, three calls each (the round-5 fault hit 1-4 % of tiles per call).
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, knobs

sys.path.insert(0, os.path.join(REPO, "tools"))
import store_hazard_scan as S  # noqa: E402

LIBDIR = os.path.join(REPO, "gsvc_amd", "lib")
_TOOLS = all(os.path.exists(os.path.join(S.LLVM, t))
             for t in ("llvm-objcopy", "llvm-objdump", "clang-offload-bundler"))

# the round-5 sequence (raster_sum_fwd_kernel<1, true>, HWC row store j = 0)
_R5 = """
0000000000001000 <k>:
	s_waitcnt lgkmcnt(0)                                       // 000000001000: BF8CC07F
	global_store_dwordx4 v[10:11], v[6:9], off nt sc1          // 000000001004: DE7E8000 007F060A
	s_or_b64 exec, exec, s[0:1]                                // 00000000100C: 87FE007E
	v_or_b32_e32 v6, 64, v18                                   // 000000001010: 280C24C0
	s_endpgm                                                   // 000000001014: BF810000
"""


def test_scanner_flags_round5_sequence_and_passes_padded():
    f = S.parse(_R5)["k"]
    hits = S.scan_function(f)
    assert len(hits) == 1 and hits[0][4] == "v_or_b32_e32" and hits[0][6] == 1
    padded = _R5.replace("	s_or_b64", "	s_nop 1                                                    "
                         "// 00000000100A: BF800001\n	s_or_b64")
    assert S.scan_function(S.parse(padded)["k"]) == []
    # a branch into a block whose first VALU overwrites the data: followed too
    branchy = """
0000000000002000 <b>:
	global_store_dwordx4 v[0:1], v[2:5], off                   // 000000002000: DC7C0000 007F0200
	s_cbranch_execz 1                                          // 000000002008: BF880001
	s_nop 4                                                    // 00000000200C: BF800004
	v_mov_b32_e32 v3, 0                                        // 000000002010: 7E060280
	s_endpgm                                                   // 000000002014: BF810000
"""
    hits = S.scan_function(S.parse(branchy)["b"])
    assert len(hits) == 1 and hits[0][6] == 1


@pytest.mark.skipif(not _TOOLS, reason="ROCm LLVM tools absent")
@pytest.mark.parametrize("lib", ["libgsvc_amd.so", "libgsvc_amd_diag.so"])
def test_libraries_have_no_store_data_hazard(lib):
    path = os.path.join(LIBDIR, lib)
    if not os.path.exists(path):
        pytest.skip(f"{lib} not built")
    assert S.scan(path) == []


def _frame(n, seed, dev):
    g = torch.Generator().manual_seed(seed)
    means = (2 * torch.rand(n, 2, generator=g) - 1)
    L = torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0.0, 0.5])
    col = torch.rand(n, 3, generator=g)
    return means.to(dev), L.to(dev), col.to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [10000, 50000])
def test_every_store_layout_matches_oracle_1080p(cuda, oracle, n):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    from gsvc_amd.rasterize_sum import _RasterizeGaussiansSum
    from gsvc_amd.render import render_frame_sum
    H, W = 1080, 1920
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    means, L, col = _frame(n, 1234 + n, cuda)
    o = torch.ones(n, 1, device=cuda)
    bg = torch.ones(3, device=cuda)
    r = oracle.render_sum(means.cpu().numpy(), L.cpu().numpy(), col.cpu().numpy(),
                          np.ones((n, 1), np.float32), H, W)
    want_hwc = r["out"]
    want_chw = np.clip(want_hwc, 0, 1).transpose(2, 0, 1)
    xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)

    def op_cpp():  # the C++ Function: id slabs, HWC rows
        return rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, o, H, W, 16, 16,
                                       background=bg)

    def op_py():  # the Python Function: counted binning, HWC rows + final_idx
        return _RasterizeGaussiansSum.apply(xys, depths, radii, conics, nth, col, o, H, W, 16, 16,
                                            bg, False)

    # render_frame_sum takes the pre-tanh centres: atanh of the means
    xyz = torch.atanh(means.clamp(-1 + 1e-7, 1 - 1e-7))
    mt = torch.tanh(xyz)
    r2 = oracle.render_sum(mt.cpu().numpy(), L.cpu().numpy(), col.cpu().numpy(),
                           np.ones((n, 1), np.float32), H, W)
    want_render = np.clip(r2["out"], 0, 1).transpose(2, 0, 1)

    def render():  # CHW planes, 16-byte write-through rows (sparse kernel)
        return render_frame_sum(xyz, L, col, H, W, bg)[0]

    routes = {"op_cpp_hwc": (op_cpp, want_hwc), "op_py_hwc": (op_py, want_hwc),
              "render_chw": (render, want_render)}
    checked = []
    for name, (fn, want) in routes.items():
        for _ in range(3):
            got = fn().detach().cpu().numpy()
            np.testing.assert_allclose(got, want, rtol=0, atol=1e-5, err_msg=name)
            checked.append(name)
    # the banded kernel: CHW planes with 8-byte stores, HWC rows (diagnostic
    # library: knob 0 = 2 forces it; the product picks it past 96 entries per tile)
    with knobs((0, 2)):
        for _ in range(3):
            np.testing.assert_allclose(render().cpu().numpy(), want_render, rtol=0, atol=1e-5,
                                       err_msg="render_chw_banded")
            np.testing.assert_allclose(op_py().detach().cpu().numpy(), want_hwc, rtol=0, atol=1e-5,
                                       err_msg="op_py_hwc_banded")
    assert len(checked) == 9
