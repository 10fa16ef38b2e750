"""The unit-opacity alpha cut as a sigma threshold (csrc/alpha_cut.hip,
common.h kSigmaCutBits), proven on the device over every float.

The reference keeps a (splat, pixel) pair when !(sigma < 0) and
!(min(1, opacity * exp(-sigma)) < 1/255) (forward.cu:598-606,
backward.cu:822-828).  At opacity 1 the kernels test bits(sigma) <=
kSigmaCutBits instead and use exp(-sigma) unclamped; this holds for every
non-NaN sigma iff the kept patterns are exactly [0, kSigmaCutBits] and none
of them has exp(-sigma) > 1.
"""
import numpy as np
import pytest
import torch


@pytest.mark.gpu
def test_sigma_cut_is_the_reference_alpha_cut(cuda):
    from gsvc_amd import _lib as L
    lib = L.load()
    out = torch.zeros(4, dtype=torch.int32, device=cuda)
    assert lib.gsvc_alpha_cut_scan(out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    kept_max, drop_min, over, nan_kept = (int(v) & 0xffffffff for v in out.cpu().tolist())
    cut = int(lib.gsvc_alpha_cut_bits())
    sigma = np.array([kept_max], dtype=np.uint32).view(np.float32)[0]
    # the kept patterns are one prefix of the non-negative floats ...
    assert drop_min == kept_max + 1, (hex(kept_max), hex(drop_min))
    # ... which is the kernels' constant (about ln 255 = 5.541)
    assert cut == kept_max, (hex(cut), hex(kept_max), float(sigma))
    assert abs(float(sigma) - np.log(255.0)) < 1e-3
    # exp(-sigma) <= 1 wherever the pair is kept: the min(1, .) is a no-op there
    assert over == 0
    # the reference keeps NaN sigma (min(1, NaN) = 1): the kernels keep the
    # exact test for chunks with non-finite geometry
    assert nan_kept > 0
