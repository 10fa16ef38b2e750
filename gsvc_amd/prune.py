"""Device-side pruning of a frame model (gsvc_prune_lowest, csrc/prune.hip).

Replaces, in GaussianSplats_Represent.py:101-125 (removal_control) and
:149-166 (adaptive_control), the sequence

    rgb_weight = torch.norm(self.rgb_W, dim=1)
    _, sorted_indices = torch.sort(rgb_weight)
    keep = torch.ones(N, dtype=torch.bool); keep[sorted_indices[:remove_count]] = False
    p = nn.Parameter(p[keep])    # _xyz, _cholesky, _features_dc, rgb_W

with one radix select and one stream compaction on the GPU: the same kept rows
in the same order (equal norms leave in index order, as the GPU's stable
torch.sort), no sort of all N keys, no boolean mask and no host sync.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import torch
from torch import Tensor

from . import _lib as L

_raw_stream = torch._C._cuda_getCurrentRawStream


def prune_lowest(rgb_w: Tensor, tensors: Sequence[Tensor], remove_count: int) -> List[Tensor]:
    """The rows of each of ``tensors`` ([N, C] fp32 on one HIP device) kept
    after removing the ``remove_count`` splats of smallest ``||rgb_w||`` per
    row (``rgb_w``: [N, 1] fp32).  Returns new tensors; the inputs are not
    modified.  ``remove_count >= N`` keeps nothing."""
    n = rgb_w.shape[0]
    if rgb_w.dim() != 2 or rgb_w.shape[1] != 1:
        raise ValueError(f"prune_lowest: rgb_w must be [N, 1], got {tuple(rgb_w.shape)}")
    remove_count = int(remove_count)
    if remove_count < 0:
        raise ValueError("prune_lowest: remove_count must be >= 0")
    if len(tensors) > 8:
        raise ValueError("prune_lowest: at most 8 tensors")
    for t in (rgb_w, *tensors):
        if not t.is_cuda:
            raise RuntimeError("prune_lowest: every tensor must be a CUDA (HIP) tensor")
        if t.dtype != torch.float32:
            raise RuntimeError("prune_lowest: every tensor must be float32")
        if t.device != rgb_w.device:
            raise RuntimeError("prune_lowest: tensors on different devices")
    srcs = []
    for t in tensors:
        if t.dim() != 2 or t.shape[0] != n:
            raise ValueError(f"prune_lowest: tensors must be [N={n}, C], got {tuple(t.shape)}")
        srcs.append(t.detach().contiguous())
    w = rgb_w.detach().contiguous()
    keep = max(n - remove_count, 0)
    outs = [torch.empty((keep, t.shape[1]), dtype=torch.float32, device=w.device) for t in srcs]
    if keep == 0 or n == 0:
        return outs
    k = len(srcs)
    ws = torch.empty((L.size("gsvc_prune_workspace_bytes", n),), dtype=torch.uint8, device=w.device)
    cols = (ctypes.c_int * max(k, 1))(*[t.shape[1] for t in srcs])
    src_p = (ctypes.c_void_p * max(k, 1))(*[t.data_ptr() for t in srcs])
    dst_p = (ctypes.c_void_p * max(k, 1))(*[t.data_ptr() for t in outs])
    L.call("gsvc_prune_lowest", n, remove_count, w.data_ptr(), k, ctypes.addressof(cols),
           ctypes.addressof(src_p), ctypes.addressof(dst_p), ws.data_ptr(), ws.numel(),
           _raw_stream(w.device.index))
    return outs
