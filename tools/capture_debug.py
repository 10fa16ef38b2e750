"""Graph-capture probe of the counted binning (tests/test_capture.py debugging):
capture gsvc_bin_tiles_counted on a torch graph in three variants, replay,
and compare the bins with the eager call.
  V1 workspace allocated inside the capture (ops.bin_tiles_counted)
  V2 workspace allocated before the capture (static)
  V3 V2 plus a captured torch zero_() of the workspace before the call"""
import sys

import torch

sys.path.insert(0, ".")
from gsvc_amd import _lib as L  # noqa: E402
from gsvc_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
H, W, n = 256, 384, 3000
g = torch.Generator().manual_seed(3011)
means = (2 * torch.rand(n, 2, generator=g) - 1).to(dev)
Lc = (torch.rand(n, 3, generator=g) + torch.tensor([0.5, 0.0, 0.5])).to(dev)
tb = ((W + 15) // 16, (H + 15) // 16, 1)
nt = tb[0] * tb[1]
cap = nt * min(n, 256)
xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(n, means, Lc, H, W, tb, 0.01)
torch.cuda.synchronize()
e_gids, e_bins, e_meta = ops.bin_tiles_counted(n, xys, radii, tb, cap, 256)
torch.cuda.synchronize()
print("eager M", int(e_meta[0]), flush=True)

ws_static = torch.empty((L.size("gsvc_bin_tiles_counted_workspace_bytes", nt) // 4 + 1,),
                        dtype=torch.int32, device=dev)
sc_static = torch.empty((cap,), dtype=torch.int32, device=dev)


def v2(zero):
    gids = torch.empty((cap,), dtype=torch.int32, device=dev)
    bins = torch.empty((nt, 2), dtype=torch.int32, device=dev)
    meta = torch.empty((2,), dtype=torch.int32, device=dev)
    if zero:
        ws_static.zero_()
    L.call("gsvc_bin_tiles_counted", n, L.ptr(xys), L.ptr(radii), tb[0], tb[1], cap, 256,
           L.ptr(sc_static), L.ptr(gids), L.ptr(bins), L.ptr(meta), L.ptr(ws_static),
           4 * ws_static.numel(), L.stream(dev))
    return gids, bins, meta


variants = {"V1": lambda: ops.bin_tiles_counted(n, xys, radii, tb, cap, 256),
            "V2": lambda: v2(False), "V3": lambda: v2(True)}
for name, fn in variants.items():
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g_gids, g_bins, g_meta = fn()
    res = []
    for r in range(3):
        graph.replay()
        torch.cuda.synchronize()
        res.append((int(g_meta[0]), torch.equal(g_bins, e_bins)))
    print(name, res, flush=True)
    del graph
