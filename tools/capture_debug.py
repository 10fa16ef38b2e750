"""Graph-capture probe of the counted binning (tests/test_capture.py debugging).
E1: replays back to back (no eager launch between them), checked after.
E2: a torch-only graph replayed with eager ops in between.
E3: the binning graph, replay -> an eager torch op -> replay.
E4: the binning graph, replay -> an eager call of our library -> replay."""
import sys

import torch

sys.path.insert(0, ".")
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
M = int(e_meta[0])
print("eager M", M, flush=True)


def capture(fn):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = fn()
    return graph, out


binfn = lambda: ops.bin_tiles_counted(n, xys, radii, tb, cap, 256)  # noqa: E731
# E1
graph, (gg, gb, gm) = capture(binfn)
for _ in range(3):
    graph.replay()
torch.cuda.synchronize()
print("E1 back-to-back x3:", int(gm[0]), torch.equal(gb, e_bins), flush=True)
graph.replay()
torch.cuda.synchronize()
print("E1 4th:", int(gm[0]), torch.equal(gb, e_bins), flush=True)
del graph
# E2
x = torch.arange(1000, device=dev, dtype=torch.float32)
tg, y = capture(lambda: x * 2 + 1)
res = []
for _ in range(3):
    tg.replay()
    torch.cuda.synchronize()
    res.append(bool(torch.equal(y, x * 2 + 1)))
    _ = (x + 3).sum().item()
print("E2 torch graph with eager ops between:", res, flush=True)
# E3
graph, (gg, gb, gm) = capture(binfn)
res = []
for _ in range(3):
    graph.replay()
    torch.cuda.synchronize()
    res.append((int(gm[0]), bool(torch.equal(gb, e_bins))))
    _ = (x + 3).sum().item()
print("E3 eager torch op between:", res, flush=True)
del graph
# E4
graph, (gg, gb, gm) = capture(binfn)
res = []
for _ in range(3):
    graph.replay()
    torch.cuda.synchronize()
    res.append((int(gm[0]), bool(torch.equal(gb, e_bins))))
    ops.bin_tiles_counted(n, xys, radii, tb, cap, 256)
    torch.cuda.synchronize()
print("E4 eager library call between:", res, flush=True)
# E0: host cost of hipStreamIsCapturing through torch's HIP runtime, on the
# default stream (handle 0) and on a created stream
import ctypes  # noqa: E402
import time  # noqa: E402
hip = ctypes.CDLL(torch.__file__.rsplit("/", 1)[0] + "/lib/libamdhip64.so")
st = ctypes.c_int(0)
for name, h in (("default", torch.cuda.current_stream().cuda_stream), ("side", torch.cuda.Stream().cuda_stream)):
    t0 = time.perf_counter()
    for _ in range(2000):
        hip.hipStreamIsCapturing(ctypes.c_void_p(h), ctypes.byref(st))
    print(f"E0 hipStreamIsCapturing({name}, handle {h}): {(time.perf_counter() - t0) / 2000 * 1e6:.2f} us", flush=True)
