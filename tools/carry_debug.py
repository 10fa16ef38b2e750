"""Debug: one step's render and gradients read from carried bins vs the
plain projection (grads_out mode, nothing updated)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gsvc_amd import train as T
from gsvc_amd.frame import make_frame_model, synthetic_gt

dev = torch.device("cuda:0")
H, W, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
m = make_frame_model(H, W, n, dev, seed=3)
gt = synthetic_gt(H, W, 4, dev)


def step(flags_first, flags):
    g = torch.empty((n, 9), device=dev)
    img = torch.empty((3, H, W), device=dev)
    args = (m._xyz.data, m._cholesky.data, m._features_dc.data, m.rgb_W.data, False,
            m.cholesky_bound, m.background, gt.contiguous(), H, W, "L2")
    ws = T._workspace(dev, n, H, W)
    if flags_first is not None:
        T.train_step_sum(*args, adan_flags=flags_first, grads_out=torch.empty((n, 9), device=dev))
        ws.frame -= 1
    loss = T.train_step_sum(*args, adan_flags=flags, render_out=img, grads_out=g)
    torch.cuda.synchronize()
    return loss.cpu(), img, g


la, ia, ga = step(None, 0)
lb, ib, gb = step(T.TRAIN_PROJECT_ONLY | T.TRAIN_CARRY, T.TRAIN_PROJECTED | T.TRAIN_CARRY)
print("loss", la.tolist(), lb.tolist())
d = (ia - ib).abs().amax(0)
tiles = d.unfold(0, 16, 16).unfold(1, 16, 16).amax((-1, -2))
print("bad tiles", int((tiles > 0).sum()), "of", tiles.numel(), "max img diff", float(d.max()))
print("grad max diff", float((ga - gb).abs().max()), "scale", float(ga.abs().max()))
bad = (tiles > 0).nonzero()[:10].tolist()
print("first bad tiles (ty, tx)", bad)
print("mean img a/b", float(ia.mean()), float(ib.mean()))
