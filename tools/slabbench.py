"""The op path's rasterizer forward alone (gsvc_rasterize_sum_forward_slabs:
id insertion + the indexed composite with its sorted-id write-back) on the
bench's trained 1080p / 50k state, with an optional A/B pass of
gsvc_debug_set(KEY, VALUE).  Run it under
``rocprofv3 --kernel-trace --stats`` for the two kernels' times.

    python tools/slabbench.py [--calls 200] [--knob KEY VALUE] [--ordered]

--ordered: the C++ operator's call (torch_ops.cpp RasterSumFn): the ordered
insertion with its order workspace (refreshed every 64 calls), the gradient
records zeroed by the insertion, no final_idx.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# A/B knobs: the diagnostic library (gsvc_amd/_lib.py)
os.environ.setdefault("GSVC_DIAG", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsvc_amd import _lib as L  # noqa: E402

H, W = 1080, 1920


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--knob", type=int, nargs=2, action="append", default=[])
    ap.add_argument("--ordered", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = L.load()
    from gsvc_amd import ops
    z = np.load(os.path.join(REPO, "tests", "golden", "train_state_1080p_n50k.npz"))
    n = int(z["n"])
    xyz = torch.from_numpy(z["state__xyz"]).to(dev)
    chol = torch.from_numpy(z["state__cholesky"]).to(dev)
    feat = torch.from_numpy(z["state__features_dc"]).to(dev)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    xys, depths, radii, conics, nth = ops.project_gaussians_2d_forward(
        n, torch.tanh(xyz), chol + torch.tensor([0.5, 0.0, 0.5], device=dev), H, W, tb, 0.01)
    opac = torch.ones(n, 1, device=dev)
    bg = torch.ones(3, device=dev)
    T = tb[0] * tb[1]
    ws = torch.zeros((L.size("gsvc_rasterize_sum_slabs_workspace_bytes", T) + 3) // 4,
                     dtype=torch.int32, device=dev)
    gids = torch.empty(T * 256, dtype=torch.int32, device=dev)
    bins = torch.empty((T, 2), dtype=torch.int32, device=dev)
    meta = torch.empty(2, dtype=torch.int32, device=dev)
    out = torch.empty((H, W, 3), device=dev)
    idx = torch.empty((H, W), dtype=torch.int32, device=dev)
    calls = [0]

    ORDER, REFRESH = 0x200, 0x400
    ows = torch.empty(L.size("gsvc_rasterize_sum_order_workspace_bytes", n), dtype=torch.uint8,
                      device=dev)
    rec = torch.empty((n, 16), device=dev)

    def fwd_ordered():
        k = calls[0]
        flags = REFRESH if k == 0 else (ORDER | (REFRESH if k % 64 == 63 else 0))
        L.call("gsvc_rasterize_sum_forward_slabs_ordered", n, L.ptr(xys), L.ptr(radii),
               L.ptr(conics), L.ptr(feat), L.ptr(opac), L.ptr(bg), H, W, k, 250000, L.ptr(ws),
               4 * ws.numel(), L.ptr(gids), L.ptr(bins), L.ptr(meta), L.ptr(rec), L.ptr(out),
               None, L.stream(dev), L.ptr(ows), ows.numel(), flags)
        calls[0] += 1

    def fwd_plain():
        L.call("gsvc_rasterize_sum_forward_slabs", n, L.ptr(xys), L.ptr(radii), L.ptr(conics),
               L.ptr(feat), L.ptr(opac), L.ptr(bg), H, W, calls[0], 250000, L.ptr(ws),
               4 * ws.numel(), L.ptr(gids), L.ptr(bins), L.ptr(meta), None, L.ptr(out), L.ptr(idx),
               L.stream(dev))
        calls[0] += 1

    fwd = fwd_ordered if a.ordered else fwd_plain
    ref = None
    for kv in [None] + a.knob:
        if kv and lib.gsvc_debug_set(kv[0], kv[1]) < 0:
            raise ValueError("unknown A/B knob key (gsvc_debug_set returned -1)")
        for _ in range(20):
            fwd()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.calls):
            fwd()
        e1.record()
        torch.cuda.synchronize()
        img, fi = out.clone(), idx.clone()
        same = True if ref is None else bool(torch.equal(img, ref[0]) and torch.equal(fi, ref[1]))
        ref = ref or (img, fi)
        if kv:
            lib.gsvc_debug_set(kv[0], 0)
        print(json.dumps(dict(knob=kv, us_per_call=round(e0.elapsed_time(e1) * 1e3 / a.calls, 2),
                              M=int(meta[0]), identical=same)), flush=True)


if __name__ == "__main__":
    main()
