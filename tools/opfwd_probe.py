"""Debug: the op path's grad-enabled forward alone (bench.py op_path "fwd") --
wall time per call, then a torch.profiler table of 50 calls (host time per op
and the GPU kernels), at the bench's trained 1080p / 50k frame.

    python tools/opfwd_probe.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from gsvc_amd.frame import make_frame_model
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(REPO, "tests", "golden", "train_state_1080p_n50k.npz"))
    n = int(z["n"])
    op = make_frame_model(1080, 1920, n, dev, seed=0, fused_train=False, fused_render=False)
    with torch.no_grad():
        for k in ("_xyz", "_cholesky", "_features_dc"):
            getattr(op, k).copy_(torch.from_numpy(z["state_" + k]))

    def timed(fn, k=200, w=20):
        for _ in range(w):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    def fwd():
        op.forward()

    def fwd_keep():
        fwd_keep.last = op.forward()

    def render():
        with torch.no_grad():
            op.forward()

    print({"fwd_us": round(timed(fwd), 1), "fwd_keep_us": round(timed(fwd_keep), 1),
           "render_us": round(timed(render), 1)}, flush=True)
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(50):
            fwd()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=60))
    if "--bench" in sys.argv:
        # the bench's op_path block, alone and after the bench's render blocks
        import bench as B
        from gsvc_amd.frame import synthetic_gt
        gt = synthetic_gt(1080, 1920, int(z["gt_seed"]), "cpu").to(dev)
        m = make_frame_model(1080, 1920, n, dev, seed=0)
        with torch.no_grad():
            for k in ("_xyz", "_cholesky", "_features_dc"):
                getattr(m, k).copy_(torch.from_numpy(z["state_" + k]))
        r = B.op_path_block(m, gt, dev)
        print("alone", {k: r[k] for k in ("fwd_us", "fwd_bwd_us", "render_fps")}, flush=True)
        B.render_10k(dev)
        B.video_decode(dev)
        r = B.op_path_block(m, gt, dev)
        print("after render blocks", {k: r[k] for k in ("fwd_us", "fwd_bwd_us", "render_fps")},
              flush=True)
        print(torch.cuda.memory_summary(abbreviated=True)[:3000], flush=True)


if __name__ == "__main__":
    main()
