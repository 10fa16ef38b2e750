"""Host-side cost of one frame render call (GaussianVideoFrame.forward under
no_grad): enqueue time per call without synchronisation, against the GPU time
per frame, to tell whether the single-frame loop is host- or GPU-bound.

    python tools/hostbench.py [--splats 10000] [--calls 2000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, default=10000)
    ap.add_argument("--calls", type=int, default=2000)
    a = ap.parse_args()
    from gsvc_amd.frame import make_frame_model
    dev = torch.device("cuda:0")
    model = make_frame_model(1080, 1920, a.splats, dev, seed=1)
    model.eval()
    with torch.no_grad():
        for _ in range(50):
            model()
        torch.cuda.synchronize()
        # enqueue cost: calls issued back to back; the GPU queue absorbs them
        t0 = time.perf_counter()
        for _ in range(a.calls):
            model()
        t_enq = (time.perf_counter() - t0) / a.calls
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / a.calls
        # pieces of the host path
        from gsvc_amd import _lib as L
        from gsvc_amd.render import render_frame_sum
        t0 = time.perf_counter()
        for _ in range(a.calls):
            torch.cuda.current_stream(dev).cuda_stream
        t_stream = (time.perf_counter() - t0) / a.calls
        t0 = time.perf_counter()
        for _ in range(a.calls):
            torch.empty((1, 3, 1080, 1920), device=dev)
        t_empty = (time.perf_counter() - t0) / a.calls
        torch.cuda.synchronize()
        lib = L.load()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            lib.gsvc_abi_version()
        t_ctypes = (time.perf_counter() - t0) / a.calls
        # host cost without any GPU back-pressure: a 16x16 frame of 16 splats
        tiny = make_frame_model(16, 16, 16, dev, seed=2)
        tiny.eval()
        for _ in range(50):
            tiny()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            tiny()
        t_tiny_model = (time.perf_counter() - t0) / a.calls
        torch.cuda.synchronize()
        xyz, chol, feat = tiny._xyz, tiny._cholesky, tiny._features_dc
        bg, bound, rgbw = tiny.background, tiny.cholesky_bound, tiny.rgb_W
        t0 = time.perf_counter()
        for _ in range(a.calls):
            render_frame_sum(xyz, chol, feat, 16, 16, bg, cholesky_bound=bound, rgb_w=rgbw)
        t_tiny_render = (time.perf_counter() - t0) / a.calls
        torch.cuda.synchronize()
        # the bare C call (two kernel launches), pointers prepared once
        from gsvc_amd import render as R
        fw = R._workspace(dev, 16, 16, 16)
        out = torch.empty((1, 3, 16, 16), device=dev)
        fn = R._render_frame_fn()
        args = (16, xyz.data_ptr(), 1, chol.data_ptr(), bound.data_ptr(), feat.data_ptr(),
                rgbw.data_ptr(), 0, bg.data_ptr(), 16, 16)
        t0 = time.perf_counter()
        for i in range(a.calls):
            fn(*args, fw.frame + i, 0, fw.meta_ptr, fw.buf_ptr, fw.buf.numel(), out.data_ptr(),
               fw.stream)
        t_c = (time.perf_counter() - t0) / a.calls
        torch.cuda.synchronize()
        fw.dirty = True
    print(json.dumps(dict(splats=a.splats, enqueue_us=round(1e6 * t_enq, 2),
                          tiny_model_call_us=round(1e6 * t_tiny_model, 2),
                          tiny_render_frame_sum_us=round(1e6 * t_tiny_render, 2),
                          bare_c_call_us=round(1e6 * t_c, 2),
                          per_frame_us=round(1e6 * t_all, 2), current_stream_us=round(1e6 * t_stream, 2),
                          torch_empty_us=round(1e6 * t_empty, 2), ctypes_call_us=round(1e6 * t_ctypes, 2))))


if __name__ == "__main__":
    main()
