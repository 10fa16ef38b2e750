"""The N > 1 path on CPU with gloo (world size 2): GOP sharding, the metric
all-reduce of SURVEY §8e, and bench.py's max-over-ranks timing reduction."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from gsvc_amd.shard import aggregate_video_metrics, forced_k_frames, gops, shard_gops  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gops_and_shards():
    g = gops([1, 5, 9, 30], 40)
    assert g == [(1, 5), (5, 9), (9, 30), (30, 41)]
    for world in (1, 2, 3, 4, 8):
        sh = shard_gops([1, 5, 9, 13, 20, 27, 33, 38], 40, world)
        flat = [x for r in sh for x in r]
        assert flat == gops([1, 5, 9, 13, 20, 27, 33, 38], 40)  # contiguous, in order, complete
        if world <= 8:
            assert all(sh[r] for r in range(world))  # every rank busy
    # 600 frames, 8 ranks, forced K-frames give 8 equal shards
    k = forced_k_frames(600, 8)
    sh = shard_gops(k, 600, 8)
    assert [sum(e - s for s, e in r) for r in sh] == [75] * 8


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r "trained" frames with PSNR 30 + frame index
        frames = [f for f in range(10) if f % world == rank]
        per = {"psnr": [30.0 + f for f in frames], "num_gaussians": [50000.0] * len(frames)}
        agg = aggregate_video_metrics(per)
        import bench
        mx = bench.all_max(float(rank + 1) * 0.5, world, torch.device("cpu"))
        q.put((rank, agg, mx))
    finally:
        dist.destroy_process_group()


def test_allreduce_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, agg, mx in res:
        assert agg["frames"] == 10
        assert agg["psnr"] == pytest.approx(30.0 + 4.5)
        assert agg["num_gaussians"] == pytest.approx(50000.0)
        assert mx == pytest.approx(1.0)
