"""Frame sharding across ranks and the one collective of the path.

Frames of a video are independent for rendering; for training, the P-frame
chain is serial inside a GOP (the run of frames from one K-frame to the next,
train_video_Represent.py:358-367), so a rank takes whole contiguous GOPs.  The
only exchange is the final metric aggregate: one all_reduce(SUM) of the
per-rank sums behind train_video_Represent.py:389-394's averages (average PSNR
is the mean of per-frame PSNRs, not the PSNR of the mean MSE).  It is ~56 bytes:
latency-bound, so xGMI bandwidth is irrelevant.  Backend: "nccl" (RCCL) on the
GPU box, "gloo" in the CPU tests.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch

METRICS = ("psnr", "ms_ssim", "training_time", "eval_time", "eval_fps", "num_gaussians")


def gops(k_frames: Sequence[int], num_frames: int) -> List[Tuple[int, int]]:
    """GOPs as half-open 1-based frame ranges [start, end) from the K-frame list
    (K_frames.txt, train_video_Represent.py:312-356; frame 1 is always a K-frame)."""
    ks = sorted({int(k) for k in k_frames if 1 <= int(k) <= num_frames} | {1})
    return [(k, (ks[i + 1] if i + 1 < len(ks) else num_frames + 1)) for i, k in enumerate(ks)]


def shard_gops(k_frames: Sequence[int], num_frames: int, world: int) -> List[List[Tuple[int, int]]]:
    """Contiguous GOP ranges per rank, balanced by frame count (greedy: a rank
    takes GOPs until it reaches its share of the remaining frames).  Ranks
    beyond the number of GOPs get nothing; SURVEY §8e adds forced K-frames at
    shard boundaries (written to K_frames.txt) when there are too few GOPs."""
    if world < 1:
        raise ValueError("world must be >= 1")
    g = gops(k_frames, num_frames)
    out: List[List[Tuple[int, int]]] = [[] for _ in range(world)]
    i = 0
    for r in range(world):
        left_frames = sum(e - s for s, e in g[i:])
        left_ranks = world - r
        share = left_frames / left_ranks if left_ranks else 0
        taken = 0
        while i < len(g):
            size = g[i][1] - g[i][0]
            # leave at least one GOP for every remaining rank when possible
            if out[r] and (taken + size / 2 > share or len(g) - i <= left_ranks - 1):
                break
            out[r].append(g[i])
            taken += size
            i += 1
    if i < len(g):
        out[-1].extend(g[i:])
    return out


def forced_k_frames(num_frames: int, world: int) -> List[int]:
    """K-frames at equal-frame shard boundaries (1-based) for when a video has
    fewer GOPs than ranks."""
    return sorted({1 + (num_frames * r) // world for r in range(world)})


def aggregate_video_metrics(per_frame: Dict[str, Sequence[float]], device=None,
                            group=None) -> Dict[str, float]:
    """Means over all frames of all ranks of the metric lists this rank
    produced (keys from METRICS; missing keys count as 0).  One all_reduce."""
    import torch.distributed as dist
    n = len(next(iter(per_frame.values()))) if per_frame else 0
    sums = [float(sum(per_frame.get(k, ()))) for k in METRICS] + [float(n)]
    t = torch.tensor(sums, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    total = float(t[-1])
    return {k: (float(t[i]) / total if total else float("nan")) for i, k in enumerate(METRICS)} | {
        "frames": int(total)}
