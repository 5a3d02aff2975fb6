"""Multi-GPU sharding of environments + the one collective the path has.

Envs are embarrassingly parallel: rank r owns the contiguous
block of global env indices ``[r * n_local, (r + 1) * n_local)`` (env k seeded
``seed + 1000 k``, ``env_offset`` in the C ABI) with its own copy of the
read-only HJ/TTR tables. There is no per-step communication.

The only cross-GPU exchange is the episode summary the runner logs
(``GMPERunner.parse_episode_info``, graph_mpe_runner.py:222-251: mean over
threads of seven fields, min of ``min_distance_min``): one ``all_reduce(SUM)`` of
a 9-float vector and one ``all_reduce(MIN)`` per episode boundary, over RCCL
(backend "nccl") on MI355X, gloo in the CPU tests.
"""
from __future__ import annotations

import os

import torch

EPKEYS = ("travel_time_mean", "travel_distance_mean", "done_percentage", "num_reached_goal_mean",
          "conflict_percentage", "min_distance_mean", "min_distance_min", "multiple_engagement_percentage")


def rank_info():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard(n_global: int, rank: int, world: int):
    """(env_offset, n_local) of a rank; the remainder goes to the first ranks."""
    base, rem = divmod(n_global, world)
    n_local = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, n_local


def global_episode_summary(ep_info: torch.Tensor, group=None) -> dict:
    """All-rank episode summary from each rank's [n_local, 8] float64 ep_info tensor."""
    import torch.distributed as dist
    s = ep_info.sum(dim=0)
    cnt = torch.tensor([float(ep_info.shape[0])], dtype=ep_info.dtype, device=ep_info.device)
    buf = torch.cat([s, cnt])
    mn = ep_info[:, 6].min().reshape(1).clone()
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
    mean = (buf[:8] / buf[8]).tolist()
    out = dict(zip(EPKEYS, mean))
    out["min_distance_min"] = float(mn.item())
    return out
