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


def init_rank(backend: str = "nccl", device_index=None):
    """Bind this rank to its GPU, then join the process group: torch.cuda.set_device before
    init_process_group, and (RCCL) the device passed as device_id, so the communicator and every
    barrier of rank r use GPU r -- a communicator created before the device is set binds to GPU 0 on
    every rank. Returns the rank's device (None without CUDA, e.g. gloo on the CPU)."""
    import torch.distributed as dist
    _, world, local_rank = rank_info()
    dev = None
    if torch.cuda.is_available():
        dev = torch.device("cuda:%d" % (local_rank if device_index is None else device_index))
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
    return dev


def barrier(backend: str = "nccl"):
    """dist.barrier on this rank's own GPU (RCCL: device_ids = [the current device])."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    if backend == "nccl" and torch.cuda.is_available():
        dist.barrier(device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier()


def shard(n_global: int, rank: int, world: int):
    """(env_offset, n_local) of a rank; the remainder goes to the first ranks."""
    base, rem = divmod(n_global, world)
    n_local = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, n_local


def global_episode_summary(ep_info: torch.Tensor, group=None) -> dict:
    """All-rank episode summary from each rank's [n_local, 8] float64 ep_info tensor
    (synchronous: returns host floats, like the runner's parse after a rollout)."""
    r = EpisodeSummaryReducer(ep_info.shape[0], ep_info.device, group=group)
    r.submit(ep_info)
    return r.results()[0]


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


class EpisodeSummaryReducer:
    """The per-episode-boundary reduction without a host synchronisation.

    ``submit(ep_info)`` enqueues, on the current stream, the column sums and the
    ``min_distance_min`` minimum of this rank's [n_local, 8] ep_info into fresh device
    buffers and, when a process group is up, the two collectives as async work (RCCL runs
    them stream-ordered after the sums; nothing waits on the host). ``results()`` waits
    for everything submitted and returns one dict per boundary. The reference runner
    likewise parses episode info once per episode, after the rollout
    (graph_mpe_runner.py:155-162), not inside the step loop."""

    def __init__(self, n_local: int, device, group=None):
        self.group = group
        self.device = torch.device(device)
        # the env count rides in the SUM buffer (one collective gives sums and the global count);
        # it is the row count of each submitted ep_info (n_local for the rollout's LSM_OUT_EP_INFO)
        self.n_local = int(n_local)
        self._pending = []
        self._free = []   # output buffers of read results, reused by later submits
        self._fn = None   # lsm_episode_summary, resolved once

    def _summary_fn(self):
        if self._fn is None:
            from . import capi
            lib = capi.load_library()
            if getattr(lib, "lsm_episode_summary", None) is None:
                raise capi.LsmError("%s lacks lsm_episode_summary (a library older than lsm_metrics.hip)"
                                    % capi.LIB_PATH)
            self._fn = lib.lsm_episode_summary
        return self._fn

    def submit(self, ep_info: torch.Tensor):
        # at an episode boundary inside a timed loop the host work is one ctypes launch: the
        # output buffer comes from the pool once a previous result has been read
        out = self._free.pop() if self._free and self._free[-1].device == ep_info.device else \
            torch.empty(10, dtype=torch.float64, device=ep_info.device)
        if ep_info.is_cuda:
            # one native launch (lsm_metrics.hip): sums, count, min -- no host sync
            import ctypes as C
            from . import capi
            ep = ep_info if ep_info.is_contiguous() else ep_info.contiguous()
            st = torch.cuda.current_stream(ep.device).cuda_stream
            if self._summary_fn()(C.c_void_p(ep.data_ptr()), int(ep.shape[0]), C.c_void_p(out.data_ptr()),
                                  C.c_void_p(st)) != 0:
                raise capi.LsmError("lsm_episode_summary failed")
        else:   # host tensors (gloo tests on the CPU): the same sums with torch
            torch.sum(ep_info, dim=0, out=out[:8])
            out[8] = float(ep_info.shape[0])   # the rows submitted, as the device path counts them
            out[9:10] = torch.amin(ep_info[:, 6:7], dim=0)
        buf, mn = out[:9], out[9:10]
        works = ()
        if _dist_on():
            import torch.distributed as dist
            works = (dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True),
                     dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=self.group, async_op=True))
        self._pending.append((out, buf, mn, works))

    def results(self):
        out = []
        for full, buf, mn, works in self._pending:
            for w in works:
                w.wait()
            mean = (buf[:8] / buf[8]).tolist()
            d = dict(zip(EPKEYS, mean))
            d["min_distance_min"] = float(mn.item())
            out.append(d)
            self._free.append(full)
        self._pending = []
        return out
