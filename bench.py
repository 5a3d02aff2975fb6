#!/usr/bin/env python
"""Benchmark: agent-env-steps/s of the navigation_graph_safe rollout on MI355X.

A "step" = one vec-env step (one rollout_kernel launch) over this GPU's batch of
envs, including device auto-resets at episode ends, with actions drawn on device.
Default workload = BASELINE.json configs[2] (the headline metric's config): double
integrator, 8 agents x 4096 envs per GPU, HJ safety filter on, reference output
layout (per-ego node_obs / adjacency). Multi-GPU: one process per GPU (torchrun),
envs sharded by global index (weak scaling), RCCL all_reduce of the episode
summary at each episode boundary, max-over-ranks timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

--gpus N > 1 starts N rank processes itself (or runs under torchrun, WORLD_SIZE = N). The timed
window always straddles an episode boundary (auto-reset launch + RCCL episode summary): the
untimed steps before it are at least --warmup, padded to that phase ("warmup" in the line is the
count actually run).
"""
from __future__ import annotations

import argparse
import json
import math
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "layered-safe-marl_amd"))

METRIC = "agent-env-steps/sec at 8 agents × 4096 envs, safety filter on; 1/2/4/8 GPU"
PEAK_HBM_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    2: dict(workload="8-agent double-integrator, 4096 envs per GPU, safety filter off",
            dynamics_type="double_integrator", num_agents=8, envs=4096, use_safety_filter=False,
            world_size=4, episode_length=250),
    3: dict(workload="8-agent double-integrator, 4096 envs per GPU, HJ safety filter on",
            dynamics_type="double_integrator", num_agents=8, envs=4096, use_safety_filter=True,
            world_size=4, episode_length=250),
    4: dict(workload="16-agent airtaxi (Dubins), 8192 envs per GPU, HJ safety filter on",
            dynamics_type="airtaxi", num_agents=16, envs=8192, use_safety_filter=True,
            world_size=6, episode_length=350),
    5: dict(workload="64-agent double-integrator, 8192 envs per GPU (65536 over 8 GPUs), HJ safety filter "
                     "on, compact adjacency", dynamics_type="double_integrator", num_agents=64, envs=8192,
            use_safety_filter=True, world_size=4, episode_length=250, adj_layout="compact",
            cpu_sample=(1, 30)),   # the oracle takes ~0.5 s per 64-agent env-step: 1 env x 30 steps per core
}


def make_args(c, seed=0):
    from lsm.config import EnvArgs
    return EnvArgs(dynamics_type=c["dynamics_type"], num_agents=c["num_agents"], num_landmarks=2,
                   world_size=c["world_size"], episode_length=c["episode_length"],
                   num_env_steps=c["episode_length"] * 4, n_rollout_threads=1,
                   use_safety_filter=c["use_safety_filter"], seed=seed)


# ---- CPU baseline: the oracle ("port") on the host cores, bounded sample --------------------
_CPU_CTX = {}


def _cpu_worker(k):
    from oracle.lsm_oracle import OracleVecEnv
    import numpy as np
    c = _CPU_CTX
    ora = OracleVecEnv(vars(c["args"]), c["envs_per_worker"], seed=0, value_table=c["vt"], ttr_table=c["tt"],
                       integrator="rk45", seed_offset=k * c["envs_per_worker"])
    ora.reset(c["ep"])
    rng = np.random.default_rng(1 + k)
    N = c["args"].num_agents
    t0 = time.perf_counter()
    for _ in range(c["steps"]):
        ora.step(rng.integers(0, 25, (c["envs_per_worker"], N)), c["ep"])
    return time.perf_counter() - t0


def cpu_baseline(args, vt, tt, ep, cores, envs_per_worker=4, steps=500):
    _CPU_CTX.update(args=args, vt=vt, tt=tt, ep=ep, envs_per_worker=envs_per_worker, steps=steps)
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        times = pool.map(_cpu_worker, range(cores))
    agent_steps = cores * envs_per_worker * steps * args.num_agents
    return dict(value=agent_steps / max(times), unit="agent-steps/s", cores=cores, kind="port",
                sample="oracle/lsm_oracle.py (reference semantics, scipy RK45), %d worker processes x %d envs x "
                       "%d steps, N=%d, filter %s, full-size synthetic HJ table; wall %.1f s"
                       % (cores, envs_per_worker, steps, args.num_agents,
                          "on" if args.use_safety_filter else "off", max(times)))


def table_dict(t):
    if t is None:
        return None
    return dict(lo=t.lo, hi=t.hi, shape=t.shape, periodic=t.periodic, values_hj=t.values_hj,
                grads_hj=t.grads_hj, separation_distance=t.separation_distance, values=t.values_hj,
                ttr_max=t.ttr_max)


def load_traffic(config, n_envs, build_id):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of the same workload, and only
    if it was collected on this library build (lsm_build_id); None otherwise."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        e = d.get("config%d" % config)
        if e and int(e.get("num_envs", -1)) == n_envs and e.get("build_id") == build_id:
            return float(e["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def bench_edges(env, dev, step_fn, reps=50):
    """process_adj (gnn.py:376-407) over this GPU's n*N per-ego graphs, two ways, on the same adjacency:
    "count_pass": count kernel + hipcub scan + emit kernel (the adjacency read twice: the emit pass
    re-reads it from beyond L2, profiles/r05_s42_edges_traffic.txt);
    "one_pass": the step kernel also wrote each graph's nonzeros (LSM_OUT_ADJ_NNZ), and the call is
    scan + emit (lsm_edges_scan_emit), the adjacency read once. step_fn(k) runs k more env steps with
    pre-drawn actions (returns their event-timed ms per step); the step time with and without the counts
    bound is measured alternately (what the counts cost the step). Algorithmic bytes: adjacency reads
    (+ mask words, compact) + counts / offsets + 16 B edge_index + 4 B edge_attr per edge. Each call
    includes its one D2H read of nnz, the torch.nonzero sync."""
    import ctypes as C
    import torch
    from lsm import capi, edges
    E, N = env.E, env.N
    # at config 5 all 8192 x 64 per-ego graphs would be ~12 G edges (200 GiB): time the envs whose
    # worst-case edge list fits 16 GiB, as a learner consuming minibatches would
    m = max(1, min(env.num_envs, (16 << 30) // (N * E * E * 20)))
    compact = env.t_adj_mask is not None
    B = m * N
    W = (E + 63) // 64
    adj_read = B * (E * E * 4 + (W * 8 if compact else 0))   # per ego graph (compact: its env's table + mask)

    def run(counts):
        if not compact:
            return edges.process_adj(env.t_adj[:m].reshape(-1, E, E), counts=counts)
        return edges.process_adj_compact(env.t_adj[:m], env.t_adj_mask[:m], N, counts=counts)

    def timed(counts):
        ei, ea = run(counts)                          # warm-up, allocates, loads kernels
        nnz = ei.shape[1]
        del ei, ea
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run(counts)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps, nnz

    out = {"op": "GNNBase.process_adj (gnn.py:376-407) on the device", "envs": m, "graphs": B, "E": E}
    one = not env.kernel_name.startswith("rollout_block_kernel")   # LSM_OUT_ADJ_NNZ: E <= 64 kernels
    cnt = torch.zeros((env.num_envs, N), dtype=torch.int64, device=dev)

    def bind(t):
        capi.check(env.lib.lsm_bind_output(env.h, capi.OUT_ADJ_NNZ, C.c_void_p(t.data_ptr() if t is not None else 0),
                                           t.numel() * 8 if t is not None else 0), env.h)

    step_ms = {"with_counts": [], "without": []}
    if one:
        for _ in range(3):
            for key, t in (("without", None), ("with_counts", cnt)):
                bind(t)
                step_fn(5)
                step_ms[key].append(step_fn(50))
        # the last steps ran with the counts bound: cnt belongs to the current adjacency
    ms, nnz = timed(None)
    read = 2 * adj_read
    written = nnz * 20 + (B + 2) * 8 + B * 8
    out["count_pass"] = {"ms_per_call": ms, "nnz": nnz, "algorithmic_bytes": read + written,
                         "achieved_GBps": (read + written) / (ms * 1e-3) / 1e9,
                         "frac_hbm_peak": (read + written) / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS,
                         "note": "count + scan + emit: the adjacency read twice (both reads counted)"}
    if not one:
        out["one_pass"] = None
        return out
    ms1, nnz1 = timed(cnt[:m].reshape(-1))
    bind(None)
    assert nnz1 == nnz
    read1 = adj_read + B * 8
    written1 = nnz1 * 20 + (B + 2) * 8
    out["one_pass"] = {"ms_per_call": ms1, "nnz": nnz1, "algorithmic_bytes": read1 + written1,
                       "achieved_GBps": (read1 + written1) / (ms1 * 1e-3) / 1e9,
                       "frac_hbm_peak": (read1 + written1) / (ms1 * 1e-3) / 1e9 / PEAK_HBM_GBPS,
                       "step_ms_without_counts": step_ms["without"], "step_ms_with_counts": step_ms["with_counts"],
                       "note": "scan of the step kernel's per-graph counts + emit: the adjacency read once"}
    return out


def cpu_share():
    """(cores this job may use, host cores): the affinity set, capped by a cgroup CPU quota if
    one is set (a GPU box lends each GPU a share of a larger host)."""
    host = len(os.sched_getaffinity(0))
    n = host
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(period))))
    except Exception:
        pass
    return n, host


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(a):
    """--gpus N > 1 without a launcher: start N fresh rank processes (one per GPU) before this
    process touches any GPU, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, and exit with
    the worst return code. Rank 0 prints the JSON line."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


_M1, _M2, _GOLD = -4658895280553007687, -7723592293110705685, -7046029254386353131   # splitmix64 constants


def _mix64(x):
    """splitmix64's finaliser on int64 tensors (wrapping multiplies; logical shifts by masking)."""
    x = x ^ ((x >> 30) & 0x3FFFFFFFF)
    x = x * _M1
    x = x ^ ((x >> 27) & 0x1FFFFFFFFF)
    x = x * _M2
    return x ^ ((x >> 31) & 0x1FFFFFFFF)


def synthetic_actions(t, env0, n_envs, N, device):
    """Discrete(25) action indices of step t for global envs [env0, env0 + n_envs) (int32 [n_envs, N]):
    a hash of (step, global env, agent), so any rank draws its own rows without the others'."""
    import torch
    idx = ((torch.arange(n_envs, device=device, dtype=torch.int64) + env0)[:, None] * N +
           torch.arange(N, device=device, dtype=torch.int64)[None, :])
    x = _mix64(idx * _GOLD + _mix64(torch.full_like(idx, 1234 + t)))
    return (((x >> 33) & 0x7FFFFFFF) % 25).to(torch.int32)


def parse_kernel_select(spec):
    """--kernel-select "team=2,lanes_per_env=64" -> {"team": 2, ...} (lsm_kernel_select fields, A/B runs
    only; None = the library's own choice, which every reported line uses)."""
    out = {}
    for item in filter(None, (spec or "").split(",")):
        k, _, v = item.partition("=")
        out[k.strip()] = int(v)
    return out or None


def timed_window(warmup, steps, epl):
    """Untimed steps before the timed window: at least `warmup`, and as many more as put an
    episode boundary (the auto-reset launch and the episode-summary collective) in the middle of
    the window, whatever --steps is."""
    return warmup + (epl - (warmup + steps // 2) % epl) % epl


def dry_run(a, rank, world):
    """--dry-run: the multi-rank plumbing without a GPU (gloo): ranks, env offsets, the
    episode-summary collective and the max-over-ranks timing reduction."""
    import torch
    import torch.distributed as dist
    from lsm.dist import global_episode_summary
    c = CONFIGS[a.config]
    n_envs = a.envs or c["envs"]
    if world > 1:
        from lsm.dist import init_rank
        init_rank("gloo")
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    ep = torch.arange(n_envs * 8, dtype=torch.float64).reshape(n_envs, 8) + rank * n_envs * 8
    summ = global_episode_summary(ep)
    info = torch.tensor([rank, rank * n_envs, n_envs, time.perf_counter()], dtype=torch.float64)
    if world > 1:
        allv = [torch.zeros_like(info) for _ in range(world)]
        dist.all_gather(allv, info)
        ms = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    else:
        allv, ms = [info], torch.tensor([1.0])
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "world_size": world,
                          "ranks": [{"rank": int(v[0]), "env_offset": int(v[1]), "envs": int(v[2])} for v in allv],
                          "max_over_ranks": float(ms[0]), "episode_summary": summ,
                          "untimed_steps": timed_window(a.warmup, a.steps, c["episode_length"])}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=250)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (default: config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-cores", type=int, default=0)
    ap.add_argument("--buffer", action="store_true",
                    help="step through lsm.buffer.DeviceGraphBuffer: outputs written straight into "
                         "GraphReplayBuffer-shaped rows + the insert kernel (runner hand-off included)")
    ap.add_argument("--edges", action="store_true",
                    help="also time GNNBase.process_adj (lsm_edges.hip) on the final adjacency and add an "
                         "'edges' object to the JSON line (SURVEY 8(f) row 2; not part of the step)")
    ap.add_argument("--rng", default="mt19937", choices=("mt19937", "philox"),
                    help="device reset stream: mt19937 = the reference's draws (default), philox = fast mode")
    ap.add_argument("--kernel-select", default="",
                    help="A/B runs only: lsm_kernel_select fields, e.g. team=2 (include/lsm_rollout.h)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: check the rank launch, env offsets and collectives with gloo")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="test only: gloo lets --gpus N ranks share one GPU (real device envs, CPU "
                         "collectives); the product path and every reported number use nccl (RCCL)")
    a = ap.parse_args()

    from lsm.dist import rank_info, EpisodeSummaryReducer
    launched = "WORLD_SIZE" in os.environ
    if not launched and a.gpus > 1:
        sys.exit(launch(a))
    rank, world, local_rank = rank_info()
    if world != a.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (one rank per GPU)" % (a.gpus, world))
    if a.dry_run:
        return dry_run(a, rank, world)
    c = CONFIGS[a.config]
    n_envs = a.envs or c["envs"]
    args = make_args(c)
    from lsm import hj_tables
    vt, tt = (hj_tables.default_tables(c["dynamics_type"]) if (c["use_safety_filter"] or
              c["dynamics_type"] != "double_integrator") else (None, None))
    ep = 4  # curriculum ratio 1: the filter is active when requested (SURVEY finding 5)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        share, host = cpu_share()
        cores = a.cpu_cores or share
        epw, csteps = c.get("cpu_sample", (4, 500))
        cpu = cpu_baseline(args, table_dict(vt), table_dict(tt), ep, cores, envs_per_worker=epw, steps=csteps)
        cpu["host_cores"] = host
        cpu["cpu_share"] = share

    import torch
    import torch.distributed as dist
    from lsm.dist import init_rank, barrier
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # one GPU per rank, bound BEFORE the process group (RCCL gets it as device_id): a communicator
    # created first would bind every rank to GPU 0. The test-only gloo mode may share one device.
    dev = init_rank(a.dist_backend, device_index=(local_rank % torch.cuda.device_count()
                                                  if a.dist_backend == "gloo" else local_rank))
    if world > 1 and dist.get_world_size() != a.gpus:
        raise SystemExit("%s world size %d != --gpus %d" % (a.dist_backend, dist.get_world_size(), a.gpus))
    from lsm.vec_env import GpuGraphVecEnv
    layout = c.get("adj_layout", "reference")
    env = GpuGraphVecEnv(args, num_envs=n_envs, device=dev, value_table=vt, ttr_table=tt,
                         env_offset=rank * n_envs, return_numpy=False, build_infos=False, adj_layout=layout,
                         rng=a.rng, kernel_select=parse_kernel_select(a.kernel_select))
    N = c["num_agents"]
    epl = c["episode_length"]
    pre = timed_window(a.warmup, a.steps, epl)
    # Synthetic policy: every step's discrete actions drawn up front, resident in HBM before the
    # timed region (the policy is outside the path; one env-step = one rollout_kernel launch).
    # A counter-based draw indexed by (step, global env, agent): each rank draws only its own rows,
    # and a sharded run steps exactly the envs of a single-process run.
    acts_all = torch.empty((pre + a.steps, n_envs, N), dtype=torch.int32, device=dev)
    for t in range(pre + a.steps):
        acts_all[t].copy_(synthetic_actions(t, rank * n_envs, n_envs, N, dev))
    buf = None
    if a.buffer:
        from lsm.buffer import DeviceGraphBuffer
        buf = DeviceGraphBuffer(env, episode_length=epl)
        buf.warmup(ep)
    else:
        env.reset(ep)

    # Episode boundary: the summary reduction and its RCCL collectives are enqueued without a
    # host sync (lsm.dist.EpisodeSummaryReducer); the values are read after the timed region.
    summaries = EpisodeSummaryReducer(n_envs, dev)

    def one_step(t):
        if buf is not None:
            buf.insert_step(acts_all[t], ep)
            if buf.step == 0:
                buf.after_update()
        else:
            env.step_async(acts_all[t], ep)
            env.step_wait()
        if (t + 1) % epl == 0:   # episode boundary: RCCL reduction of the episode summary
            summaries.submit(env.t_epinfo)

    summaries.submit(env.t_epinfo)   # load the reduction kernels / RCCL before any timed call
    summaries.results()
    # No Python garbage collection inside the window: a collection pass stalls the host for ~0.1 ms,
    # and with the launch queue that shallow the GPU idles (a 73 us gap in
    # profiles/r05_v3_driver_window.txt). The collection runs before the untimed steps, so the
    # memory it returns is taken up again by them, not by the window's first step.
    # (the driver's 20-step window: 7.74-7.95e8 -> 8.60-9.27e8 agent-steps/s with this ordering and the
    # events below, same session: profiles/r05_s31_*.json)
    import gc
    gc.collect()
    gc.disable()
    try:
        for t in range(pre):
            one_step(t)
        summaries.results()
    # Kernel time: HIP events on the launch stream bracketing the whole timed region (per-launch
    # event pairs would add their own GPU-side markers between back-to-back launches). Both are
    # recorded once before the window: the HIP events are created at their first record.
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        ev1.record()
        torch.cuda.synchronize()
        barrier(a.dist_backend)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record()
        for t in range(a.steps):
            one_step(pre + t)
        ev1.record()
        torch.cuda.synchronize()
        barrier(a.dist_backend)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    finally:   # an exception in the window must not leave the collector off
        gc.enable()
    kern_ms = ev0.elapsed_time(ev1) / a.steps   # includes the inter-launch gaps (conservative)
    per_rank = [elapsed * 1e3 / a.steps]
    if world > 1:
        mine = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        allt = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allt, mine)
        per_rank = [float(x[0]) * 1e3 / a.steps for x in allt]
        elapsed = max(float(x[0]) for x in allt)
        kern_ms = max(float(x[1]) for x in allt)
    ep_summaries = summaries.results()   # after the timed region: the boundary's global summary
    offsets = [rank * n_envs]
    if world > 1:
        o = torch.tensor([env.env_offset], dtype=torch.float64, device=dev)
        allo = [torch.zeros_like(o) for _ in range(world)]
        dist.all_gather(allo, o)
        offsets = [int(x.item()) for x in allo]
    total_agent_steps = world * n_envs * N * a.steps
    value = total_agent_steps / elapsed
    from lsm.perf_model import step_bytes
    sb = step_bytes(N, 2, c["dynamics_type"], c["use_safety_filter"], layout)
    bytes_launch = sb["hbm_bytes"] * n_envs
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    # (an A/B run may load an older library without lsm_build_id: tools/ab_bench.py --allow-old)
    build_id = env.lib.lsm_build_id().decode() if hasattr(env.lib, "lsm_build_id") else "unknown"
    traffic = load_traffic(a.config, n_envs, build_id)
    resets = int((pre + a.steps) // epl - pre // epl)
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "agent-steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": pre, "warmup_requested": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": c["workload"], "num_agents": N, "envs_per_gpu": n_envs,
                       "total_envs": world * n_envs, "dynamics": c["dynamics_type"],
                       "safety_filter": c["use_safety_filter"], "episode_length": epl,
                       "episode_boundaries_timed": resets,
                       "output_layout": ("reference (per-ego node_obs/adj, fp32)" if layout == "reference" else
                                         "per-ego node_obs fp32; compact adjacency (E x E fp32 + per-ego "
                                         "u64 disconnect masks, lossless)"),
                       "hj_table": "synthetic %s" % (str(vt.shape) if vt is not None else "none"),
                       "parallelism": "env-sharded dp%d" % world,
                       "reset_rng": a.rng,
                       "handoff": ("DeviceGraphBuffer rows (ring-bound outputs + insert kernel)" if a.buffer
                                   else "env output tensors")},
            "ranks": {"rccl_world_size": (dist.get_world_size() if world > 1 else 1), "ms_per_step": per_rank,
                      "env_offsets": offsets, "backend": a.dist_backend if world > 1 else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic, "traffic_unit": "HBM bytes/launch (rocprofv3 PMC of this build_id; null if none)",
                         "kernel": env.kernel_name, "build_id": build_id,
                         "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_launch,
                         "gather_bytes_per_launch": sb["gather_bytes"] * n_envs,
                         "bytes_model": "lsm/perf_model.py: record + outputs + HJ gathers (SURVEY 8(d))"},
            "cpu_baseline": cpu,
            "episode_summaries_timed": ep_summaries,
        }
        if a.edges:
            def more_steps(k):
                # the window's pre-drawn actions again (the state has moved on; the step is the same work)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for t in range(k):
                    env.step_async(acts_all[pre + t % a.steps], ep)
                    env.step_wait()
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / k
            line["edges"] = bench_edges(env, dev, more_steps)
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
