"""Device time of lsm_episode_summary (lsm_metrics.hip) at the bench's 4096 envs: back-to-back
launches on an idle stream, and one launch right behind a rollout step (as at an episode boundary),
HIP events around each.

    python layered-safe-marl_amd/tools/summary_time.py [--envs 4096]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    a = ap.parse_args()
    import torch
    from lsm import capi, hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    lib = capi.load_library()
    st = torch.cuda.current_stream().cuda_stream
    ep = torch.rand((a.envs, 8), dtype=torch.float64, device="cuda:0")
    out = torch.empty(10, dtype=torch.float64, device="cuda:0")
    call = lambda t: lib.lsm_episode_summary(C.c_void_p(t.data_ptr()), a.envs, C.c_void_p(out.data_ptr()), C.c_void_p(st))
    for _ in range(10):
        call(ep)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(100):
        call(ep)
    e1.record()
    torch.cuda.synchronize()
    idle_us = e0.elapsed_time(e1) * 10.0
    args = EnvArgs(num_agents=8, num_env_steps=250 * 4, use_safety_filter=True, seed=0)
    vt, _ = hj_tables.default_tables("double_integrator")
    env = GpuGraphVecEnv(args, num_envs=a.envs, device="cuda:0", value_table=vt, return_numpy=False)
    env.reset(4)
    acts = torch.randint(0, 25, (a.envs, 8), device="cuda:0", dtype=torch.int32)
    after = []
    for _ in range(20):
        env.step_async(acts, 4)
        env.step_wait()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        call(env.t_epinfo)
        s1.record()
        torch.cuda.synchronize()
        after.append(s0.elapsed_time(s1) * 1e3)
    after.sort()
    print(json.dumps({"envs": a.envs, "us_per_launch_back_to_back": idle_us,
                      "us_after_a_step_median": after[len(after) // 2], "us_after_a_step_min": after[0]}))
    env.close()


if __name__ == "__main__":
    main()
