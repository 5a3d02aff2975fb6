"""Host cost of one GpuGraphVecEnv.step_async + step_wait (device tensors), i.e. how far ahead of
the GPU the Python loop can enqueue. The loop runs K launches without synchronising (the launch
queue absorbs them) and reports host microseconds per call, then the GPU time per step.

    python layered-safe-marl_amd/tools/host_overhead.py [--envs 4096] [--calls 400]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--calls", type=int, default=400)
    a = ap.parse_args()
    import torch
    from lsm import hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    args = EnvArgs(num_agents=8, num_env_steps=250 * 4, use_safety_filter=True, seed=0)
    vt, _ = hj_tables.default_tables("double_integrator")
    env = GpuGraphVecEnv(args, num_envs=a.envs, device="cuda:0", value_table=vt, return_numpy=False)
    env.reset(4)
    acts = torch.randint(0, 25, (a.calls, a.envs, 8), device="cuda:0", dtype=torch.int32)
    for t in range(20):
        env.step_async(acts[t], 4)
        env.step_wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(a.calls):
        env.step_async(acts[t], 4)
        env.step_wait()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"envs": a.envs, "calls": a.calls, "host_us_per_call": (t1 - t0) * 1e6 / a.calls,
                      "wall_us_per_step": (t2 - t0) * 1e6 / a.calls}))
    env.close()


if __name__ == "__main__":
    main()
