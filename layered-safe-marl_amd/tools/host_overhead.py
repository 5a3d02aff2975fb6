"""DIAGNOSTIC: host-side cost of one GpuGraphVecEnv.step_async + step_wait at config 3 (4096 envs,
filter on), and the idle time in front of the first launch of a window (what a 20-step driver window
pays once): (1) host microseconds per call with the launch queue deep; (2) event time of one step
launched onto an idle GPU, minus the kernel's own time from a back-to-back run.

    python layered-safe-marl_amd/tools/host_overhead.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import torch
    import bench
    from lsm import hj_tables
    from lsm.vec_env import GpuGraphVecEnv
    c = bench.CONFIGS[3]
    args = bench.make_args(c)
    vt, _ = hj_tables.default_tables("double_integrator")
    env = GpuGraphVecEnv(args, num_envs=c["envs"], device="cuda:0", value_table=vt, return_numpy=False,
                         build_infos=False)
    env.reset(4)
    acts = torch.randint(0, 25, (c["envs"], c["num_agents"]), device="cuda:0", dtype=torch.int32)
    for _ in range(20):
        env.step_async(acts, 4)
        env.step_wait()
    torch.cuda.synchronize()
    # (1) host time per call, queue deep (the GPU is the slower side)
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        env.step_async(acts, 4)
        env.step_wait()
    host_us = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    # back-to-back kernel time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        env.step_async(acts, 4)
    e1.record()
    torch.cuda.synchronize()
    b2b_us = e0.elapsed_time(e1) / n * 1e3
    # (2) one step onto an idle GPU: event time from a marker recorded just before the call
    one = []
    for _ in range(50):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        env.step_async(acts, 4)
        b.record()
        torch.cuda.synchronize()
        one.append(a.elapsed_time(b) * 1e3)
    one.sort()
    # (3) the host cost of each part of step_async (no launch): curriculum lookup, action tensor,
    # stream handle
    t0 = time.perf_counter()
    for _ in range(2000):
        env._curriculum(4)
    cur_us = (time.perf_counter() - t0) / 2000 * 1e6
    t0 = time.perf_counter()
    for _ in range(2000):
        env._actions_device(acts)
    act_us = (time.perf_counter() - t0) / 2000 * 1e6
    t0 = time.perf_counter()
    for _ in range(2000):
        env._stream()
    st_us = (time.perf_counter() - t0) / 2000 * 1e6
    print(json.dumps({"host_us_per_step_queue_deep": host_us, "kernel_us_back_to_back": b2b_us,
                      "idle_gpu_one_step_event_us_median": one[len(one) // 2], "min": one[0],
                      "front_latency_us_median": one[len(one) // 2] - b2b_us,
                      "host_us_curriculum": cur_us, "host_us_actions": act_us, "host_us_stream": st_us}))
    env.close()


if __name__ == "__main__":
    main()
