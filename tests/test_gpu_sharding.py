"""Device-side evidence for the multi-GPU partitioning.

Rank r of a sharded run owns the global envs [r n, (r + 1) n) through ``env_offset`` and seeds
env k with seed + 1000 k (MPE_env.py:56-84 with the factory's rank rule). Sharding is only
correct if a handle at offset o steps exactly the envs [o, o + n) of one big handle: checked
here bit for bit on the GPU, every output, across an auto-reset. The bench's rank plumbing
(rank processes, env offsets, the episode-summary collective, max-over-ranks timing) runs with
real device envs through the test-only gloo backend, two ranks on the one GPU of the box.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(n_envs, offset, vt):
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    args = EnvArgs(dynamics_type="double_integrator", num_agents=8, num_landmarks=2, world_size=4,
                   episode_length=250, num_env_steps=250 * 4, n_rollout_threads=1, use_safety_filter=True,
                   seed=0)
    return GpuGraphVecEnv(args, num_envs=n_envs, device="cuda:0", value_table=vt, env_offset=offset,
                          return_numpy=False)


def test_gpu_two_shards_equal_one_handle():
    """Handles at env_offset 0 and 2048 (2048 envs each) produce, bit for bit, the two halves of
    one 4096-env handle over 260 steps (auto-reset at step 250): obs, node_obs, adj, rewards,
    dones, reset flags, info, state and the episode summaries (t_epinfo)."""
    import torch
    from lsm import hj_tables
    vt, _ = hj_tables.default_tables("double_integrator")
    full = _env(4096, 0, vt)
    parts = [_env(2048, 0, vt), _env(2048, 2048, vt)]
    outs = lambda e: (e.t_obs, e.t_node, e.t_adj, e.t_rew, e.t_done, e.t_reset, e.t_info, e.t_state, e.t_epinfo)
    names = ("obs", "node_obs", "adj", "reward", "done", "reset", "info", "state", "ep_info")

    def check(ctx):
        for nm, f, a, b in zip(names, outs(full), outs(parts[0]), outs(parts[1])):
            assert torch.equal(f[:2048], a), "%s: %s differs in shard 0" % (ctx, nm)
            assert torch.equal(f[2048:], b), "%s: %s differs in shard 1" % (ctx, nm)

    full.reset(4)
    for p in parts:
        p.reset(4)
    check("reset")
    gen = torch.Generator(device="cuda:0").manual_seed(7)
    resets = 0
    for t in range(260):
        a = torch.randint(0, 25, (4096, 8), device="cuda:0", generator=gen, dtype=torch.int32)
        full.step(a, 4)
        parts[0].step(a[:2048], 4)
        parts[1].step(a[2048:], 4)
        if t % 10 == 0 or t >= 248:
            check("step %d" % t)
        resets += int(full.t_reset.sum().item()) if t in (249,) else 0
    assert resets == 4096
    for e in [full] + parts:
        e.close()


def _bench(extra, timeout=400):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5", "--no-cpu-baseline"] + extra
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_gpu_bench_two_ranks_gloo_on_one_gpu():
    """bench.py --gpus 2 with real GpuGraphVecEnvs (gloo, both ranks on cuda:0): the world size,
    the per-rank env offsets, max-over-ranks timing, and the episode summary reduced across the
    ranks equal the single-process run over the same 512 global envs (same seeds, same global
    action stream)."""
    two = _bench(["--gpus", "2", "--dist-backend", "gloo", "--envs", "256"])
    one = _bench(["--gpus", "1", "--envs", "512"])
    assert two["n_gpus"] == 2 and two["ranks"]["rccl_world_size"] == 2 and two["ranks"]["backend"] == "gloo"
    assert two["ranks"]["env_offsets"] == [0, 256]
    assert len(two["ranks"]["ms_per_step"]) == 2
    assert two["ms_per_step"] == pytest.approx(max(two["ranks"]["ms_per_step"]))
    assert two["config"]["total_envs"] == 512 and one["config"]["total_envs"] == 512
    s2, s1 = two["episode_summaries_timed"], one["episode_summaries_timed"]
    assert len(s2) == len(s1) == 1
    for k in s1[0]:
        np.testing.assert_allclose(s2[0][k], s1[0][k], rtol=1e-12, atol=1e-12, err_msg=k)
