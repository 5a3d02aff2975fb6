"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path: env sharding and the
episode-summary collective (lsm/dist.py), the only cross-rank exchange of the rollout."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "layered-safe-marl_amd"))

from lsm import dist as ldist  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_eps(n_global, seed=3):
    rng = np.random.default_rng(seed)
    ep = rng.uniform(0, 10, (n_global, 8))
    ep[:, 6] = rng.uniform(0.1, 4.0, n_global)
    return ep


def _worker(rank, world, port, n_global, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, lr = ldist.rank_info()
    assert (r, w, lr) == (rank, world, rank)
    off, n = ldist.shard(n_global, rank, world)
    ep = torch.tensor(_global_eps(n_global)[off:off + n], dtype=torch.float64)
    summ = ldist.global_episode_summary(ep)
    if rank == 0:
        np.save(out_path, np.array([summ[k] for k in ldist.EPKEYS]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_global", [10, 4096 * 2 + 3])
def test_episode_summary_world2_matches_single_process(tmp_path, n_global):
    out = str(tmp_path / "summ.npy")
    torch.multiprocessing.spawn(_worker, args=(2, _free_port(), n_global, out), nprocs=2, join=True)
    got = np.load(out)
    ep = _global_eps(n_global)
    want = ep.mean(axis=0)
    want[6] = ep[:, 6].min()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)


def test_shard_covers_all_envs_once():
    for n_global in (1, 7, 4096, 8192 + 5):
        for world in (1, 2, 3, 8):
            if n_global < world:
                continue
            seen = []
            for r in range(world):
                off, n = ldist.shard(n_global, r, world)
                seen.extend(range(off, off + n))
            assert seen == list(range(n_global))


def test_single_process_summary_without_init():
    ep = torch.tensor(_global_eps(33), dtype=torch.float64)
    s = ldist.global_episode_summary(ep)
    np.testing.assert_allclose([s[k] for k in ldist.EPKEYS][:6], ep.numpy().mean(axis=0)[:6], rtol=1e-12)
    assert s["min_distance_min"] == float(ep[:, 6].min())


def test_sharded_oracle_envs_equal_global_envs():
    """Rank r's envs (env_offset = r * n) are the global envs [r*n, (r+1)*n): same seeds, same
    trajectories (the kernel uses the same seed rule, checked on the GPU in test_gpu_parity)."""
    sys.path.insert(0, os.path.dirname(HERE))
    from oracle.lsm_oracle import OracleVecEnv
    meta = dict(dynamics_type="double_integrator", num_agents=3, num_landmarks=2, world_size=4,
                episode_length=20, num_env_steps=20 * 4, n_rollout_threads=1, use_safety_filter=False,
                use_masking=True, num_internal_step=1)
    full = OracleVecEnv(meta, 4, seed=11, integrator="closed")
    parts = [OracleVecEnv(meta, 2, seed=11, integrator="closed", seed_offset=off) for off in (0, 2)]
    full.reset(2)
    for p in parts:
        p.reset(2)
    rng = np.random.default_rng(0)
    for _ in range(25):
        a = rng.integers(0, 25, (4, 3))
        g = full.step(a, 2)
        r0 = parts[0].step(a[:2], 2)
        r1 = parts[1].step(a[2:], 2)
        np.testing.assert_array_equal(g[0], np.concatenate([r0[0], r1[0]]))
        np.testing.assert_array_equal(g[4], np.concatenate([r0[4], r1[4]]))
