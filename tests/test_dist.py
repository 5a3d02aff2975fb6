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


def test_init_rank_binds_the_device_before_the_process_group(monkeypatch):
    """RCCL rank setup (bench.py, INTEGRATION.md factory): torch.cuda.set_device(local_rank) comes
    BEFORE init_process_group, which gets the same device as device_id, and barriers name it; a
    communicator created first would bind every rank to GPU 0."""
    import torch.distributed as dist
    calls = []
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls.append(("set_device", str(d))))
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 1)
    state = {"init": False}
    monkeypatch.setattr(dist, "is_initialized", lambda: state["init"])
    monkeypatch.setattr(dist, "is_available", lambda: True)

    def fake_init(backend, **kw):
        calls.append(("init_process_group", backend, str(kw.get("device_id"))))
        state["init"] = True
    monkeypatch.setattr(dist, "init_process_group", fake_init)
    monkeypatch.setattr(dist, "barrier", lambda **kw: calls.append(("barrier", kw.get("device_ids"))))
    dev = ldist.init_rank("nccl")
    ldist.barrier("nccl")
    assert str(dev) == "cuda:1"
    assert calls == [("set_device", "cuda:1"), ("init_process_group", "nccl", "cuda:1"), ("barrier", [1])]


def test_bench_uses_init_rank_and_per_rank_actions():
    """bench.py joins the process group only through lsm.dist.init_rank (device first), and each
    rank's synthetic actions are exactly its rows of the single-process draw."""
    import inspect
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    src = inspect.getsource(bench.main)
    assert "init_process_group" not in src and "init_rank(" in src
    assert src.index("init_rank(") < src.index("GpuGraphVecEnv(")
    full = bench.synthetic_actions(7, 0, 64, 8, "cpu")
    assert full.dtype == torch.int32 and int(full.min()) >= 0 and int(full.max()) < 25
    assert len(torch.unique(full)) == 25
    for r in range(4):
        np.testing.assert_array_equal(bench.synthetic_actions(7, 16 * r, 16, 8, "cpu").numpy(),
                                      full[16 * r:16 * (r + 1)].numpy())
    assert not torch.equal(bench.synthetic_actions(8, 0, 64, 8, "cpu"), full)
