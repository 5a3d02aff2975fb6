"""Replay-buffer hand-off (GMPERunner.warmup / insert, GraphReplayBuffer.insert / after_update):
lsm_buffer.hip + ring-bound outputs vs the numpy restatement (oracle/runner_insert.py) and vs a
plainly bound env on the same seeds. Bit-exact (rows are copies and 0/1 masks)."""
import numpy as np
import pytest

from oracle.runner_insert import insert_rows


def test_oracle_insert_rows_hand_case():
    obs = np.arange(2 * 3 * 2, dtype=np.float32).reshape(2, 3, 2)
    aid = np.tile(np.arange(3).reshape(1, 3, 1), (2, 1, 1))
    dones = np.array([[True, False, False], [True, True, True]])
    r = insert_rows(obs, aid, dones, centralized=True)
    np.testing.assert_array_equal(r["masks"][..., 0], [[0, 1, 1], [0, 0, 0]])
    np.testing.assert_array_equal(r["active_masks"][..., 0], [[0, 1, 1], [1, 1, 1]])
    assert r["share_obs"].shape == (2, 3, 6)
    np.testing.assert_array_equal(r["share_obs"][1, 2], obs[1].reshape(-1))
    np.testing.assert_array_equal(r["share_agent_id"][0, 1], [0, 1, 2])
    r = insert_rows(obs, aid, None, centralized=False)
    assert "masks" not in r and r["share_obs"].shape == (2, 3, 2)


# ---------------- GPU ----------------

def _insert_gpu(obs, dones, centralized):
    import ctypes as C
    import torch
    from lsm import capi
    lib = capi.load_library()
    n, N, OBS = obs.shape
    dev = "cuda:0"
    t_obs = torch.as_tensor(obs, device=dev)
    t_d = torch.as_tensor(dones.astype(np.uint8), device=dev) if dones is not None else None
    so = torch.full((n, N, N * OBS if centralized else OBS), -7.0, device=dev)
    aid = torch.full((n, N, 1), -7, dtype=torch.int32, device=dev)
    said = torch.full((n, N, N if centralized else 1), -7, dtype=torch.int32, device=dev)
    m = torch.full((n, N, 1), -7.0, device=dev)
    am = torch.full((n, N, 1), -7.0, device=dev)
    rc = lib.lsm_buffer_insert(C.c_void_p(t_obs.data_ptr()), C.c_void_p(t_d.data_ptr()) if t_d is not None else None,
                               n, N, OBS, int(centralized), C.c_void_p(so.data_ptr()), C.c_void_p(aid.data_ptr()),
                               C.c_void_p(said.data_ptr()), C.c_void_p(m.data_ptr()), C.c_void_p(am.data_ptr()),
                               C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.lsm_buffer_last_error()
    torch.cuda.synchronize()
    return dict(share_obs=so.cpu().numpy(), agent_id=aid.cpu().numpy(), share_agent_id=said.cpu().numpy(),
                masks=m.cpu().numpy(), active_masks=am.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("n,N,OBS", [(37, 8, 7), (5, 3, 7), (9, 16, 6), (6, 64, 7), (1, 65, 6)])
@pytest.mark.parametrize("centralized", [True, False])
def test_gpu_insert_rows(n, N, OBS, centralized):
    rng = np.random.default_rng(n * N + OBS)
    obs = rng.standard_normal((n, N, OBS)).astype(np.float32)
    dones = rng.random((n, N)) < 0.3
    dones[0] = True                       # an all-done env (active_masks back to 1)
    if n > 1:
        dones[1] = False
    aid = np.tile(np.arange(N).reshape(1, N, 1), (n, 1, 1))
    got = _insert_gpu(obs, dones, centralized)
    want = insert_rows(obs, aid, dones, centralized)
    for k, v in want.items():
        np.testing.assert_array_equal(got[k], v, err_msg=k)
    got = _insert_gpu(obs, None, centralized)   # warmup form: masks untouched
    assert (got["masks"] == -7).all()
    np.testing.assert_array_equal(got["share_obs"], want["share_obs"])


@pytest.mark.gpu
@pytest.mark.parametrize("layout,centralized", [("reference", True), ("compact", True), ("reference", False)])
def test_gpu_buffer_rollout_matches_plain_env(layout, centralized):
    """warmup + 2.5 episodes with auto-resets and after_update: the ring-bound buffer rows equal a
    plainly bound env's outputs on the same seeds and actions, and the derived rows equal the
    oracle's insert of those outputs."""
    import torch
    from lsm import hj_tables
    from lsm.buffer import DeviceGraphBuffer
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    T, n = 20, 48
    args = EnvArgs(num_agents=8, episode_length=T, num_env_steps=T * 4, use_safety_filter=True, seed=11)
    vt, _ = hj_tables.default_tables("double_integrator", small=True)
    mk = lambda: GpuGraphVecEnv(args, num_envs=n, device="cuda:0", value_table=vt, return_numpy=False,
                                build_infos=False, adj_layout=layout)
    plain, ringed = mk(), mk()
    buf = DeviceGraphBuffer(ringed, episode_length=T, use_centralized_V=centralized)
    assert buf.fused == centralized   # kernel-written rows (centralized) or the insert kernel
    plain.reset(4)
    buf.warmup(4)
    aid = np.tile(np.arange(8).reshape(1, 8, 1), (n, 1, 1))

    def rows_equal(row, dones=None):
        np.testing.assert_array_equal(buf.obs[row].cpu().numpy(), plain.t_obs.cpu().numpy())
        np.testing.assert_array_equal(buf.node_obs[row].cpu().numpy(), plain.t_node.cpu().numpy())
        np.testing.assert_array_equal(buf.adj[row].cpu().numpy(), plain.t_adj.cpu().numpy())
        if layout == "compact":
            np.testing.assert_array_equal(buf.adj_mask[row].cpu().numpy(), plain.t_adj_mask.cpu().numpy())
        want = insert_rows(plain.t_obs.cpu().numpy(), aid, dones, centralized)
        for k, v in want.items():
            np.testing.assert_array_equal(getattr(buf, k)[row].cpu().numpy(), v, err_msg=k)

    rows_equal(0)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    resets = 0
    for it in range(2 * T + T // 2):
        t = buf.step
        a = torch.randint(0, 25, (n, 8), generator=g, device="cuda:0", dtype=torch.int32)
        plain.step(a, 4)
        dones, _ = buf.insert_step(a, 4)
        d = plain.t_done.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(dones.cpu().numpy().astype(bool), d)
        np.testing.assert_array_equal(buf.rewards[t, ..., 0].cpu().numpy(), plain.t_rew.cpu().numpy())
        rows_equal(t + 1, d)
        resets += int(plain.t_reset.cpu().numpy().sum())
        if buf.step == 0:
            buf.after_update()
            rows_equal(0, d)
    assert resets > 0   # auto-resets happened inside the ring-bound run
    buf.detach()
    a = torch.randint(0, 25, (n, 8), generator=g, device="cuda:0", dtype=torch.int32)
    plain.step(a, 4)
    ringed.step(a, 4)   # plain bindings again
    np.testing.assert_array_equal(ringed.t_obs.cpu().numpy(), plain.t_obs.cpu().numpy())
    plain.close()
    ringed.close()
