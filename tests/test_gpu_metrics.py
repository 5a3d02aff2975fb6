"""Runner metrics on the device against the oracle's info dicts.

The kernel's info tensor [n][N][LSM_INFO_FIELDS] after each step goes through
``lsm.metrics.process_infos`` / ``log_means``; the oracle's per-agent info dicts (the reference's
``info_callback`` + ``individual_reward``, oracle/lsm_oracle.py ``info``) go through the
restatement of ``BaseRunner.process_infos`` (onpolicy/runner/shared/base_runner.py:222-301) and
``log_env``'s ``np.mean`` (:317-331). Same keys, same list lengths, values within the info
tolerance (rtol 1e-9; individual rewards as rewards, 1e-5), across auto-resets.
"""
import numpy as np
import pytest

from golden_replay import table_dict
from test_metrics import _reference_process_infos

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dyn,n_agents,filt", [("double_integrator", 8, True), ("airtaxi", 6, True),
                                               ("double_integrator", 5, False)])
def test_gpu_metrics_match_reference_restatement(dyn, n_agents, filt):
    import torch
    from lsm import metrics
    from lsm.config import EnvArgs
    from lsm.hj_tables import default_tables
    from lsm.vec_env import GpuGraphVecEnv
    from oracle.lsm_oracle import OracleVecEnv
    ws, epl = (4, 40) if dyn == "double_integrator" else (6, 40)
    dt = 0.1 if dyn == "double_integrator" else 1.0
    args = EnvArgs(dynamics_type=dyn, num_agents=n_agents, world_size=ws, episode_length=epl,
                   num_env_steps=epl * 4, use_safety_filter=filt, seed=13)
    n = 12
    vt, tt = default_tables(dyn, small=True)
    env = GpuGraphVecEnv(args, num_envs=n, device="cuda:0", value_table=vt if filt else None, ttr_table=tt,
                         return_numpy=False)
    ora = OracleVecEnv(vars(args), n, seed=13, value_table=table_dict(vt) if filt else None,
                       ttr_table=table_dict(tt), integrator="restated")
    env.reset(4)
    ora.reset(4)
    rng = np.random.default_rng(3)
    for t in range(int(1.5 * epl)):
        a = rng.integers(0, 25, (n, n_agents))
        env.step(a, 4)
        _, _, _, _, _, _, oinfos = ora.step(a, 4)
        ref = _reference_process_infos(oinfos, n_agents, epl, dt)
        got = metrics.process_infos(env.t_info, n_agents, epl, dt)
        assert set(got) == set(ref)
        for k, v in ref.items():
            assert len(got[k]) == len(v), k
            tol = 1e-5 if k.endswith("individual_rewards") else 1e-9
            np.testing.assert_allclose(got[k], v, rtol=tol, atol=tol, err_msg="step %d %s" % (t, k))
        means = metrics.log_means(env.t_info, n_agents, epl, dt)
        for k, v in ref.items():
            if not v:
                assert k not in means
                continue
            tol = 1e-5 if k.endswith("individual_rewards") else 1e-9
            np.testing.assert_allclose(means[k], np.mean(v), rtol=tol, atol=tol, err_msg="step %d %s" % (t, k))
    assert isinstance(env.t_info, torch.Tensor) and env.t_info.is_cuda
    env.close()


@pytest.mark.parametrize("n", [0, 1, 255, 4096, 8195])
def test_gpu_episode_summary_kernel(n):
    """lsm_episode_summary (one launch, no host sync) equals the column sums, the count and the
    NaN-propagating min of min_distance_min that GMPERunner's parse reduces (graph_mpe_runner.py:
    222-251); EpisodeSummaryReducer's means equal numpy's."""
    import ctypes as C
    import torch
    from lsm import capi
    from lsm.dist import EPKEYS, EpisodeSummaryReducer
    lib = capi.load_library()
    rng = np.random.default_rng(n)
    ep = rng.uniform(-3, 10, (n, 8))
    ep[:, 6] = rng.uniform(0.01, 4.0, n)
    t = torch.tensor(ep, dtype=torch.float64, device="cuda:0")
    out = torch.full((10,), -7.0, dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    assert lib.lsm_episode_summary(C.c_void_p(t.data_ptr()), n, C.c_void_p(out.data_ptr()), C.c_void_p(st)) == 0
    o = out.cpu().numpy()
    np.testing.assert_allclose(o[:8], ep.sum(axis=0), rtol=1e-13, atol=1e-12)
    assert o[8] == n
    assert o[9] == (ep[:, 6].min() if n else np.inf)
    if n:
        r = EpisodeSummaryReducer(n, "cuda:0")
        r.submit(t)
        r.submit(t)
        got = r.results()
        assert len(got) == 2 and got[0] == got[1]
        want = ep.mean(axis=0)
        want[6] = ep[:, 6].min()
        np.testing.assert_allclose([got[0][k] for k in EPKEYS], want, rtol=1e-12, atol=1e-12)
        ep[n // 2, 6] = np.nan
        t = torch.tensor(ep, dtype=torch.float64, device="cuda:0")
        lib.lsm_episode_summary(C.c_void_p(t.data_ptr()), n, C.c_void_p(out.data_ptr()), C.c_void_p(st))
        assert np.isnan(out[9].item())


def test_gpu_metrics_match_reference_runner_functions():
    """Pinned to the reference's own functions: tests/golden/runner_metrics.npz holds what
    Runner.process_infos / log_env (base_runner.py:222-331) returned on K reference envs
    (make_runner_metrics.py). A device handle with the same seeds and actions, through
    lsm.metrics on its info tensor, gives the same per-env lists and log means every step across
    the auto-reset (rtol 1e-9; individual rewards -- float32 outputs -- 1e-5)."""
    import ast
    import os
    from golden_replay import tables_for
    from lsm import metrics
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runner_metrics.npz"))
    m = ast.literal_eval(str(z["meta"]))
    vt, _ = tables_for(m)
    args = EnvArgs(dynamics_type=m["dynamics_type"], num_agents=m["num_agents"], world_size=m["world_size"],
                   episode_length=m["episode_length"], num_env_steps=m["num_env_steps"], use_safety_filter=True,
                   seed=m["seed"])
    env = GpuGraphVecEnv(args, num_envs=m["n_envs"], device="cuda:0", value_table=vt, return_numpy=False)
    env.reset(m["ep"])
    keys = [str(k) for k in z["keys"]]
    log_keys = [str(k) for k in z["log_keys"]]
    N, L, dt = m["num_agents"], m["episode_length"], m["dt"]
    for t in range(len(z["act"])):
        env.step(z["act"][t], m["ep"])
        got = metrics.process_infos(env.t_info, N, L, dt)
        assert sorted(got) == keys
        means = metrics.log_means(env.t_info, N, L, dt)
        assert sorted(means) == log_keys
        for i, k in enumerate(keys):
            want = z["vals"][t, i, :int(z["lens"][i])]
            tol = 1e-5 if k.endswith("individual_rewards") else 1e-9
            np.testing.assert_allclose(got[k], want, rtol=tol, atol=tol, err_msg="step %d %s" % (t, k))
        for j, k in enumerate(log_keys):
            tol = 1e-5 if k.endswith("individual_rewards") else 1e-9
            np.testing.assert_allclose(means[k], z["log_vals"][t, j], rtol=tol, atol=tol, err_msg="step %d %s" % (t, k))
    env.close()
