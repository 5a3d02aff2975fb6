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
