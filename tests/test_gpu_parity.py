"""GPU parity tests: the HIP path (through the C ABI) vs the reference's golden vectors and
the CPU oracle. Tolerances (BASELINE.json north_star): graph edges / adjacency nonzero
pattern / done masks bit-exact; fp32 outputs within 1e-5; float64 states within 1e-9
(the kernel integrates in closed form, the reference with RK45: they differ by ~1e-16)."""
import numpy as np
import pytest

from golden_replay import EPKEYS, INFOKEYS, adj_bits, fixture_names, load, step_ep, table_dict, tables_for

pytestmark = pytest.mark.gpu

STATE_ATOL = 1e-9
F32_ATOL = 1e-5


def _gpu_env(meta, n_envs=1, seed=None, **kw):
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    args = EnvArgs.from_namespace(type("A", (), meta)())
    args.seed = meta["env_seed"] if seed is None else seed
    vt, tt = tables_for(meta)
    return GpuGraphVecEnv(args, num_envs=n_envs, device="cuda:0", value_table=vt, ttr_table=tt, **kw)


def _info_col(name):
    from lsm import capi
    return capi.INFO_FIELDS.index(name)


GPU_FIXTURES = list(fixture_names())


@pytest.mark.parametrize("kernel", ["wave", "block", "blockc"])
@pytest.mark.parametrize("name", GPU_FIXTURES)
def test_gpu_matches_reference_golden(name, kernel):
    """Every golden fixture through the one-wave kernel and the workgroup-per-env kernel
    (kernel_select workgroup_per_env; "blockc": compact adjacency layout, expanded for the comparison)."""
    ksel = {"workgroup_per_env": 1} if kernel != "wave" else None
    z, meta = load(name)
    env = _gpu_env(meta, emit_edges=True, adj_layout="compact" if kernel == "blockc" else "reference",
                   kernel_select=ksel)
    obs, aid, node, adj, ep = env.reset(meta["ep"])
    np.testing.assert_allclose(obs[0], z["reset0_obs"], rtol=0, atol=F32_ATOL)
    np.testing.assert_allclose(node[0], z["reset0_node"], rtol=0, atol=F32_ATOL)
    np.testing.assert_allclose(adj[0], z["reset0_adj"], rtol=0, atol=F32_ATOL)
    np.testing.assert_array_equal(adj[0] != 0, z["reset0_adj"] != 0)
    np.testing.assert_allclose(env.state().cpu().numpy()[0], z["reset0_state"], rtol=0, atol=STATE_ATOL)
    np.testing.assert_allclose([ep[0][k] for k in EPKEYS], z["resets_info"][0], rtol=1e-12, atol=1e-12)
    if "inject_state" in z.files:   # the fixture edited the world after the reset (finding 4)
        env.set_agent_state(0, z["inject_state"], z["inject_reached"])
    n_reset = 1
    c_mr, c_sf, c_dec = _info_col("min_relative_distance"), _info_col("Safety filtered"), \
        _info_col("deconflicting_agent_index")
    c_rg = _info_col("reached_goal")
    for t in range(meta["steps"]):
        ctx = "%s step %d" % (name, t)
        obs, aid, node, adj, rew, dones, infos = env.step(z["act"][t][None], step_ep(z, meta, t))
        info = env.t_info.cpu().numpy()[0]
        reset = bool(env.t_reset.cpu().numpy()[0])
        np.testing.assert_array_equal(dones[0], z["dones"][t], err_msg=ctx)
        np.testing.assert_allclose(rew[0], z["rew"][t], rtol=1e-6, atol=1e-5, err_msg=ctx)
        np.testing.assert_array_equal(info[:, c_rg], z["reached"][t], err_msg=ctx)
        np.testing.assert_allclose(info[:, c_mr], z["minrel"][t], rtol=0, atol=STATE_ATOL, err_msg=ctx)
        np.testing.assert_array_equal(info[:, c_sf].astype(bool), z["sfilt"][t], err_msg=ctx)
        np.testing.assert_array_equal(info[:, c_dec].astype(int), z["decon"][t], err_msg=ctx)
        ref_info = z["info_num"][t]
        for j, k in enumerate(INFOKEYS):
            np.testing.assert_allclose(info[:, _info_col(k)], ref_info[:, j], rtol=1e-9, atol=1e-9,
                                       err_msg=ctx + " info " + k)
        if not reset:
            np.testing.assert_allclose(env.state().cpu().numpy()[0], z["state"][t], rtol=0, atol=STATE_ATOL,
                                       err_msg=ctx)
            np.testing.assert_allclose(obs[0], z["obs"][t], rtol=0, atol=F32_ATOL, err_msg=ctx)
            np.testing.assert_array_equal(adj_bits(adj[0]), z["adj_bits"][t], err_msg=ctx)
            key = "t%03d_node" % t
            if key in z.files:
                np.testing.assert_allclose(node[0], z[key], rtol=0, atol=F32_ATOL, err_msg=ctx)
                np.testing.assert_allclose(adj[0], z["t%03d_adj" % t], rtol=0, atol=F32_ATOL, err_msg=ctx)
                e = np.stack(np.nonzero(env.t_edges.cpu().numpy()[0]))
                np.testing.assert_array_equal(e, z["t%03d_edges" % t], err_msg=ctx)
        else:
            assert z["resets_t"][n_reset] == t + 1, ctx
            assert len(infos[0]) == meta["num_agents"] + 1
            np.testing.assert_allclose([infos[0][-1][k] for k in EPKEYS], z["resets_info"][n_reset],
                                       rtol=1e-9, atol=1e-9, err_msg=ctx)
            np.testing.assert_allclose(env.state().cpu().numpy()[0], z["t%03d_reset_state" % t],
                                       rtol=0, atol=STATE_ATOL, err_msg=ctx)
            np.testing.assert_allclose(obs[0], z["t%03d_reset_obs" % t], rtol=0, atol=F32_ATOL, err_msg=ctx)
            np.testing.assert_allclose(node[0], z["t%03d_reset_node" % t], rtol=0, atol=F32_ATOL, err_msg=ctx)
            np.testing.assert_allclose(adj[0], z["t%03d_reset_adj" % t], rtol=0, atol=F32_ATOL, err_msg=ctx)
            n_reset += 1
    assert n_reset == len(z["resets_t"])
    env.close()


ALL_TERMS = ("safety_violation", "potential_conflict", "diff_from_filtered_action", "hj_value")


def _oracle_for(meta, seed, n_envs, env_offset=0):
    from oracle.lsm_oracle import OracleVecEnv
    vt, tt = tables_for(meta)
    return OracleVecEnv(meta, n_envs, seed=seed, value_table=table_dict(vt), ttr_table=table_dict(tt),
                        integrator="restated", seed_offset=env_offset)


CASES = [
    dict(dynamics_type="double_integrator", num_agents=8, world_size=4, episode_length=250,
         num_env_steps=250 * 4, use_safety_filter=True, ep=4),
    dict(dynamics_type="double_integrator", num_agents=8, world_size=4, episode_length=250,
         num_env_steps=250 * 4, use_safety_filter=False, ep=1),
    dict(dynamics_type="double_integrator", num_agents=5, world_size=4, episode_length=60,
         num_env_steps=60 * 4, use_safety_filter=True, ep=3),
    dict(dynamics_type="airtaxi", num_agents=6, world_size=6, episode_length=80,
         num_env_steps=80 * 4, use_safety_filter=True, ep=4),
    dict(dynamics_type="airtaxi", num_agents=4, world_size=6, episode_length=80,
         num_env_steps=80 * 4, use_safety_filter=False, ep=2),
    # BASELINE config 4's env: 16 airtaxi agents (E = 48), filter on -> rollout_kernel<1, 64, 16>
    dict(dynamics_type="airtaxi", num_agents=16, world_size=6, episode_length=20,
         num_env_steps=20 * 4, use_safety_filter=True, ep=4, n_envs=8),
    # compile-time N = 8 / N = 3 double integrator (rollout_kernel<0, 64, 8> / <0, 64, 3>)
    dict(dynamics_type="double_integrator", num_agents=3, world_size=4, episode_length=60,
         num_env_steps=60 * 4, use_safety_filter=True, ep=4),
    # RewardBinaryConfig's four optional terms and the shared reward of --collaborative
    # (navigation_graph_safe.py:793-850, environment.py:1031-1037) through every kernel variant: the
    # team kernel's agent wave at N = 8 (stair ratio the int 1: float32 HJ-value products) ...
    dict(dynamics_type="double_integrator", num_agents=8, world_size=4, episode_length=60,
         num_env_steps=60 * 4, use_safety_filter=True, ep=4, collaborative=True, reward_terms=ALL_TERMS),
    # ... airtaxi N = 16 mid-curriculum (float64 weights) ...
    dict(dynamics_type="airtaxi", num_agents=16, world_size=6, episode_length=20,
         num_env_steps=20 * 4, use_safety_filter=True, ep=2, n_envs=8, collaborative=True,
         reward_terms=ALL_TERMS),
    # ... and the HJ-value term with the filter off (the handle exists only for the reward)
    dict(dynamics_type="double_integrator", num_agents=5, world_size=4, episode_length=60,
         num_env_steps=60 * 4, use_safety_filter=False, ep=1, reward_terms=("hj_value", "safety_violation")),
    # ... and the HJ-value term alone with the filter on: reward_reach_goal's Python-float base
    # (`rew -= 1.0`) plus float32 terms stays float32 (fixture di_n8_rw_hjf)
    dict(dynamics_type="double_integrator", num_agents=8, world_size=4, episode_length=60,
         num_env_steps=60 * 4, use_safety_filter=True, ep=4, collaborative=True, reward_terms=("hj_value",)),
]


_ORACLE_RUNS = {}


def _case_meta(case):
    c = dict(CASES[case])
    ep = c.pop("ep")
    nb = c.pop("n_envs", 16)   # the oracle takes ~36 ms per 16-agent airtaxi env-step
    meta = dict(num_landmarks=2, n_rollout_threads=1, use_masking=True, num_internal_step=1, seed=5,
                env_seed=5, **c)
    return meta, ep, nb


def _oracle_run(case):
    """The oracle's trajectory of CASES[case] over its nb envs, computed once per session and
    shared by every kernel variant: env k's episodes depend only on its own seed (seed + 1000 k)
    and actions, and the actions are drawn for all nb envs every step, so a variant running the
    first nb - 1 envs sees the same trajectories. Graph outputs kept as float32 (the kernel's
    output type; the tolerance is 1e-5 absolute)."""
    if case in _ORACLE_RUNS:
        return _ORACLE_RUNS[case]
    meta, ep, nb = _case_meta(case)
    steps = min(meta["episode_length"] + 20, 120)
    ora = _oracle_for(meta, 5, nb)
    o = ora.reset(ep)
    f32 = lambda x: np.asarray(x, dtype=np.float32)
    run = dict(reset=(f32(o[0]), f32(o[2]), f32(o[3])), steps=[])
    rng = np.random.default_rng(case)
    for _ in range(steps):
        a = rng.integers(0, 25, (nb, meta["num_agents"]))
        o = ora.step(a, ep)
        run["steps"].append(dict(a=a, obs=f32(o[0]), node=f32(o[2]), adj=f32(o[3]), rew=np.asarray(o[4]),
                                 dones=np.asarray(o[5]), state=np.stack([e.s.copy() for e in ora.envs]),
                                 ind_rew=np.array([[d["individual_reward"] for d in inf[:meta["num_agents"]]]
                                                   for inf in o[6]], dtype=np.float64)))
    _ORACLE_RUNS[case] = run
    return run


@pytest.mark.parametrize("lpe", [16, 32, 64, "64w", "t2", "t4", "t8", "64g", "block", "blockc"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_gpu_matches_oracle_multi_env(case, lpe):
    """16 (or 15: a partly filled last wave / workgroup) envs with per-env seeds seed + 1000 k,
    random actions, across an auto-reset; every kernel variant: 1, 2 or 4 envs/wave; at one env
    per wave the default dispatch ("64": the team kernel for N = 8 double integrator (8 envs per
    workgroup) and N = 16 airtaxi (4 per workgroup), the compile-time-N rollout_kernel for
    N = 3), the one-wave rollout_kernel forced ("64w", team 0), the team kernel with 2 / 4
    envs per workgroup ("t2", "t4", "t8"; one fewer env than a whole number of workgroups), the
    generic kernel ("64g"), and the workgroup-per-env
    kernel in both adjacency layouts ("block", "blockc"). The oracle's trajectory is computed once
    per case (_oracle_run)."""
    c0 = CASES[case]
    if lpe == 16 and c0["num_agents"] == 16 and c0["dynamics_type"] == "airtaxi":
        pytest.skip("4 airtaxi envs of 16 agents per wave need 98 KB of LDS (> 64 KB per workgroup)")
    team_spec = (c0["num_agents"], c0["dynamics_type"]) in ((8, "double_integrator"), (16, "airtaxi"))
    if lpe in ("t2", "t4", "t8", "64w") and not team_spec:
        pytest.skip("the team kernel is specialised for N = 8 double integrator and N = 16 airtaxi")
    if lpe == "t8" and c0["num_agents"] == 16:
        pytest.skip("8 airtaxi envs of 16 agents do not fit one 64-lane agent wave")
    # "t4" at airtaxi N = 16: 4 envs x 19.3 KB in the lean LDS layout (77 KB per workgroup)
    partial = lpe in (16, 32, "t2", "t4", "t8")
    ksel = {}
    if lpe in ("t2", "t4", "t8", "64w"):
        ksel["team"] = 0 if lpe == "64w" else int(lpe[1:])
        lpe = 64
    layout = "reference"
    if lpe in ("block", "blockc"):
        ksel["workgroup_per_env"] = 1
        layout = "compact" if lpe == "blockc" else "reference"
        lpe = 64
    if lpe == "64g":
        ksel["generic"] = 1
        lpe = 64
    ksel["lanes_per_env"] = lpe
    meta, ep, nb = _case_meta(case)
    run = _oracle_run(case)
    n = nb - 1 if partial else nb
    env = _gpu_env(meta, n_envs=n, seed=5, adj_layout=layout, kernel_select=ksel)
    g = env.reset(ep)
    o = run["reset"]
    np.testing.assert_allclose(g[0], o[0][:n], rtol=0, atol=F32_ATOL)
    np.testing.assert_allclose(g[2], o[1][:n], rtol=0, atol=F32_ATOL)
    np.testing.assert_array_equal(g[3] != 0, o[2][:n] != 0)
    mism = 0
    drew = dind = 0.0
    for t, r in enumerate(run["steps"]):
        g = env.step(r["a"][:n], ep)
        ctx = "case %d step %d" % (case, t)
        np.testing.assert_array_equal(g[5], r["dones"][:n], err_msg=ctx)
        np.testing.assert_array_equal(g[3] != 0, r["adj"][:n] != 0, err_msg=ctx)
        np.testing.assert_allclose(g[0], r["obs"][:n], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[2], r["node"][:n], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[3], r["adj"][:n], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[4], r["rew"][:n], rtol=1e-6, atol=1e-5, err_msg=ctx)
        ind = env.t_info.cpu().numpy()[:, :, _info_col("individual_reward")]
        np.testing.assert_allclose(ind, r["ind_rew"][:n], rtol=1e-9, atol=1e-9, err_msg=ctx + " individual_reward")
        drew = max(drew, float(np.abs(np.asarray(g[4], dtype=np.float64).reshape(n, -1) -
                                      np.asarray(r["rew"][:n], dtype=np.float64).reshape(n, -1)).max()))
        dind = max(dind, float(np.abs(ind - r["ind_rew"][:n]).max()))
        st = env.state().cpu().numpy()
        np.testing.assert_allclose(st, r["state"][:n], rtol=0, atol=STATE_ATOL, err_msg=ctx)
        mism += int(np.any(st != r["state"][:n], axis=(1, 2)).sum())
    # states are compared at STATE_ATOL; how many env-steps were not bit-identical is reported
    print("state_mismatch case=%d lpe=%s env_steps_not_bit_identical=%d of %d" % (case, lpe, mism,
                                                                              len(run["steps"]) * n))
    # the largest reward deviations from the oracle (float32 output; float64 individual_reward)
    print("reward_deviation case=%d lpe=%s max_abs_reward=%.3g max_abs_individual_reward=%.3g" % (case, lpe, drew, dind))
    env.close()


def _full_tables(meta):
    """The full-shape synthetic tables bench.py times (lsm.hj_tables.default_tables): DI (61, 61, 41,
    41), airtaxi (41, 41, 36, 9, 9) + TTR (41, 41, 36, 9) -- not golden_replay.tables_for's small ones."""
    from lsm import hj_tables
    return hj_tables.default_tables(meta["dynamics_type"])


def _full_env_and_oracles(meta, n_envs, sample, **kw):
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    from oracle.lsm_oracle import OracleVecEnv
    args = EnvArgs.from_namespace(type("A", (), meta)())
    args.seed = meta["env_seed"]
    vt, tt = _full_tables(meta)
    env = GpuGraphVecEnv(args, num_envs=n_envs, device="cuda:0", value_table=vt, ttr_table=tt,
                         return_numpy=False, **kw)
    oras = [OracleVecEnv(meta, 1, seed=meta["env_seed"], value_table=table_dict(vt), ttr_table=table_dict(tt),
                         integrator="restated", seed_offset=k) for k in sample]
    return env, oras


def _check_all_envs(ora_all, s, obs, adj, dones, rew, st, ctx):
    """Step s of every env against the oracle pool's run: dones and adjacency bits exact, obs and
    rewards within the fp32 tolerance, states within STATE_ATOL."""
    n = obs.shape[0]
    np.testing.assert_array_equal(dones.cpu().numpy(), ora_all["dones"][:, s], err_msg=ctx + " dones")
    bits = np.packbits((adj != 0).reshape(n, -1).cpu().numpy(), axis=1)
    bad = np.nonzero((bits != ora_all["adj"][:, s]).any(axis=1))[0]
    assert len(bad) == 0, "%s: adjacency bits differ in envs %s" % (ctx, bad[:10].tolist())
    np.testing.assert_allclose(obs.cpu().numpy(), ora_all["obs"][:, s], rtol=0, atol=F32_ATOL, err_msg=ctx)
    np.testing.assert_allclose(rew.cpu().numpy(), ora_all["rew"][:, s], rtol=1e-6, atol=1e-5, err_msg=ctx)
    np.testing.assert_allclose(st.cpu().numpy(), ora_all["state"][:, s], rtol=0, atol=STATE_ATOL, err_msg=ctx)


def test_gpu_full_size_properties_and_sampled_oracle():
    """BASELINE config 3 exactly as bench.py times it (8 agents x 4096 envs, filter on, the full-shape
    (61, 61, 41, 41) HJ table): ALL 4096 envs against the oracle at the reset and the first 3 steps
    (dones, adjacency bits, obs, rewards, states; the oracle over worker processes, tests/oracle_pool.py);
    invariants over 260 steps (one auto-reset at step 250) + exact replay of sampled envs through it."""
    import torch
    from oracle_pool import run_all_envs
    meta = dict(dynamics_type="double_integrator", num_agents=8, num_landmarks=2, world_size=4,
                episode_length=250, num_env_steps=250 * 4, n_rollout_threads=1, use_safety_filter=True,
                use_masking=True, num_internal_step=1, seed=0, env_seed=0)
    n_envs, N, S_ALL, T = 4096, 8, 3, 260
    acts = np.random.default_rng(0).integers(0, 25, (T, n_envs, N)).astype(np.int32)
    ora_all = run_all_envs(meta, 0, n_envs, 4, np.ascontiguousarray(acts[:S_ALL].transpose(1, 0, 2)))
    sample = [0, 1, 1337, 4095]
    env, oras = _full_env_and_oracles(meta, n_envs, sample)
    assert env.value_table.shape == (61, 61, 41, 41)
    obs, aid, node, adj, ep = env.reset(4)
    np.testing.assert_allclose(obs.cpu().numpy(), ora_all["reset_obs"], rtol=0, atol=F32_ATOL)
    bits = np.packbits((adj != 0).reshape(n_envs, -1).cpu().numpy(), axis=1)
    np.testing.assert_array_equal(bits, ora_all["reset_adj"])
    for k, o in zip(sample, oras):
        o.reset(4)
    for t in range(T):
        a = torch.as_tensor(acts[t], device="cuda:0")
        obs, aid, node, adj, rew, dones, (info, reset, epinfo) = env.step(a, 4)
        st = env.state()
        if t < S_ALL:
            _check_all_envs(ora_all, t, obs, adj, dones, rew, st, "all envs, step %d" % t)
        if t % 20 == 0 or t >= 248:
            assert torch.isfinite(obs).all() and torch.isfinite(node).all() and torch.isfinite(adj).all()
            assert (adj >= 0).all() and (adj <= 4).all()   # the float32 cast of d < 4 may be 4.0f
            d = torch.diagonal(adj, dim1=2, dim2=3)
            assert (d == 0).all()
            assert torch.equal(adj, adj.transpose(2, 3))
            sp = torch.sqrt(st[..., 2] ** 2 + st[..., 3] ** 2)
            assert (sp <= 0.5 + 1e-12).all()
        if t == 249:
            assert bool(reset.all())
        elif t < 249:
            assert not bool(reset.any()) or bool(dones.all(dim=1)[reset.bool()].all())
        for k, o in zip(sample, oras):
            r = o.step(acts[t][k:k + 1], 4)
            np.testing.assert_array_equal(dones[k].cpu().numpy(), r[5][0], err_msg="env %d step %d" % (k, t))
            np.testing.assert_array_equal((adj[k] != 0).cpu().numpy(), r[3][0] != 0)
            np.testing.assert_allclose(obs[k].cpu().numpy(), r[0][0], rtol=0, atol=F32_ATOL)
            np.testing.assert_allclose(st[k].cpu().numpy(), o.envs[0].s, rtol=0, atol=STATE_ATOL)
    env.close()


LARGE_CASES = [
    # BASELINE config 5's env (64 double-integrator agents, E = 192), filter on, short episodes
    dict(dynamics_type="double_integrator", num_agents=64, world_size=4, episode_length=10,
         num_env_steps=10 * 4, use_safety_filter=True, ep=4),
    # filter off (magnetic-field penalty over 256 lanes), curriculum mid-way
    dict(dynamics_type="double_integrator", num_agents=64, world_size=4, episode_length=10,
         num_env_steps=10 * 4, use_safety_filter=False, ep=1),
    # generic workgroup kernel: odd N, E = 99 (not a multiple of 4, two mask words)
    dict(dynamics_type="double_integrator", num_agents=33, world_size=4, episode_length=10,
         num_env_steps=10 * 4, use_safety_filter=True, ep=4),
    # airtaxi with E = 120
    dict(dynamics_type="airtaxi", num_agents=40, world_size=6, episode_length=10,
         num_env_steps=10 * 4, use_safety_filter=True, ep=4),
]


@pytest.mark.parametrize("layout", ["compact", "reference"])
@pytest.mark.parametrize("case", range(len(LARGE_CASES)))
def test_gpu_large_n_matches_oracle(case, layout):
    """N > 32 (the workgroup-per-env kernel, chosen automatically): 2 envs over 13 steps
    (one auto-reset at step 10) vs the oracle, every output."""
    c = dict(LARGE_CASES[case])
    ep = c.pop("ep")
    meta = dict(num_landmarks=2, n_rollout_threads=1, use_masking=True, num_internal_step=1, seed=11,
                env_seed=11, **c)
    n_envs, N = 2, meta["num_agents"]
    env = _gpu_env(meta, n_envs=n_envs, seed=11, adj_layout=layout, emit_edges=True)
    ora = _oracle_for(meta, 11, n_envs)
    g = env.reset(ep)
    o = ora.reset(ep)
    np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL)
    np.testing.assert_allclose(g[2], o[2], rtol=0, atol=F32_ATOL)
    np.testing.assert_allclose(g[3], o[3], rtol=0, atol=F32_ATOL)
    np.testing.assert_array_equal(g[3] != 0, o[3] != 0)
    rng = np.random.default_rng(100 + case)
    for t in range(13):
        a = rng.integers(0, 25, (n_envs, N))
        g = env.step(a, ep)
        o = ora.step(a, ep)
        ctx = "case %d step %d" % (case, t)
        np.testing.assert_array_equal(g[5], o[5], err_msg=ctx)
        np.testing.assert_array_equal(g[3] != 0, o[3] != 0, err_msg=ctx)
        np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[2], o[2], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[3], o[3], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[4], o[4], rtol=1e-6, atol=1e-5, err_msg=ctx)
        st = env.state().cpu().numpy()
        info = env.t_info.cpu().numpy()
        for k, e in enumerate(ora.envs):
            np.testing.assert_allclose(st[k], e.s, rtol=0, atol=STATE_ATOL, err_msg=ctx)
        for k in range(n_envs):
            for i in range(N):
                oi = o[6][k][i]
                for name in ("min_relative_distance", "Num_agent_collisions", "Dist_to_goal", "Distance_mean",
                             "Time_mean"):
                    np.testing.assert_allclose(info[k, i, _info_col(name)], oi[name], rtol=1e-9, atol=1e-9,
                                               err_msg=ctx + " " + name)
                assert bool(info[k, i, _info_col("Safety filtered")]) == bool(oi["Safety filtered"]), ctx
            e = ora.envs[k]
            if env.t_reset.cpu().numpy()[k]:
                continue   # the oracle env's per-step arrays were re-initialised by its reset
            np.testing.assert_array_equal(info[k, :, _info_col("deconflicting_agent_index")].astype(int),
                                          e.deconflicting, err_msg=ctx)
            np.testing.assert_allclose(info[k, :, _info_col("action_diff")], e.action_diff, rtol=0, atol=1e-12,
                                       err_msg=ctx)
    env.close()


def test_gpu_config5_full_size_compact():
    """BASELINE config 5's per-GPU shard (64 DI agents x 8192 envs, filter on, compact
    adjacency): invariants over 12 steps + exact replay of sampled envs through the oracle."""
    import torch
    meta = dict(dynamics_type="double_integrator", num_agents=64, num_landmarks=2, world_size=4,
                episode_length=250, num_env_steps=250 * 4, n_rollout_threads=1, use_safety_filter=True,
                use_masking=True, num_internal_step=1, seed=0, env_seed=0)
    n_envs, N, E = 8192, 64, 192
    env = _gpu_env(meta, n_envs=n_envs, seed=0, return_numpy=False, adj_layout="compact")
    sample = [0, 8191]
    oras = [_oracle_for(meta, 0, 1, env_offset=k) for k in sample]
    obs, aid, node, adj, ep = env.reset(4)
    assert adj.shape == (n_envs, E, E) and env.t_adj_mask.shape == (n_envs, N, 3)
    for k, o in zip(sample, oras):
        r = o.reset(4)
        np.testing.assert_allclose(obs[k].cpu().numpy(), r[0][0], rtol=0, atol=F32_ATOL)
    gen = torch.Generator(device="cuda:0").manual_seed(0)
    for t in range(12):
        a = torch.randint(0, 25, (n_envs, N), device="cuda:0", generator=gen, dtype=torch.int32)
        obs, aid, node, adj, rew, dones, (info, reset, epinfo) = env.step(a, 4)
        assert torch.isfinite(obs).all() and torch.isfinite(node).all()
        # d < 4 in float64; the float32 cast may round up to exactly 4.0f
        assert (adj >= 0).all() and (adj <= 4).all() and torch.equal(adj, adj.transpose(1, 2))
        assert (torch.diagonal(adj, dim1=1, dim2=2) == 0).all()
        st = env.state()
        assert (torch.sqrt(st[..., 2] ** 2 + st[..., 3] ** 2) <= 0.5 + 1e-12).all()
        a_h = a.cpu().numpy()
        ref_adj = env.reference_adj()
        for k, o in zip(sample, oras):
            r = o.step(a_h[k:k + 1], 4)
            np.testing.assert_array_equal(dones[k].cpu().numpy(), r[5][0])
            np.testing.assert_allclose(ref_adj[k].cpu().numpy(), r[3][0], rtol=0, atol=F32_ATOL)
            np.testing.assert_allclose(node[k].cpu().numpy(), r[2][0], rtol=0, atol=F32_ATOL)
            np.testing.assert_allclose(obs[k].cpu().numpy(), r[0][0], rtol=0, atol=F32_ATOL)
            np.testing.assert_allclose(st[k].cpu().numpy(), o.envs[0].s, rtol=0, atol=STATE_ATOL)
    env.close()


@pytest.mark.gpu
def test_gpu_action_encodings_and_dummy_semantics():
    """The runner's one-hot actions (float32 / float64, graph_mpe_runner.py:432-433) decode like
    indices (environment.py:386-410); auto_reset=False (GraphDummyVecEnv, env_wrappers.py:918-928)
    returns the 8-tuple, keeps stepping past the episode end without resetting, and matches the
    oracle with auto_reset=False."""
    import torch
    c = dict(CASES[2])
    ep = c.pop("ep")
    c["episode_length"], c["num_env_steps"] = 12, 48
    meta = dict(num_landmarks=2, n_rollout_threads=1, use_masking=True, num_internal_step=1, seed=2, ep=ep, **c)
    n, N, T = 6, meta["num_agents"], 16
    rng = np.random.default_rng(4)
    acts = rng.integers(0, 25, (T, n, N))
    envs = {k: _gpu_env(meta, n_envs=n, seed=2, return_numpy=True) for k in ("idx", "f32", "f64")}
    for e in envs.values():
        e.reset(meta["ep"])
    eye = np.eye(25)
    for t in range(T):
        outs = {}
        for k, e in envs.items():
            a = acts[t] if k == "idx" else eye[acts[t]].astype(np.float32 if k == "f32" else np.float64)
            if k == "f64":
                a = torch.as_tensor(a, device="cuda:0")   # device one-hot tensor
            outs[k] = e.step(a, meta["ep"])
        for k in ("f32", "f64"):
            for i in (0, 2, 3, 4, 5):
                np.testing.assert_array_equal(outs[k][i], outs["idx"][i], err_msg="%s t=%d out %d" % (k, t, i))
    for e in envs.values():
        e.close()

    gpu = _gpu_env(meta, n_envs=n, seed=2, return_numpy=True, auto_reset=False)
    ora = _oracle_for(meta, 2, n)
    ora.auto_reset = False
    g, o = gpu.reset(meta["ep"]), ora.reset(meta["ep"])
    np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL)
    for t in range(T):
        g = gpu.step(acts[t], meta["ep"])
        o = ora.step(acts[t], meta["ep"])
        assert len(g) == 8 and g[7] == 0
        np.testing.assert_array_equal(g[5], o[5], err_msg="t=%d" % t)
        np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL, err_msg="t=%d" % t)
        np.testing.assert_allclose(g[4], o[4], rtol=1e-6, atol=1e-5, err_msg="t=%d" % t)
        np.testing.assert_array_equal(g[3] != 0, o[3] != 0, err_msg="t=%d" % t)
        if t >= meta["episode_length"] - 1:
            assert g[5].all()                    # past the end: every agent done, no reset
    assert not gpu.t_reset.cpu().numpy().any()
    gpu.close()


def _goal_policy(envs, rng, eps=0.1):
    """Goal-seeking discrete actions from the oracle envs' states (make_golden.py's policy)."""
    out = []
    for e in envs:
        idx = np.zeros(e.N, dtype=np.int64)
        for i in range(e.N):
            if rng.random() < eps:
                idx[i] = rng.integers(0, 25)
                continue
            g, s = e.lm_pos[e.goal_index(i)], e.s[i]
            acc = 1.2 * (g - s[:2]) - 1.5 * s[2:]
            q = np.clip(np.round(acc / 0.25), -2, 2).astype(int) + 2
            idx[i] = q[0] * 5 + q[1]
        out.append(idx)
    return np.array(out)


def _arrive_all(e):
    """Every agent of oracle env e placed on its last goal at the goal's speed and heading with
    reached_goal = L - 1 (make_golden.py's inject_goal_arrival for all agents): with zero
    acceleration the next step reaches every final goal, so the env is all-done early."""
    L, N = e.L, e.N
    st = e.s.copy()
    for i in range(N):
        g = (L - 1) * N + i
        sp, h = e.lm_speed[g], e.lm_heading[g]
        st[i] = [e.lm_pos[g][0], e.lm_pos[g][1], sp * np.cos(h), sp * np.sin(h)]
    return st, np.full(N, L - 1, dtype=np.int32)


@pytest.mark.parametrize("kernel", ["wave", "block"])
def test_gpu_runner_call_pattern_separation_curriculum(kernel):
    """GMPERunner's real call pattern (graph_mpe_runner.py:72-103): step(actions, episode) with the
    episode index advancing every episode_length steps, the worker auto-resetting with it
    (env_wrappers.py:866-871). With SEPARATION_DISTANCE_CURRICULUM each reset shifts that env's own
    HJ table (safety_filter.py:170-174 via navigation_graph_safe.py:349-364); envs driven all-done
    mid-episode reset at the newer stair level while the others keep the older one, so envs hold
    different tables at once. 16 envs vs the oracle, every step."""
    ksel = {"workgroup_per_env": 1} if kernel == "block" else None
    epl, ep0, n_envs, N = 60, 3, 16, 3
    meta = dict(dynamics_type="double_integrator", num_agents=N, num_landmarks=2, world_size=4,
                episode_length=epl, num_env_steps=epl * 10, n_rollout_threads=1, use_safety_filter=True,
                use_masking=True, num_internal_step=1, seed=9, env_seed=9, separation_distance_curriculum=True)
    env = _gpu_env(meta, n_envs=n_envs, seed=9, kernel_select=ksel)
    ora = _oracle_for(meta, 9, n_envs)
    g, o = env.reset(ep0), ora.reset(ep0)
    np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL)
    rng = np.random.default_rng(17)
    early = {epl + 20: (0, 5, 11), 2 * epl + 7: (0, 3), 3 * epl + 30: (5, 9, 14), 3 * epl + 31: (5,)}
    c_sf = _info_col("Safety filtered")
    split_seen = early_resets = 0
    for t in range(5 * epl):
        ep = ep0 + t // epl
        a = _goal_policy(ora.envs, rng)
        for k in early.get(t - 1, ()):
            a[k] = 12                                       # zero acceleration after the arrival
        g = env.step(a, ep)
        o = ora.step(a, ep)
        ctx = "step %d ep %d" % (t, ep)
        np.testing.assert_array_equal(g[5], o[5], err_msg=ctx)
        np.testing.assert_array_equal(g[3] != 0, o[3] != 0, err_msg=ctx)
        np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[2], o[2], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[3], o[3], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[4], o[4], rtol=1e-6, atol=1e-5, err_msg=ctx)
        st = env.state().cpu().numpy()
        info = env.t_info.cpu().numpy()
        for k, e in enumerate(ora.envs):
            np.testing.assert_allclose(st[k], e.s, rtol=0, atol=STATE_ATOL, err_msg=ctx)
            np.testing.assert_array_equal(info[k, :, c_sf].astype(bool),
                                          [bool(x["Safety filtered"]) for x in o[6][k][:N]], err_msg=ctx)
        reset = env.t_reset.cpu().numpy()
        if (t + 1) % epl:
            early_resets += int(reset.sum())
        split_seen += len({e.hj_sep for e in ora.envs}) > 1
        for k in early.get(t, ()):                          # drive env k all-done at the next step
            s, r = _arrive_all(ora.envs[k])
            env.set_agent_state(k, s, r)
            e = ora.envs[k]
            e.s[:] = s
            e.reached_goal[:] = r
            e.calculate_distances()
    assert early_resets >= 8, early_resets
    assert split_seen > 0
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["wave", "block", "team"])
def test_gpu_separation_chain_unbounded(kernel):
    """HjDataHandle.update_separation_distance (safety_filter.py:170-174) has no limit: 24 separation
    changes (alternating stair levels, well past the record's 8 slots: the chain continues in the
    per-env HBM overflow, grown twice) and the filter after each still matches the oracle, whose
    table is shifted in place as the reference's is; a re-upload then starts every chain afresh.
    "team": 8 agents, the config-3 kernel (rollout_team_kernel<0, 8, 4>)."""
    ksel = {"workgroup_per_env": 1} if kernel == "block" else None
    meta = dict(dynamics_type="double_integrator", num_agents=8 if kernel == "team" else 4, num_landmarks=2, world_size=4,
                episode_length=5, num_env_steps=5 * 20, n_rollout_threads=1, use_safety_filter=True,
                use_masking=True, num_internal_step=1, seed=1, env_seed=1, separation_distance_curriculum=True)
    n = 3
    env = _gpu_env(meta, n_envs=n, seed=1, kernel_select=ksel)
    ora = _oracle_for(meta, 1, n)
    # stair levels of ep = 0, 4, 8, 12, 16 (0, .25, .5, .75, 1); up and down, 24 changes
    seq = [0] + [4, 8, 12, 16, 12, 8, 4, 8] * 3
    rng = np.random.default_rng(3)
    for k, ep in enumerate(seq):
        g, o = env.reset(ep), ora.reset(ep)
        np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL)
        for t in range(3):
            a = rng.integers(0, 25, (n, meta["num_agents"]))
            g, o = env.step(a, ep), ora.step(a, ep)
            ctx = "reset %d (ep %d) step %d" % (k, ep, t)
            np.testing.assert_array_equal(g[5], o[5], err_msg=ctx)
            np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL, err_msg=ctx)
            np.testing.assert_allclose(env.state().cpu().numpy(), np.stack([e.s for e in ora.envs]), rtol=0,
                                       atol=STATE_ATOL, err_msg=ctx)
            info = env.t_info.cpu().numpy()
            np.testing.assert_array_equal(info[:, :, _info_col("deconflicting_agent_index")].astype(int),
                                          np.stack([e.deconflicting for e in ora.envs]), err_msg=ctx)
            np.testing.assert_array_equal(info[:, :, _info_col("Safety filtered")].astype(bool),
                                          np.stack([e.safety_filtered for e in ora.envs]), err_msg=ctx)
    name = env.lib.lsm_kernel_name(env.h).decode()
    assert ("team" in name) == (kernel == "team"), name
    env._upload_value_table()   # a new HjDataHandle: chains start empty, nothing refused
    env.reset(12)
    env.close()


def test_gpu_config4_full_size_properties_and_sampled_oracle():
    """BASELINE config 4 exactly as bench.py times it (16 airtaxi agents x 8192 envs, HJ filter on,
    episode_length 350, the full-shape (41, 41, 36, 9, 9) value and (41, 41, 36, 9) TTR tables):
    ALL 8192 envs against the oracle at the reset and the first step (tests/oracle_pool.py);
    rollout_team_kernel<1, 16, 4> over 360 steps spanning the auto-reset at step 350: invariants
    every 20 steps and around the reset, and sampled envs replayed exactly through the oracle."""
    import torch
    from oracle_pool import run_all_envs
    meta = dict(dynamics_type="airtaxi", num_agents=16, num_landmarks=2, world_size=6,
                episode_length=350, num_env_steps=350 * 4, n_rollout_threads=1, use_safety_filter=True,
                use_masking=True, num_internal_step=1, seed=0, env_seed=0)
    n_envs, N, E, S_ALL, T = 8192, 16, 48, 1, 360
    acts = np.random.default_rng(4).integers(0, 25, (T, n_envs, N)).astype(np.int32)
    ora_all = run_all_envs(meta, 0, n_envs, 4, np.ascontiguousarray(acts[:S_ALL].transpose(1, 0, 2)))
    sample = [0, 8191]   # the oracle takes ~36 ms per env-step here
    env, oras = _full_env_and_oracles(meta, n_envs, sample)
    assert env.value_table.shape == (41, 41, 36, 9, 9) and env.ttr_table.shape == (41, 41, 36, 9)
    obs, aid, node, adj, ep = env.reset(4)
    assert node.shape == (n_envs, N, E, 11) and adj.shape == (n_envs, N, E, E)
    np.testing.assert_allclose(obs.cpu().numpy(), ora_all["reset_obs"], rtol=0, atol=F32_ATOL)
    bits = np.packbits((adj != 0).reshape(n_envs, -1).cpu().numpy(), axis=1)
    np.testing.assert_array_equal(bits, ora_all["reset_adj"])
    for k, o in zip(sample, oras):
        o.reset(4)
    vmin, vmax = 60 * 0.514444 * 0.001, 175 * 0.514444 * 0.001
    for t in range(T):
        a = torch.as_tensor(acts[t], device="cuda:0")
        obs, aid, node, adj, rew, dones, (info, reset, epinfo) = env.step(a, 4)
        st = env.state()
        if t < S_ALL:
            _check_all_envs(ora_all, t, obs, adj, dones, rew, st, "all envs, step %d" % t)
        if t % 20 == 0 or t >= 348:
            assert torch.isfinite(obs).all() and torch.isfinite(node).all() and torch.isfinite(adj).all()
            assert (adj >= 0).all() and (adj <= 3 * 1.60934 + 1e-6).all()
            assert (torch.diagonal(adj, dim1=2, dim2=3) == 0).all()
            assert torch.equal(adj, adj.transpose(2, 3))
            live = ~dones
            spd = st[..., 3]
            assert ((spd >= vmin - 1e-15) & (spd <= vmax + 1e-15) | ~live).all()
            assert (rew >= -40).all() and (rew <= 50).all()
        if t == 349:
            assert bool(reset.all())
        for k, o in zip(sample, oras):
            r = o.step(acts[t][k:k + 1], 4)
            ctx = "env %d step %d" % (k, t)
            np.testing.assert_array_equal(dones[k].cpu().numpy(), r[5][0], err_msg=ctx)
            np.testing.assert_array_equal((adj[k] != 0).cpu().numpy(), r[3][0] != 0, err_msg=ctx)
            np.testing.assert_allclose(obs[k].cpu().numpy(), r[0][0], rtol=0, atol=F32_ATOL, err_msg=ctx)
            np.testing.assert_allclose(rew[k].cpu().numpy(), r[4][0], rtol=1e-6, atol=1e-5, err_msg=ctx)
            np.testing.assert_allclose(st[k].cpu().numpy(), o.envs[0].s, rtol=0, atol=STATE_ATOL, err_msg=ctx)
            if t % 50 == 0:
                np.testing.assert_allclose(node[k].cpu().numpy(), r[2][0], rtol=0, atol=F32_ATOL, err_msg=ctx)
                np.testing.assert_allclose(adj[k].cpu().numpy(), r[3][0], rtol=0, atol=F32_ATOL, err_msg=ctx)
    env.close()


def test_gpu_action_index_out_of_range_is_reported():
    """Index actions outside Discrete(25): host arrays are refused before launch; a device tensor
    is clamped in the kernel (the launch stays in bounds) and reported by check_actions()."""
    import torch
    meta = dict(dynamics_type="double_integrator", num_agents=3, num_landmarks=2, world_size=4,
                episode_length=20, num_env_steps=20 * 4, n_rollout_threads=1, use_safety_filter=False,
                use_masking=True, num_internal_step=1, seed=1, env_seed=1)
    env = _gpu_env(meta, n_envs=4, seed=1, return_numpy=False)
    env.reset(2)
    with pytest.raises(ValueError):
        env.step(np.full((4, 3), 25), 2)
    env.step(torch.zeros((4, 3), dtype=torch.int32, device="cuda:0"), 2)
    env.check_actions()                                   # nothing flagged
    bad = torch.zeros((4, 3), dtype=torch.int32, device="cuda:0")
    bad[2, 1] = -3
    env.step(bad, 2)
    with pytest.raises(ValueError, match="outside"):
        env.check_actions()
    env.check_actions()                                   # the flag was cleared
    env.close()


@pytest.mark.parametrize("kernel", ["wave", "block"])
def test_gpu_collision_forces_reported_never_applied(kernel):
    """World.get_entity_collision_force (core.py:741-774) has no caller, so the step
    must never apply contact forces. With lsm_config.collision_forces the kernel reports the
    per-agent force (LSM_OUT_COLLISION_FORCE) -- compared with the oracle's restatement (itself
    pinned to the reference's own function, tests/test_collision_forces.py) -- while every output
    stays bit-identical to a run without the flag (the default)."""
    ksel = {"workgroup_per_env": 1} if kernel == "block" else None
    meta = dict(dynamics_type="double_integrator", num_agents=8, num_landmarks=2, world_size=4,
                episode_length=30, num_env_steps=30 * 4, n_rollout_threads=1, use_safety_filter=True,
                use_masking=True, num_internal_step=1, seed=13, env_seed=13, collision_forces=True)
    n = 12
    on = _gpu_env(meta, n_envs=n, seed=13, collision_forces=True, kernel_select=ksel)
    off = _gpu_env(meta, n_envs=n, seed=13, kernel_select=ksel)
    assert off.t_cforce is None
    ora = _oracle_for(meta, 13, n)
    for e in (on, off, ora):
        e.reset(4)
    rng = np.random.default_rng(9)
    strong = 0
    for t in range(40):
        if t in (5, 21):   # push agents 1 and 2 of some envs into contact (overlapping discs)
            for k in (0, 3, 7):
                oe = ora.envs[k]
                st = oe.s.copy()
                st[2, :2] = st[1, :2] + np.array([0.07, 0.02])
                st[3, :2] = st[1, :2] + np.array([-0.04, 0.09])
                for env in (on, off):
                    env.set_agent_state(k, st)
                oe.s[:] = st
                oe.calculate_distances()
        a = rng.integers(0, 25, (n, 8))
        g_on, g_off, o = on.step(a, 4), off.step(a, 4), ora.step(a, 4)
        for i in (0, 2, 3, 4, 5):
            np.testing.assert_array_equal(g_on[i], g_off[i], err_msg="t=%d output %d" % (t, i))
        np.testing.assert_array_equal(on.state().cpu().numpy(), off.state().cpu().numpy())
        np.testing.assert_array_equal(g_on[5], o[5])
        f = on.t_cforce.cpu().numpy()
        want = np.stack([e.cforce for e in ora.envs])
        np.testing.assert_allclose(f, want, rtol=1e-12, atol=1e-300, err_msg="t=%d" % t)
        strong += int((np.abs(want) > 1e-3).any())
    assert strong >= 2
    on.close()
    off.close()


@pytest.mark.parametrize("team", ["4", "2", "8", "4s"])
@pytest.mark.parametrize("dyn,N", [("double_integrator", 8), ("airtaxi", 16)])
def test_gpu_team_kernel_resets_match_oracle(dyn, N, team):
    """The team kernel's auto-resets (all of a workgroup's envs, or some, reset in one launch; each
    resetting env's wave draws its scenario with the agents in parallel from the staged MT19937
    stream, crossing block boundaries over successive resets) against the oracle: 10-step episodes,
    75 steps (7 resets per env), envs driven all-done early at different steps so resets do not line
    up, every output. "4s": the staged stream serves only 40 words (lsm_test_set_mt_stage), so every draw runs
    out and takes the cooperative redraw, whose stream state goes back to HBM."""
    import torch
    if dyn == "airtaxi" and team == "8":
        pytest.skip("8 airtaxi envs of 16 agents do not fit one 64-lane agent wave")
    stage = None
    if team == "4s":
        stage = 40
        team = "4"
    ws = 4 if dyn == "double_integrator" else 6
    meta = dict(dynamics_type=dyn, num_agents=N, num_landmarks=2, world_size=ws, episode_length=10,
                num_env_steps=10 * 4, n_rollout_threads=1, use_safety_filter=True, use_masking=True,
                num_internal_step=1, seed=21, env_seed=21)
    n_envs = 15   # a partly filled last workgroup
    env = _gpu_env(meta, n_envs=n_envs, seed=21, kernel_select={"team": int(team)})
    if stage is not None:
        assert env.lib.lsm_test_set_mt_stage(env.h, stage) == 0
    assert env.kernel_name.startswith("rollout_team_kernel<")
    ora = _oracle_for(meta, 21, n_envs)
    g, o = env.reset(4), ora.reset(4)
    np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL)
    rng = np.random.default_rng(31)
    # double integrator: envs driven all-done early (at a goal, zero acceleration) so their
    # resets fall between the episode boundaries of the others
    early = {13: (0, 5), 27: (3,), 44: (7, 8, 14), 58: (1,)} if dyn == "double_integrator" else {}
    for t in range(75):
        a = rng.integers(0, 25, (n_envs, N))
        for k in early.get(t - 1, ()):
            a[k] = 12
        g = env.step(a, 4)
        o = ora.step(a, 4)
        ctx = "%s team %s step %d" % (dyn, team, t)
        np.testing.assert_array_equal(g[5], o[5], err_msg=ctx)
        np.testing.assert_array_equal(env.t_reset.cpu().numpy(), np.array([len(x) > N for x in o[6]]), err_msg=ctx)
        np.testing.assert_array_equal(g[3] != 0, o[3] != 0, err_msg=ctx)
        np.testing.assert_allclose(g[0], o[0], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[2], o[2], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[3], o[3], rtol=0, atol=F32_ATOL, err_msg=ctx)
        np.testing.assert_allclose(g[4], o[4], rtol=1e-6, atol=1e-5, err_msg=ctx)
        st = env.state().cpu().numpy()
        for k, e in enumerate(ora.envs):
            np.testing.assert_allclose(st[k], e.s, rtol=0, atol=STATE_ATOL, err_msg=ctx)
        for k in early.get(t, ()):   # env k all-done at the next step (an off-phase reset)
            s, r = _arrive_all(ora.envs[k])
            env.set_agent_state(k, s, r)
            e = ora.envs[k]
            e.s[:] = s
            e.reached_goal[:] = r
            e.calculate_distances()
    env.close()

