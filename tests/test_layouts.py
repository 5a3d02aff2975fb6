"""Evaluation layouts (lsm/layouts.py) and RealisticScenario departures against the reference.

Fixtures ev_* / ba_* were recorded by tests/golden/make_golden.py from the stub-imported
reference: navigation_graph_safe_eval (eval_scenario_type set per fixture) and the Bay Area maps
(RealisticScenario with departure timers; a blank map image of the recorded size stands in for
the absent picture, whose size is all the reference reads), with GraphDummyVecEnv semantics
(reset after every episode_length steps, scripts/eval_mpe.py).

* lsm.layouts draws each reset's layout (agent states, landmarks, departure timers, init
  headings) from the env's numpy stream exactly as the reference's scenario function;
* the oracle, given those layouts, replays every step bit for bit (integrator 'rk45' = the
  reference's own solve_ivp), including departures, waiting freezes and the recursive goal update.
"""
import numpy as np
import pytest

from golden_replay import EPKEYS, INFOKEYS, adj_bits, layout_fixture_names, layout_for, load, step_ep, \
    table_dict, tables_for

NAMES = layout_fixture_names()


def _reset_keys(z):
    """(step after which the reset happened or -1, state key, landmark key, departure key)."""
    out = [(-1, "reset0_state", "reset0_lm", "reset0_dep")]
    for t in range(len(z["act"])):
        if "t%03d_reset_state" % t in z.files:
            out.append((t, "t%03d_reset_state" % t, "t%03d_reset_lm" % t, "t%03d_reset_dep" % t))
    return out


@pytest.mark.parametrize("name", NAMES)
def test_layout_draws_match_reference(name):
    z, meta = load(name)
    lay, _ = layout_for(meta)
    rng = np.random.RandomState(meta["env_seed"])
    prev = np.zeros((meta["num_agents"], 4))
    for t, ks, kl, kd in _reset_keys(z):
        if t >= 0:
            prev = z["state"][t]
        d = lay.draw(rng, prev)
        np.testing.assert_array_equal(d.state, z[ks], err_msg="%s reset after %d" % (name, t))
        np.testing.assert_array_equal(d.landmarks, z[kl], err_msg="%s reset after %d" % (name, t))
        if lay.departures:
            np.testing.assert_array_equal(d.departed, z[kd][:, 0])
            np.testing.assert_array_equal(d.timer, z[kd][:, 1])
            np.testing.assert_array_equal(d.init_theta, z[kd][:, 2])
        else:
            assert d.departed is None and np.all(z[kd][:, 0] == 1.0)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_layouts(name):
    from oracle.lsm_oracle import OracleEnv
    z, meta = load(name)
    lay, m = layout_for(meta)
    vt, tt = tables_for(meta)
    env = OracleEnv(m, meta["env_seed"], table_dict(vt), table_dict(tt), integrator="rk45")
    rng = np.random.RandomState(meta["env_seed"])
    obs, aid, node, adj, info = env.reset(meta["ep"], lay.draw(rng, env.s))
    np.testing.assert_array_equal(np.array(obs), z["reset0_obs"])
    np.testing.assert_array_equal(np.array(node, dtype=np.float32), z["reset0_node"])
    np.testing.assert_array_equal(np.array(adj, dtype=np.float32), z["reset0_adj"])
    np.testing.assert_array_equal(env.edge_list, z["reset0_edges"])
    n_reset = 1
    for t in range(meta["steps"]):
        obs, aid, node, adj, rew, dones, infos = env.step(z["act"][t])
        ctx = "%s step %d" % (name, t)
        np.testing.assert_array_equal(env.s, z["state"][t], err_msg=ctx)
        np.testing.assert_array_equal(env.reached_goal, z["reached"][t], err_msg=ctx)
        np.testing.assert_array_equal(env.done, z["done"][t], err_msg=ctx)
        np.testing.assert_array_equal(env.departed, z["departed"][t], err_msg=ctx)
        np.testing.assert_array_equal(dones, z["dones"][t], err_msg=ctx)
        np.testing.assert_array_equal(np.array(rew, dtype=np.float64), z["rew"][t], err_msg=ctx)
        np.testing.assert_array_equal(np.array(obs), z["obs"][t], err_msg=ctx)
        np.testing.assert_array_equal(adj_bits(adj), z["adj_bits"][t], err_msg=ctx)
        np.testing.assert_array_equal(env.min_rel_dist, z["minrel"][t], err_msg=ctx)
        np.testing.assert_array_equal(env.safety_filtered, z["sfilt"][t], err_msg=ctx)
        np.testing.assert_array_equal(env.deconflicting, z["decon"][t], err_msg=ctx)
        np.testing.assert_array_equal(
            np.array([[inf[k] for k in INFOKEYS] for inf in infos], dtype=np.float64), z["info_num"][t],
            err_msg=ctx)
        key = "t%03d_node" % t
        if key in z.files:
            np.testing.assert_array_equal(np.array(node, dtype=np.float32), z[key], err_msg=ctx)
            np.testing.assert_array_equal(np.array(adj, dtype=np.float32), z["t%03d_adj" % t], err_msg=ctx)
        if (t + 1) % meta["episode_length"] == 0:   # GraphDummyVecEnv: the render loop resets
            obs, aid, node, adj, info = env.reset(step_ep(z, meta, t), lay.draw(rng, env.s))
            assert z["resets_t"][n_reset] == t + 1
            np.testing.assert_array_equal([info[k] for k in EPKEYS], z["resets_info"][n_reset], err_msg=ctx)
            np.testing.assert_array_equal(env.s, z["t%03d_reset_state" % t], err_msg=ctx)
            np.testing.assert_array_equal(np.array(obs), z["t%03d_reset_obs" % t], err_msg=ctx)
            np.testing.assert_array_equal(np.array(node, dtype=np.float32), z["t%03d_reset_node" % t])
            n_reset += 1
    assert n_reset == len(z["resets_t"])


def test_layout_fixtures_exercise_departures():
    """The Bay Area fixtures hold undeparted agents, departures and waiting freezes."""
    for name in ("ba_merge_n8", "ba_cross_n4"):
        z, meta = load(name)
        dep = z["departed"]
        assert not dep[0].all() and dep[-1].any(), name
        assert (np.diff(dep.astype(int), axis=0) == 1).any(), name   # a departure happens mid-run


def test_layout_rejections():
    from lsm import layouts
    with pytest.raises(ValueError):
        layouts.ScenarioLayout("bayarea_merge", "double_integrator", 8, image_size=(100, 100))
    with pytest.raises(ValueError):
        layouts.ScenarioLayout("bayarea_merge", "airtaxi", 8)           # map size needed
    with pytest.raises(ValueError):
        layouts.ScenarioLayout("eval:left_to_right_cross", "airtaxi", 2)   # reference reward raises
    lay = layouts.ScenarioLayout("eval:circular_config", "airtaxi", 4, num_landmarks=2)
    with pytest.raises(ValueError):   # the layout sets N landmarks, the env has 2N
        lay.draw(np.random.RandomState(0))
