"""Model of ``summary_lane`` (csrc/lsm_rollout.hip): the episode summary's eight outputs computed on
eight lanes at once, output k on lane k, each lane summing its own stats row (a per-lane LDS address;
the two ratio outputs divide by the travel time, the others by nothing). This restates that row and
denominator mapping in numpy and checks it against the oracle's ``_save_summary``
(save_summary_of_episode, environment.py:895-911) on random statistics, bit for bit. CPU only.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.lsm_oracle import OracleEnv

KEYS = ["travel_time_mean", "travel_distance_mean", "done_percentage", "num_reached_goal_mean",
        "conflict_percentage", "min_distance_mean", "min_distance_min", "multiple_engagement_percentage"]
TTR = dict(lo=[0] * 4, hi=[1] * 4, shape=(2, 2, 2, 2), values=np.zeros((2, 2, 2, 2), np.float32), ttr_max=1.0)


def summary_lane_model(stats, rpost, dt, coord_range):
    """stats: [6][N] rows tl td dn cf md mu (the record's layout); rpost: reached counts (int)."""
    out = []
    N = stats.shape[1]
    for k in range(8):
        row = k if k < 3 else (0 if k == 3 else (k - 1 if k <= 5 else k - 2))
        x = rpost.astype(np.float64) if k == 3 else stats[row].copy()
        if k in (4, 7):
            x = x / np.where(stats[0] == 0, 1.0, stats[0])
        o = np.mean(x)   # np_sum_acc / N: numpy's pairwise order
        if k == 0:
            o = dt * o
        if k == 6:
            o = stats[4][0]
            for i in range(1, N):
                o = stats[4][i] if stats[4][i] < o else o
        if k in (5, 6) and o == np.inf:
            o = coord_range
        out.append(o)
    return out


@pytest.mark.parametrize("n", [3, 8, 16, 64])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_summary_lane_model_matches_oracle(n, seed):
    rng = np.random.default_rng(seed)
    args = dict(dynamics_type="double_integrator", num_agents=n, num_landmarks=2, world_size=4,
                episode_length=250, num_env_steps=1000, n_rollout_threads=1, use_safety_filter=False)
    ora = OracleEnv(args, 0, value_table=None, ttr_table=TTR)
    tl = rng.integers(0, 250, n).astype(np.float64)
    tl[rng.random(n) < 0.2] = 0.0
    md = rng.random(n) * 3
    md[rng.random(n) < 0.3] = np.inf
    if seed == 2:
        md[:] = np.inf
    stats = np.stack([tl, rng.random(n) * 9, (rng.random(n) < 0.5).astype(float),
                      rng.integers(0, 30, n).astype(float), md, rng.integers(0, 20, n).astype(float)])
    rpost = rng.integers(0, 3, n)
    ora.stats = dict(travel_length=stats[0].copy(), travel_distance=stats[1].copy(), done=stats[2].copy(),
                     reached=rpost.astype(np.float64), conflict=stats[3].copy(), min_distance=stats[4].copy(),
                     multiple=stats[5].copy())
    ora._save_summary()
    got = summary_lane_model(stats, rpost, ora.dt, ora.coordination_range)
    want = [ora.prev[k] for k in KEYS]
    assert got == want
