"""Runner-side metrics straight from the device info tensor.

The reference runner turns every env's info dicts into per-agent lists
(``BaseRunner.process_infos``, onpolicy/runner/shared/base_runner.py:222-301) and logs their
means (``log_env``, :317-331). Here both work on the ``[n][N][LSM_INFO_FIELDS]`` float64
tensor the kernel writes:

* ``process_infos(info, ...)`` returns the same dict of lists (one host copy of the tensor,
  no per-env dicts). It is equal, key for key and element for element, to the reference
  function applied to ``GpuGraphVecEnv``'s info dicts (tests/test_metrics.py).
* ``log_means(info, ...)`` keeps the reduction on the device and returns the per-key means
  that ``log_env`` computes with ``np.mean`` (a float64 device mean; ulp-level vs numpy's
  pairwise sum, logging only).

The names are the reference's; keys whose info field the navigation_graph_safe scenario never
sets (``formation_dist``) stay empty lists, as in the reference.
"""
from __future__ import annotations

from . import capi

_F = {k: j for j, k in enumerate(capi.INFO_FIELDS)}

# (reference log key suffix, how to get the per-env value column)
_PLAIN = (
    ("individual_rewards", "individual_reward"),
    ("min_time_to_goal", "Min_time_to_goal"),
    ("dist_to_goal", "Dist_to_goal"),
    ("num_agent_collisions", "Num_agent_collisions"),
    ("distance_mean", "Distance_mean"),
    ("distance_variance", "Distance_variance"),
    ("dists_traveled", "Dists_traveled"),
    ("time_taken", "Time_req_to_goal"),      # 'Time_taken' = world.times_required (info_callback)
    ("time_mean", "Time_mean"),
    ("time_variance", "Time_stddev"),         # the reference logs Time_stddev under this name
)
KEYS = ("individual_rewards", "time_to_goal", "min_time_to_goal", "dist_to_goal", "num_agent_collisions",
        "num_obstacle_collisions", "distance_mean", "distance_variance", "mean_variance", "dists_traveled",
        "time_taken", "formation_dist", "time_mean", "time_variance", "time_mn_by_stddev")


def _columns(x, a, episode_length, dt, xp):
    """Per-key value columns over envs for agent a (x: [n][N][F] array of module xp)."""
    col = lambda name: x[:, a, _F[name]]
    out = {k: col(f) for k, f in _PLAIN}
    tr = col("Time_req_to_goal")
    out["time_to_goal"] = xp.where(tr == -1, episode_length * dt, tr)
    out["num_obstacle_collisions"] = col("Num_agent_collisions") * 0.0   # no obstacles: 0.0 each
    out["mean_variance"] = col("Distance_mean") / (col("Distance_variance") + 0.0001)
    out["time_mn_by_stddev"] = col("Time_mean") / (col("Time_stddev") + 0.0001)
    return out


def process_infos(info, num_agents: int, episode_length: int, dt: float) -> dict:
    """``BaseRunner.process_infos`` on the info tensor: {'agent{i}/<key>': [value per env]}."""
    import numpy as np
    x = info.cpu().numpy() if hasattr(info, "cpu") else np.asarray(info)
    out = {}
    for a in range(num_agents):
        cols = _columns(x, a, episode_length, dt, np)
        for k in KEYS:
            out["agent%d/%s" % (a, k)] = [] if k == "formation_dist" else [float(v) for v in cols[k]]
    return out


def log_means(info, num_agents: int, episode_length: int, dt: float) -> dict:
    """``log_env``'s per-key means, reduced on the device (one float per key; empty keys skipped)."""
    import torch
    out = {}
    for a in range(num_agents):
        cols = _columns(info, a, episode_length, dt, torch)
        for k in KEYS:
            if k != "formation_dist":
                out["agent%d/%s" % (a, k)] = cols[k].mean()
    keys = list(out)
    vals = torch.stack([out[k] for k in keys]).cpu().tolist()   # one transfer for all keys
    return dict(zip(keys, vals))
