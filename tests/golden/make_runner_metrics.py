#!/usr/bin/env python
"""Record the runner's metric functions FROM THE REFERENCE ITSELF (build container only).

SURVEY.md §8(f) row 3: the per-step info dicts become the runner's logged metrics through
``Runner.process_infos`` (onpolicy/runner/shared/base_runner.py:222-301) and ``Runner.log_env``
(:317-331: ``np.mean`` of each non-empty list). This script drives K reference envs
(``GraphMPEEnv`` seeded seed + 1000 k, the factory's rule) with GraphSubprocVecEnv's worker
semantics (auto-reset on all-done, ep_info appended, env_wrappers.py:851-874), calls the
reference's own two functions on the envs' info lists every step, and stores their outputs:

  keys [n_keys]              process_infos keys, sorted
  vals [T][n_keys][K]        the lists (NaN-padded; lens [n_keys] = K or 0)
  log_keys / log_vals [T][.] what log_env hands the writer ({k: np.mean(v)} for non-empty v)
  act [T][K][N]              the actions (indices), so a GPU handle with the same seeds replays it

``process_infos`` reads ``self.dt``, which the reference runner never sets (its "NOTE: Hardcoding
`dt`"): the stand-in runner sets it to the scenario's dt (0.1 for the double integrator).
``wandb`` / ``tensorboardX`` (absent here) are stubs in oracle/ref_stubs; log_env runs with
use_wandb=False and a recording writer.

Usage:  python tests/golden/make_runner_metrics.py
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "layered-safe-marl_amd"))

from oracle import ref_harness  # noqa: E402
from lsm import hj_tables  # noqa: E402

K, N, EPL, STEPS, SEED, EP = 4, 5, 30, 45, 41, 4


class _Writer:
    def __init__(self):
        self.rows = {}

    def add_scalars(self, k, d, step):
        self.rows[k] = float(d[k])


def main():
    if not ref_harness.reference_available():
        raise SystemExit("reference not available here")
    work = tempfile.mkdtemp(prefix="lsm_ref_")
    args = ref_harness.default_args(num_agents=N, episode_length=EPL, num_env_steps=EPL * 4,
                                    use_safety_filter=True, n_rollout_threads=K)
    ref_harness.write_data_files(work, di_table=hj_tables.synthetic_di_stored((31, 31, 21, 21)))
    # each GraphSubprocVecEnv worker is its own process with its own global numpy stream (seeded by
    # env.seed); in one process each env's stream state is swapped in around its calls
    envs, streams = [], []
    for k in range(K):
        envs.append(ref_harness.make_reference_env(args, work, SEED + 1000 * k))
        streams.append(np.random.get_state())

    def call(k, fn, *a):
        np.random.set_state(streams[k])
        r = ref_harness.run_in(work, fn, *a)
        streams[k] = np.random.get_state()
        return r

    from onpolicy.runner.shared.base_runner import Runner
    fake = types.SimpleNamespace(num_agents=N, all_args=args, dt=envs[0].world.dt, use_wandb=False)
    for k, e in enumerate(envs):
        call(k, e.reset, EP)
    rng = np.random.default_rng(5)
    acts, vals, logs, keys, log_keys = [], [], [], None, None
    resets = 0
    for t in range(STEPS):
        a = rng.integers(0, 25, (K, N))
        infos = []
        for k, e in enumerate(envs):
            obs, aid, node, adj, rew, done, info = call(k, e.step, list(ref_harness.one_hot_actions(a[k])))
            info = list(info)
            if np.all(done):   # GraphSubprocVecEnv worker: auto-reset, ep_info appended
                *_, ep_info = call(k, e.reset, EP)
                info.append(ep_info)
                resets += 1
            infos.append(info)
        env_infos = Runner.process_infos(fake, infos)
        fake.writter = _Writer()
        Runner.log_env(fake, env_infos, t)
        if keys is None:
            keys = sorted(env_infos)
            log_keys = sorted(fake.writter.rows)
        assert sorted(env_infos) == keys and sorted(fake.writter.rows) == log_keys
        v = np.full((len(keys), K), np.nan)
        for i, k in enumerate(keys):
            v[i, :len(env_infos[k])] = env_infos[k]
        acts.append(a)
        vals.append(v)
        logs.append([fake.writter.rows[k] for k in log_keys])
    lens = np.array([len(env_infos[k]) for k in keys])
    path = os.path.join(HERE, "runner_metrics.npz")
    np.savez_compressed(path, keys=np.array(keys), vals=np.array(vals), lens=lens, log_keys=np.array(log_keys),
                        log_vals=np.array(logs), act=np.array(acts),
                        meta=np.array(repr(dict(num_agents=N, episode_length=EPL, num_env_steps=EPL * 4, seed=SEED,
                                                ep=EP, n_envs=K, dt=float(fake.dt), use_safety_filter=True,
                                                dynamics_type="double_integrator", world_size=4))))
    print("wrote", path, os.path.getsize(path) // 1024, "KB; keys", len(keys), "log keys", len(log_keys),
          "auto-resets", resets)


if __name__ == "__main__":
    main()
