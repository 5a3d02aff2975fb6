"""Every env of a full-size GPU run against the oracle (test infrastructure).

The full-size parity tests (BASELINE configs 3 and 4) compare ALL envs of a launch with the oracle
over the first steps after a reset, on the full-shape synthetic HJ / TTR tables the bench times
(``lsm.hj_tables.default_tables``, ``bench.py``). One oracle env-step costs ~4 ms (DI, N = 8) to
~36 ms (airtaxi, N = 16) on one core, so the envs are split over worker processes. Workers are
started with the "spawn" method: fresh interpreters that never touch the GPU (the test process has
initialised it; forked children would inherit its device handles). Each worker rebuilds the tables
(deterministic, ~2 s) and runs its envs one at a time (an oracle env copies its 20-25 MB value table,
as HjDataHandle shifts it in place, so thousands cannot be alive at once).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tables(dyn):
    sys.path.insert(0, os.path.join(ROOT, "layered-safe-marl_amd"))
    from lsm import hj_tables
    from golden_replay import table_dict
    vt, tt = hj_tables.default_tables(dyn)
    return table_dict(vt), table_dict(tt)


def _chunk(job):
    meta, seed, k0, k1, ep, actions = job
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle.lsm_oracle import OracleVecEnv
    vt, tt = _tables(meta["dynamics_type"])
    f32 = lambda x: np.asarray(x, dtype=np.float32)
    S = actions.shape[1]
    out = dict(reset_obs=[], reset_adj=[], state=[], obs=[], adj=[], dones=[], rew=[])
    for k in range(k0, k1):
        ora = OracleVecEnv(meta, 1, seed=seed, value_table=vt, ttr_table=tt, integrator="restated",
                           seed_offset=k)
        r = ora.reset(ep)
        out["reset_obs"].append(f32(r[0][0]))
        out["reset_adj"].append(np.packbits(np.asarray(r[3][0]) != 0))
        st, ob, ad, dn, rw = [], [], [], [], []
        for s in range(S):
            o = ora.step(actions[k - k0, s][None], ep)
            ob.append(f32(o[0][0]))
            ad.append(np.packbits(np.asarray(o[3][0]) != 0))
            dn.append(np.asarray(o[5][0], dtype=bool))
            rw.append(f32(o[4][0]))
            st.append(ora.envs[0].s.copy())
        out["obs"].append(np.stack(ob))
        out["adj"].append(np.stack(ad))
        out["dones"].append(np.stack(dn))
        out["rew"].append(np.stack(rw))
        out["state"].append(np.stack(st))
        del ora
    return k0, {k: np.stack(v) for k, v in out.items()}


def workers_for_box(cap=16):
    """Worker processes: the job's CPU share (the affinity set, capped by a cgroup quota; a GPU box
    lends each GPU a share of a larger host), at most `cap`."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(period))))
    except Exception:
        pass
    return max(1, min(cap, n))


def run_all_envs(meta, seed, n_envs, ep, actions, workers=None):
    """Oracle of envs [0, n_envs) (seed + 1000 k): reset(ep), then actions[k, s] for s < S.
    actions: int [n_envs, S, N]. Returns dict of arrays with a leading env axis: reset_obs f32
    [n, N, OBS], reset_adj packed bits, then per step: obs, adj (packed bits of adj != 0), dones,
    rew (f32), state (f64 [n, S, N, 4])."""
    workers = workers or workers_for_box()
    edges = np.linspace(0, n_envs, workers * 4 + 1).astype(int)   # several chunks per worker
    jobs = [(dict(meta), seed, int(a), int(b), ep, np.ascontiguousarray(actions[a:b]))
            for a, b in zip(edges[:-1], edges[1:]) if b > a]
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        parts = sorted(pool.map(_chunk, jobs), key=lambda x: x[0])
    return {k: np.concatenate([p[1][k] for p in parts]) for k in parts[0][1]}
