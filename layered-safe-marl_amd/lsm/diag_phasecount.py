"""Diagnostic: per-phase dynamic instruction counts of rollout_kernel.

Runs the stamps build with LSM_STOP_AFTER=k (the step ends right after phase k) for
k = 0..10, REPS launches each, in a fixed order; run it under
``rocprofv3 --pmc SQ_INSTS_VALU ...`` and reduce with ``lsm.diag_phasecount --reduce DIR``:
counter(k) - counter(k-1) = what phase k issues.

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d D -o run \
        --output-format csv -- python3 -m lsm.diag_phasecount
    python -m lsm.diag_phasecount --reduce D

``--team``: the team kernel's stops (lsm_team.h TSTOP): 1 record in LDS, 2 pair lookups, 3 end of
phase A, 4 end of B, 5 end of C, 6 end of D, 7 the whole step (E).
"""
from __future__ import annotations

import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
STOPS = list(range(0, 12))
TEAM_STOPS = list(range(1, 8))
TEAM_PHASES = ["A record", "A pairs", "A filter prep", "B agent wave", "C distances", "D reward/info",
               "E outputs"]
REPS = 4
WARM = 6


def run(config, team=False):
    from .diag_stamps import STAMP_LIB
    os.environ["LSM_LIB"] = STAMP_LIB
    import torch
    import ctypes as C
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import bench
    from . import capi, hj_tables
    from .vec_env import GpuGraphVecEnv
    c = bench.CONFIGS[config]
    args = bench.make_args(c)
    vt, tt = hj_tables.default_tables(c["dynamics_type"]) if (c["use_safety_filter"] or
                                                              c["dynamics_type"] != "double_integrator") else (None, None)
    env = GpuGraphVecEnv(args, num_envs=c["envs"], device="cuda:0", value_table=vt, ttr_table=tt,
                         return_numpy=False, build_infos=False)
    N = c["num_agents"]
    env.reset(4)
    gen = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(WARM):   # full steps: a mid-episode state
        env.step(torch.randint(0, 25, (c["envs"], N), device="cuda:0", dtype=torch.int32, generator=gen), 4)
    for k in (TEAM_STOPS if team else STOPS):
        os.environ["LSM_STOP_AFTER"] = str(k if not (team and k == 7) else -1)
        for _ in range(REPS):
            env.step(torch.randint(0, 25, (c["envs"], N), device="cuda:0", dtype=torch.int32, generator=gen), 4)
    torch.cuda.synchronize()
    os.environ.pop("LSM_STOP_AFTER")
    env.close()


def reduce(d, config=3, team=False):
    import statistics
    from .pmc import _rows
    per = {}
    for r in _rows(d, "counter_collection.csv"):
        if ("lsm::rollout" if team else "rollout_kernel") not in r.get("Kernel_Name", ""):
            continue
        k = int(r.get("Dispatch_Id") or 0)
        per.setdefault(k, {})
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    # launches: reset (1) + WARM full steps + len(STOPS) * REPS
    ids = ids[1 + WARM:]
    stops = TEAM_STOPS if team else STOPS
    assert len(ids) == len(stops) * REPS, len(ids)
    names = sorted(per[ids[0]])
    waves = None
    cum = {}
    for i, k in enumerate(stops):
        grp = ids[i * REPS:(i + 1) * REPS]
        cum[k] = {n: statistics.fmean(per[g][n] for g in grp) for n in names}
    from .diag_stamps import PHASES
    print("%-14s" % "phase" + "".join("%16s" % n for n in names) + "   (per wave)")
    prev = {n: 0.0 for n in names}
    print("(per wave: counters / envs; the team kernel's agent-wave phases B and D run on one wave "
          "of each 4, so their per-wave share is a quarter of that wave's)")
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import bench
    nw = float(bench.CONFIGS[config]["envs"])
    for k in stops:
        if team:
            label = TEAM_PHASES[k - 1]
        else:
            label = "start" if k == 0 else (PHASES[k - 1] if k <= len(PHASES) else "store")
        print("%-14s" % label + "".join("%16.0f" % ((cum[k][n] - prev[n]) / nw) for n in names))
        prev = cum[k]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--reduce", default=None)
    ap.add_argument("--team", action="store_true")
    a = ap.parse_args()
    if a.reduce:
        reduce(a.reduce, a.config, a.team)
    else:
        run(a.config, a.team)
