"""Diagnostic: per-phase dynamic instruction counts of rollout_kernel.

Runs the stamps build with LSM_STOP_AFTER=k (the step ends right after phase k) for
k = 0..10, REPS launches each, in a fixed order; run it under
``rocprofv3 --pmc SQ_INSTS_VALU ...`` and reduce with ``lsm.diag_phasecount --reduce DIR``:
counter(k) - counter(k-1) = what phase k issues.

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d D -o run \
        --output-format csv -- python3 -m lsm.diag_phasecount
    python -m lsm.diag_phasecount --reduce D
"""
from __future__ import annotations

import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
STOPS = list(range(0, 12))
REPS = 4
WARM = 6


def run(config):
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
    for k in STOPS:
        os.environ["LSM_STOP_AFTER"] = str(k)
        for _ in range(REPS):
            env.step(torch.randint(0, 25, (c["envs"], N), device="cuda:0", dtype=torch.int32, generator=gen), 4)
    torch.cuda.synchronize()
    os.environ.pop("LSM_STOP_AFTER")
    env.close()


def reduce(d, config=3):
    import statistics
    from .pmc import _rows
    per = {}
    for r in _rows(d, "counter_collection.csv"):
        if "rollout_kernel" not in r.get("Kernel_Name", ""):
            continue
        k = int(r.get("Dispatch_Id") or 0)
        per.setdefault(k, {})
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    # launches: reset (1) + WARM full steps + len(STOPS) * REPS
    ids = ids[1 + WARM:]
    assert len(ids) == len(STOPS) * REPS, len(ids)
    names = sorted(per[ids[0]])
    waves = None
    cum = {}
    for i, k in enumerate(STOPS):
        grp = ids[i * REPS:(i + 1) * REPS]
        cum[k] = {n: statistics.fmean(per[g][n] for g in grp) for n in names}
    from .diag_stamps import PHASES
    print("%-14s" % "phase" + "".join("%16s" % n for n in names) + "   (per wave)")
    prev = {n: 0.0 for n in names}
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import bench
    nw = float(bench.CONFIGS[config]["envs"])
    for k in STOPS:
        label = "start" if k == 0 else (PHASES[k - 1] if k <= len(PHASES) else "store")
        print("%-14s" % label + "".join("%16.0f" % ((cum[k][n] - prev[n]) / nw) for n in names))
        prev = cum[k]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--reduce", default=None)
    a = ap.parse_args()
    if a.reduce:
        reduce(a.reduce, a.config)
    else:
        run(a.config)
