"""Airtaxi integration drift: the kernel's closed-form step (the oracle's integrator='restated') against
the reference's own RK45 states recorded in the airtaxi golden fixtures, over every recorded step
(the longest, ba_cross_n16, is 750 steps). The reference's RK45 right-hand side calls numpy's float64
cos / sin, which on this container's AVX512_SKX CPU dispatch to numpy's vendored SVML kernels (no
libm path to restate), so the kernel integrates in closed form; this measures what that costs.

    python layered-safe-marl_amd/tools/airtaxi_drift.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from golden_replay import fixture_names, layout_fixture_names, layout_for, load, step_ep, table_dict, tables_for
    from oracle.lsm_oracle import OracleEnv
    worst = (0.0, None)
    for name in fixture_names() + layout_fixture_names():
        z, meta = load(name)
        if meta["dynamics_type"] != "airtaxi":
            continue
        vt, tt = tables_for(meta)
        lay = None
        if name in layout_fixture_names():
            lay, m = layout_for(meta)
            rng = np.random.RandomState(meta["env_seed"])
            env = OracleEnv(m, meta["env_seed"], table_dict(vt), table_dict(tt), integrator="restated")
            env.reset(meta["ep"], lay.draw(rng, env.s))
        else:
            env = OracleEnv(meta, meta["env_seed"], table_dict(vt), table_dict(tt), integrator="restated")
            env.reset(meta["ep"])
        if "inject_state" in z.files:
            env.s[:] = z["inject_state"]
            env.reached_goal[:] = z["inject_reached"]
            env.calculate_distances()
        dmax, tmax, flips = 0.0, -1, 0
        per = []
        for t in range(meta["steps"]):
            _, _, _, _, _, dones, _ = env.step(z["act"][t])
            d = float(np.max(np.abs(env.s - z["state"][t])))
            per.append(d)
            if d > dmax:
                dmax, tmax = d, t
            flips += int(np.any(env.done != z["done"][t]) or np.any(env.reached_goal != z["reached"][t]))
            if lay is not None and (t + 1) % meta["episode_length"] == 0:   # GraphDummyVecEnv
                env.reset(step_ep(z, meta, t), lay.draw(rng, env.s))
                env.s[:] = z["t%03d_reset_state" % t]
            elif lay is None and np.all(dones):
                env.reset(step_ep(z, meta, t))
                env.s[:] = z["t%03d_reset_state" % t]   # reset states are drawn, not integrated
        per = np.array(per)
        q = [float(np.max(per[: k])) for k in (100, 250, 500, len(per)) if k <= len(per)]
        print("%-16s steps %4d  max |state - RK45| %.3e at step %d  (by step 100/250/500/end: %s)  "
              "done/reached mismatches %d" % (name, meta["steps"], dmax, tmax,
                                               " ".join("%.1e" % x for x in q), flips))
        if dmax > worst[0]:
            worst = (dmax, name)
    print("worst: %.3e (%s)" % worst)


if __name__ == "__main__":
    main()
