"""Diagnostic: per-phase cycle breakdown of rollout_kernel from in-kernel s_memtime stamps.

Uses a separate build (``-DLSM_STAMPS`` -> ``csrc/liblsm_rollout_stamps.so``); the
product library never executes a stamp. Read the SHARES, not absolute times (the
stamps' barriers forbid overlap the real kernel has).

    python -m lsm.diag_stamps [--config 3] [--steps 40]
"""
from __future__ import annotations

import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
STAMP_LIB = os.path.join(CSRC, "liblsm_rollout_stamps.so")
PHASES = ["load", "decode", "filter-pairs", "filter-ego", "integrate", "dist+minrel", "obs+reward",
          "info", "stats+dones", "emit-graph"]


def build_stamps():
    from . import build
    build.build_variant("stamps", ["LSM_STAMPS"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--envs", type=int, default=0)
    ap.add_argument("--team", action="store_true",
                    help="the team kernel's stamps (lsm_team.h): phases A-E, work vs barrier wait")
    ap.add_argument("--lib", default="", help="another stamps build (csrc/liblsm_rollout_<name>.so)")
    ap.add_argument("--kernel-select", default="",
                    help="lsm_kernel_select fields, e.g. team=2 (include/lsm_rollout.h; default: the library's choice)")
    ap.add_argument("--pick", default="",
                    help="comma-separated step indices to keep (e.g. 250: the step after the first "
                         "episode boundary at episode length 250); default every step from 10 on")
    a = ap.parse_args()
    if a.build or not os.path.exists(STAMP_LIB):
        build_stamps()
        if a.build:
            return
    os.environ["LSM_LIB"] = os.path.join(CSRC, a.lib) if a.lib else STAMP_LIB
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import bench
    from . import capi, hj_tables
    from .vec_env import GpuGraphVecEnv
    import ctypes as C
    c = bench.CONFIGS[a.config]
    args = bench.make_args(c)
    vt, tt = hj_tables.default_tables(c["dynamics_type"]) if (c["use_safety_filter"] or
                                                              c["dynamics_type"] != "double_integrator") else (None, None)
    n_envs = a.envs or c["envs"]
    ksel = bench.parse_kernel_select(a.kernel_select)
    env = GpuGraphVecEnv(args, num_envs=n_envs, device="cuda:0", value_table=vt, ttr_table=tt,
                         return_numpy=False, build_infos=False, adj_layout=c.get("adj_layout", "reference"),
                         kernel_select=ksel)
    G = ksel.get("team", 4) if ksel and ksel.get("team", -1) > 0 else 4
    stamps = torch.zeros((n_envs, 40), dtype=torch.int64, device="cuda:0")   # LSM_NSTAMP
    capi.check(env.lib.lsm_bind_output(env.h, capi.OUT_DEBUG_STAMPS, C.c_void_p(stamps.data_ptr()),
                                       stamps.numel() * 8), env.h)
    env.reset(4)
    N = c["num_agents"]
    acc, rt, tstamps, tstamps12 = [], [], [], []
    for t in range(a.steps + 10):
        act = torch.randint(0, 25, (n_envs, N), device="cuda:0", dtype=torch.int32)
        env.step(act, 4)
        torch.cuda.synchronize()
        picks = {int(x) for x in a.pick.split(",") if x}
        if (t >= 10 and not picks) or t in picks:
            raw = stamps.cpu().numpy()
            hw = raw[:, 15].astype(np.uint64)   # HW_ID | XCC_ID << 32 of this step's waves
            s = raw.astype(np.float64)
            tstamps.append(s[:, :9].copy())
            tstamps12.append(s[:, :40].copy())
            stamps.zero_()
            acc.append(np.diff(s[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10]], axis=1))
            t0 = s[:, 13].min()
            rt.append(np.stack([s[:, 13] - t0, s[:, 14] - t0], axis=1) * 10.0)   # ns (100 MHz)
        else:
            stamps.zero_()   # a picked step sees only its own stamps
    if a.team:
        # 0 start, 6 A done, 1 after W1, 2 after W2 (B), 7 C done, 3 after W3, 8 D done, 4 after W4, 5 end
        segs = [("A work", 0, 6), ("A wait", 6, 1), ("B (agent wave)", 1, 2), ("C work", 2, 7),
                ("C wait", 7, 3), ("D own work", 3, 8), ("D wait", 8, 4), ("E", 4, 5)]
        allst = np.concatenate(tstamps, axis=0)
        print("team phase          median cycles   share   p90")
        tot = np.median(allst[:, 5] - allst[:, 0])
        for name, i, j in segs:
            v = allst[:, j] - allst[:, i]
            print("%-18s %12.0f   %5.1f%%  %8.0f" % (name, np.median(v), 100 * np.median(v) / tot,
                                                      np.percentile(v, 90)))
        print("%-18s %12.0f" % ("total", tot))
        # per wave slot (env % G): phase medians and end time; and the slowest 2 % of waves
        slots = np.concatenate([np.arange(x.shape[0]) % G for x in tstamps])
        rts = np.concatenate([x[:, 1] for x in rt])   # end (ns since the launch's first wave start)
        print("slot   " + " ".join("%10s" % n[:10] for n, _, _ in segs) + "      end us")
        for w in range(G):
            m = slots == w
            print("%-6d " % w + " ".join("%10.0f" % np.median(allst[m, j] - allst[m, i]) for _, i, j in segs) +
                  "  %10.2f" % (np.median(rts[m]) / 1e3))
        late = rts >= np.percentile(rts, 98)
        print("late2% " + " ".join("%10.0f" % np.median(allst[late, j] - allst[late, i]) for _, i, j in segs) +
              "  %10.2f  slots %s" % (np.median(rts[late]) / 1e3, np.bincount(slots[late], minlength=G).tolist()))
        ag = np.concatenate(tstamps12, axis=0)
        for name, i, j in [("A record", 0, 12), ("A decode+pairs", 12, 16), ("A argmin+grad", 16, 17),
                           ("A: to pair loop", 12, 30), ("A: pair loop", 30, 16), ("A: argmins", 16, 32),
                           ("A: gradient", 32, 17),
                           ("A decode..prep", 12, 6), ("B filter", 1, 9),
                           ("B integrate", 9, 2), ("B: to RK45 start", 9, 29), ("B: initial step", 29, 27),
                           ("B: RK45 steps", 27, 28), ("B: clamp+sync", 28, 2), ("D reward", 3, 10),
                           ("D info", 10, 11), ("D rows+stats", 11, 8), ("E info/dones", 4, 18),
                           ("E graph+record", 18, 5), ("R prep", 18, 19), ("R prep->draws", 19, 20),
                           ("R finish+dist", 20, 21), ("R emit", 21, 22), ("R store", 22, 5),
                           ("R draw: states", 19, 23), ("R draw: blocks+chain", 23, 24),
                           ("R draw: agents+keep", 24, 25), ("R draw: tail", 25, 26), ("R draw->20", 26, 20)]:
            v = ag[:, j] - ag[:, i]
            v = v[(ag[:, i] != 0) & (ag[:, j] != 0)]
            print("%-18s %12.0f   (agent-wave rows: %d)" % (name, np.median(v), len(v)))
        acc = [np.zeros((1, 10))]
    d = np.concatenate(acc, axis=0)
    med = np.median(d, axis=0)
    tot = med.sum()
    print("phase               median cycles   share")
    for name, v in zip(PHASES, med):
        print("%-18s %12.0f   %5.1f%%" % (name, v, 100 * v / tot))
    print("%-18s %12.0f" % ("total", tot))
    r = np.stack(rt)   # [steps][envs][2] ns since the first wave started
    q = lambda x: "p0 %.2f  p10 %.2f  p50 %.2f  p90 %.2f  p100 %.2f us" % tuple(
        np.percentile(x, [0, 10, 50, 90, 100]) / 1e3)
    print("wave start  ", q(r[..., 0].ravel()))
    print("wave end    ", q(r[..., 1].ravel()))
    print("wave life   ", q((r[..., 1] - r[..., 0]).ravel()))
    xcc = (hw >> np.uint64(32)) & np.uint64(0xf)
    hid = hw & np.uint64(0xffffffff)
    simd = (hid >> np.uint64(4)) & np.uint64(3)
    cu = (hid >> np.uint64(8)) & np.uint64(0xf)
    se = (hid >> np.uint64(13)) & np.uint64(0x7)
    life = (r[..., 1] - r[..., 0]).mean(axis=0) / 1e3   # per env, mean over steps (us)
    print("mean wave life by XCC: " + " ".join("%d:%.1f" % (x, life[xcc == x].mean())
                                                  for x in np.unique(xcc)))
    print("mean wave life by SE:  " + " ".join("%d:%.1f" % (x, life[se == x].mean()) for x in np.unique(se)))
    key = (xcc * np.uint64(1000) + se * np.uint64(100) + cu * np.uint64(4) + simd)
    u, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    print("waves per SIMD (last step): min %d max %d  distinct SIMDs %d" % (cnt.min(), cnt.max(), len(u)))
    per = np.array([life[inv == k].mean() for k in range(len(u))])
    print("SIMD mean-life spread: p0 %.1f p50 %.1f p100 %.1f us" % tuple(np.percentile(per, [0, 50, 100])))
    wv = [life[inv == k] for k in range(len(u))]
    c = np.corrcoef(cnt[inv], life)[0, 1] if cnt.min() != cnt.max() else float("nan")
    print("corr(waves on SIMD, life) %.2f" % c)
    if a.team:
        # SIMD placement of each wave slot w of the team workgroups (env = G * block + w), and how
        # many distinct SIMDs the agent-phase waves (w = 0 for B, w = 1 for D) of one CU occupy
        slot = np.arange(len(simd)) % G
        cukey = xcc * np.uint64(1000) + se * np.uint64(100) + cu
        for w in range(G):
            h = np.bincount(simd[slot == w].astype(np.int64), minlength=4)
            print("wave slot %d: SIMD histogram %s" % (w, h.tolist()))
        for w in (0, 1 % G):
            m = slot == w
            ks, inv2 = np.unique(cukey[m], return_inverse=True)
            nd = [len(np.unique(simd[m][inv2 == k])) for k in range(len(ks))]
            nw = np.bincount(inv2)
            print("slot %d waves per CU: %s; distinct SIMDs among them: %s" % (
                w, np.bincount(nw).nonzero()[0].tolist(), np.bincount(nd).tolist()))
    env.close()


if __name__ == "__main__":
    main()
