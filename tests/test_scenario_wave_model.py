"""Model of the team kernel's parallel scenario draw (``random_scenario_wave2``, csrc/lsm_team.h).

The device draws a reset's scenario with the agents in parallel: an agent-by-agent pass resolves only
where each agent's words start (point 0 and a ballot over 64 tries of the rejection loop), then every
agent's draws, the keep-previous / airtaxi-swap chain and the headings run for all agents at once. That
is correct only if the stream accounting -- agent i's block is [point 0: 4 words][tries: 4 (acc + 1)]
[keep: 4, i > 0][speeds: 6, double integrator][noise: 2] -- is the reference's. This test runs the same
algorithm in numpy on the raw MT19937 words of the env's seed and checks it against the oracle's
sequential ``random_scenario`` (navigation_graph_safe.py:1199-1367, utils.py:39-68) on the same seed:
identical states, goals, speeds and headings, and the same number of words consumed (the generator
state afterwards). CPU only; the GPU parity tests check the device code itself.
"""
from __future__ import annotations

import numpy as np
import pytest

from lsm.config import EnvArgs
from oracle.lsm_oracle import OracleEnv

TTR = dict(lo=[0] * 4, hi=[1] * 4, shape=(2, 2, 2, 2), values=np.zeros((2, 2, 2, 2), np.float32), ttr_max=1.0)


def raw_words(seed, n):
    """The first n 32-bit outputs of RandomState(seed) (randint over the full uint32 range draws one
    word per value, unmasked)."""
    return np.random.RandomState(seed).randint(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint64)


def uni(w, k, lo, hi):
    a = int(w[k]) >> 5
    b = int(w[k + 1]) >> 6
    return lo + (hi - lo) * ((a * 67108864.0 + b) / 9007199254740992.0)


def _accept(w, cs, j, box):
    """Try j of the agent whose block starts at word cs (point 0 = words cs..cs+3): accepted?
    (randomly_generate_separated_positions' test, utils.py:39-68; the 1000th try is kept)"""
    x0, x1, y0, y1, dmin, dmax = box
    ax, ay = uni(w, cs, x0, x1), uni(w, cs + 2, y0, y1)
    x, y = uni(w, cs + 4 + 4 * j, x0, x1), uni(w, cs + 6 + 4 * j, y0, y1)
    d = np.sqrt((ax - x) * (ax - x) + (ay - y) * (ay - y))
    return (d > dmin and d < dmax) or j == 999


def chain_sequential(w, N, c, box, after):
    """The reference's order: agent after agent, try after try."""
    starts, accs = [], []
    for i in range(N):
        acc = next(j for j in range(1000) if _accept(w, c, j, box))
        starts.append(c)
        accs.append(acc)
        c += 4 + 4 * (acc + 1) + after - (4 if i == 0 else 0)
    return starts, accs, c


def chain_two_per_ballot(w, N, c, box, after):
    """random_scenario_wave2's chain: one 64-lane ballot per two agents -- lanes 0-7 try 0-7 of agent
    i, lanes 8 + 8 g + t try t of agent i + 1 as if agent i accepted try g (g < 7); tries past those
    take 64-lane ballots from try 8 (first_from)."""
    def first_from(cs, j0):
        for base in range(j0, 1000, 64):
            m = [j < 1000 and _accept(w, cs, j, box) for j in range(base, base + 64)]
            if any(m):
                return base + m.index(True)
        return 999

    starts, accs = [], []
    i = 0
    while i < N:
        after_i = after - (4 if i == 0 else 0)
        two = i + 1 < N
        bits = []
        for lane in range(64):
            if lane < 8:
                bits.append(_accept(w, c, lane, box))
            else:
                g, t = (lane - 8) >> 3, lane & 7
                bits.append(two and _accept(w, c + 4 + 4 * (g + 1) + after_i, t, box))
        acc = bits.index(True) if any(bits[:8]) else first_from(c, 8)
        starts.append(c)
        accs.append(acc)
        c += 4 + 4 * (acc + 1) + after_i
        i += 1
        if two and acc < 7:
            grp = bits[8 + 8 * acc: 16 + 8 * acc]
            acc1 = grp.index(True) if any(grp) else first_from(c, 8)
            starts.append(c)
            accs.append(acc1)
            c += 4 + 4 * (acc1 + 1) + after
            i += 1
    return starts, accs, c


@pytest.mark.parametrize("N", [2, 3, 8, 9, 16])
def test_chain_two_per_ballot(N):
    """The two-agents-per-ballot chain equals the sequential rejection loops: the default boxes, and
    narrow acceptance bands that make tries past 7 (both fallbacks) and acc = 7 (no group) common."""
    w = raw_words(77 + N, 200000)
    rng = np.random.default_rng(N)
    boxes = [(-2.0, 2.0, -2.0, 2.0, 1.0, 3.0), (0.0, 4.5, -3.0, 3.0, 2.4, 4.8)]
    for _ in range(6):   # narrow bands: acceptance 2-20 % per try
        lo = rng.uniform(0.5, 2.5)
        boxes.append((-2.0, 2.0, -2.0, 2.0, lo, lo + rng.uniform(0.02, 0.3)))
    for box in boxes:
        for c0, after in ((0, 12), (37, 6), (1001, 12)):
            assert chain_two_per_ballot(w, N, c0, box, after) == chain_sequential(w, N, c0, box, after)


def wave2_model(w, dyn, N, ws, cra, cr, crange, gsmin, gsmax):
    """random_scenario_wave2's algorithm, lane loops written as Python loops."""
    st = np.zeros((N, 4))
    c = 0
    per = 4 if dyn == 0 else 8
    for i in range(N):   # agent states, agent i on lane i
        k = c + per * i
        if dyn == 0:
            st[i] = (uni(w, k, -0.8 * ws, 0.8 * ws), uni(w, k + 2, -0.8 * ws, 0.8 * ws), 0.0, 0.0)
        else:
            y = uni(w, k, -0.5 * ws, 0.5 * ws)
            x = uni(w, k + 2, -0.5 * ws, 0.25 * ws * cra + 0.0 * (1 - cra) * ws)
            spd = uni(w, k + 4, gsmin, gsmax)
            th = uni(w, k + 6, 0.0, 2 * np.pi)
            st[i] = (x, y, th, spd)
    c += per * N
    if dyn == 0:
        x0, x1, y0, y1 = -0.5 * ws, 0.5 * ws, -0.5 * ws, 0.5 * ws
        dmin, dmax = 0.25 * crange, 0.75 * crange
    else:
        yw = 0.1 * (1 - cra) + 0.5 * cra
        x0, x1, y0, y1 = 0.0, 0.75 * ws, -yw * ws, yw * ws
        dmin, dmax = 0.5 * crange, crange
    after = 4 + (6 if dyn == 0 else 0) + 2
    box = (x0, x1, y0, y1, dmin, dmax)
    # (1) the chain of block starts: point 0, then the first accepted try -- two agents per ballot on
    # the device (chain_two_per_ballot), the same as the sequential loop (test_chain_two_per_ballot)
    starts, accs, c = chain_two_per_ballot(w, N, c, box, after)
    # (2) every agent's draws on its lane
    draw, keep, mcs = [], [], []
    for i in range(N):
        s, t = starts[i], starts[i] + 4 + 4 * accs[i]
        draw.append((uni(w, s, x0, x1), uni(w, s + 2, y0, y1), uni(w, t, x0, x1), uni(w, t + 2, y0, y1)))
        k = t + 4
        if i > 0:
            keep.append((uni(w, k, 0.0, 1.0) < 0.5, uni(w, k + 2, 0.0, 1.0) < 0.5))
            k += 4
        else:
            keep.append((False, False))
        mcs.append(k)
    # (3) keep-previous and the airtaxi swap, in agent order
    final, prev = [], None
    for i in range(N):
        ax, ay, bx, by = draw[i]
        if i > 0:
            if keep[i][0]:
                ax, ay = prev[0], prev[1]
            if keep[i][1]:
                bx, by = prev[2], prev[3]
        if dyn != 0 and ax > bx:
            ax, ay, bx, by = bx, by, ax, ay
        final.append((ax, ay, bx, by))
        prev = final[-1]
    # (4) headings, speeds, noise on lane i
    lm = np.zeros((2 * N, 4))
    for i in range(N):
        ax, ay, bx, by = final[i]
        h = np.arctan2(by - ay, bx - ax)
        if dyn != 0:
            s0 = s1 = gsmax * 1.0
        else:
            var = uni(w, mcs[i] + 4, 0.0, 1.0)
            use_rnd = var < min(cr, 1 - 0.2)
            r0, r1 = uni(w, mcs[i], gsmin, gsmax), uni(w, mcs[i] + 2, gsmin, gsmax)
            s0 = r0 if use_rnd else gsmax * 1.0
            s1 = r1 if use_rnd else gsmin
        pr = cr * 0.25 * np.pi if dyn == 0 else cra * 0.1 * np.pi
        h0 = h + uni(w, mcs[i] + (6 if dyn == 0 else 0), -pr, pr)
        lm[i] = (ax, ay, h0, s0)
        lm[N + i] = (bx, by, h, s1)
    return st, lm, c


def _cases():
    for dyn in ("double_integrator", "airtaxi"):
        for n in (3, 8, 16):
            for ep in (0, 2, 4):
                for filt in (False, True):
                    yield dyn, n, ep, filt


@pytest.mark.parametrize("dyn,n,ep,filt", list(_cases()))
def test_parallel_draw_model_matches_oracle(dyn, n, ep, filt):
    ws = 4 if dyn == "double_integrator" else 6
    args = EnvArgs(dynamics_type=dyn, num_agents=n, world_size=ws, num_env_steps=250 * 4, use_safety_filter=filt)
    for seed in (17 + 1000 * n, 5, 123456):
        oargs = dict(vars(args))
        oargs["use_safety_filter"] = False
        ora = OracleEnv(oargs, seed, value_table=None, ttr_table=TTR)
        ora.use_safety_filter = filt
        ora.curriculum_ratio = np.clip(ep / ora.num_total_episode, 0.0, 1.0)
        cra = 1 if filt else ora.sloped(start=0.25, end=0.75)
        cr = 1 if filt else ora.sloped()
        ora.random_scenario()
        w = raw_words(seed, 20000)
        st, lm, used = wave2_model(w, 0 if ora.di else 1, n, ws, cra, cr, ora.coordination_range,
                                   ora.goal_speed_min, ora.goal_speed_max)
        np.testing.assert_array_equal(st, ora.s)
        np.testing.assert_array_equal(lm[:, :2], ora.lm_pos)
        np.testing.assert_array_equal(lm[:, 2], ora.lm_heading)
        np.testing.assert_array_equal(lm[:, 3], ora.lm_speed)
        # the same number of words consumed: the oracle's generator is where `used` raw words lead
        adv = np.random.RandomState(seed)
        adv.randint(0, 2 ** 32, size=used, dtype=np.uint64)
        a, b = adv.get_state(), ora.rng.get_state()
        assert a[2] == b[2] and np.array_equal(a[1], b[1])


def test_raw_words_are_the_uniform_stream():
    """uni() over raw_words() reproduces RandomState.uniform, the premise of the model."""
    w = raw_words(9, 64)
    r = np.random.RandomState(9)
    for k in range(0, 64, 2):
        assert uni(w, k, -3.0, 5.0) == r.uniform(-3.0, 5.0)


def _sq_band(dmin, dmax):
    """fill_params' squared-distance band (lsm_rollout.hip): the largest s with sqrt(s) <= dmin and
    the smallest s with sqrt(s) >= dmax, for the correctly rounded sqrt."""
    lo = dmin * dmin
    while np.sqrt(lo) > dmin:
        lo = np.nextafter(lo, 0.0)
    while np.sqrt(np.nextafter(lo, np.inf)) <= dmin:
        lo = np.nextafter(lo, np.inf)
    hi = dmax * dmax
    while np.sqrt(hi) < dmax:
        hi = np.nextafter(hi, np.inf)
    while np.sqrt(np.nextafter(hi, 0.0)) >= dmax:
        hi = np.nextafter(hi, 0.0)
    return lo, hi


@pytest.mark.parametrize("cr,f0,f1", [(4.0, 0.25, 0.75), (3 * 1.60934, 0.5, 1.0)])
def test_squared_band_equals_sqrt_band(cr, f0, f1):
    """random_scenario_wave2 accepts a try on d2 = dx*dx + dy*dy in (d2lo, d2hi) instead of
    sqrt(d2) in (dmin, dmax): the same decision for every double d2 (both band ends probed a few
    hundred ulps either side, plus random squared distances of the draw's range)."""
    dmin, dmax = f0 * cr, f1 * cr
    lo, hi = _sq_band(dmin, dmax)
    probes = []
    for t in (lo, hi, dmin * dmin, dmax * dmax):
        x = t
        for _ in range(300):
            x = np.nextafter(x, 0.0)
        for _ in range(600):
            probes.append(x)
            x = np.nextafter(x, np.inf)
    rng = np.random.default_rng(7)
    probes = np.concatenate([np.array(probes), rng.uniform(0.0, 4 * dmax * dmax, 200000)])
    d = np.sqrt(probes)
    np.testing.assert_array_equal((d > dmin) & (d < dmax), (probes > lo) & (probes < hi))
