"""CPU tests of the C ABI library (no GPU): it loads, exports every declared symbol, and its
host-side RNG / scenario code (the same template the reset kernel runs) replays numpy's
legacy RandomState draw-for-draw."""
import os
import re

import numpy as np
import pytest

from lsm import capi, curriculum
from lsm.config import EnvArgs
from oracle.lsm_oracle import OracleEnv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from lsm import build
    build.build(verbose=False)
    return capi.load_library()


def test_exports_every_declared_symbol(lib):
    hdr = open(os.path.join(ROOT, "include", "lsm_rollout.h")).read()
    declared = set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(lsm_\w+)\s*\(", hdr, re.M))
    assert declared == set(capi.EXPORTED)
    for name in declared:
        assert hasattr(lib, name), name


@pytest.mark.parametrize("seed", [0, 1, 1000, 4095001, 2 ** 32 - 1])
def test_host_mt_matches_numpy_legacy(lib, seed):
    n = 2000
    out = np.zeros(n)
    assert lib.lsm_host_mt_uniforms(seed, n, -3.2, 3.2, out.ctypes.data) == 0
    ref = np.random.RandomState(seed).uniform(-3.2, 3.2, n)
    np.testing.assert_array_equal(out, ref)


def _scenario_cases():
    for dyn in ("double_integrator", "airtaxi"):
        for n in (3, 8, 16):
            for ep in (0, 2, 4):
                for filt in (False, True):
                    yield dyn, n, ep, filt


@pytest.mark.parametrize("dyn,n,ep,filt", list(_scenario_cases()))
def test_host_scenario_matches_oracle(lib, dyn, n, ep, filt):
    ws = 4 if dyn == "double_integrator" else 6
    args = EnvArgs(dynamics_type=dyn, num_agents=n, world_size=ws, num_env_steps=250 * 4,
                   use_safety_filter=filt)
    seed = 17 + 1000 * n
    oargs = dict(vars(args))
    oargs["use_safety_filter"] = False
    ora = OracleEnv(oargs, seed, value_table=None, ttr_table=dict(lo=[0] * 4, hi=[1] * 4,
                    shape=(2, 2, 2, 2), values=np.zeros((2, 2, 2, 2), np.float32), ttr_max=1.0))
    ora.use_safety_filter = filt
    ora.curriculum_ratio = np.clip(ep / ora.num_total_episode, 0.0, 1.0)
    ora.random_scenario()
    blk = curriculum.curriculum_block(args, ep)
    cfg = capi.LsmConfig(dynamics=0 if dyn == "double_integrator" else 1, num_envs=1, num_agents=n,
                         num_landmarks=2, episode_length=250, use_safety_filter=int(filt), use_masking=1,
                         auto_reset=1, emit_edges=0, adj_layout=0, world_size=ws, seed=seed, env_offset=0)
    st = np.zeros((n, 4))
    lm = np.zeros((2 * n, 4))
    cur = curriculum.to_struct(blk)
    import ctypes as C
    assert lib.lsm_host_scenario(C.byref(cfg), C.byref(cur), seed, st.ctypes.data, lm.ctypes.data) == 0
    np.testing.assert_array_equal(st, ora.s)
    np.testing.assert_array_equal(lm[:, :2], ora.lm_pos)
    np.testing.assert_array_equal(lm[:, 3], ora.lm_speed)
    # headings go through atan2: glibc (here) vs numpy's arctan2 may differ in the last ulp
    np.testing.assert_allclose(lm[:, 2], ora.lm_heading, rtol=4e-16, atol=4e-16)


@pytest.mark.parametrize("dyn", ["double_integrator", "airtaxi"])
@pytest.mark.parametrize("filt", [False, True])
@pytest.mark.parametrize("ep", [0, 1, 2, 3, 4, 7, 100])
def test_curriculum_block_matches_oracle(dyn, filt, ep):
    args = EnvArgs(dynamics_type=dyn, num_agents=3, num_env_steps=250 * 8, use_safety_filter=filt,
                   world_size=4 if dyn == "double_integrator" else 6)
    ora = OracleEnv(vars(args), 0, value_table=dict(lo=[0] * 5, hi=[1] * 5, shape=(2,) * 5,
                    values_hj=np.zeros((2,) * 5, np.float32), grads_hj=np.zeros((2,) * 5 + (5,), np.float32),
                    separation_distance=ora_sep(dyn)) if filt else None,
                    ttr_table=dict(lo=[0] * 4, hi=[1] * 4, shape=(2,) * 4, values=np.zeros((2,) * 4, np.float32),
                                   ttr_max=1.0))
    ora.update_curriculum(ep)
    b = curriculum.curriculum_block(args, ep)
    assert b["curriculum_ratio"] == ora.curriculum_ratio
    assert b["goal_heading_error_thresh"] == ora.ghe
    assert b["goal_speed_error_thresh"] == ora.gse
    assert b["min_dist_thresh"] == ora.min_dist_thresh
    assert b["separation_distance"] == ora.separation_distance
    assert b["engagement_distance"] == ora.engagement_distance
    assert bool(b["world_use_safety_filter"]) == ora.world_filter_on
    assert b["sloped"] == ora.sloped()


def ora_sep(dyn):
    from lsm.config import AirTaxiConfig, DoubleIntegratorConfig
    return (DoubleIntegratorConfig if dyn == "double_integrator" else AirTaxiConfig).SEPARATION_DISTANCE


def test_config_validation():
    with pytest.raises(ValueError):
        EnvArgs(num_obstacles=1).validate()
    with pytest.raises(ValueError):
        EnvArgs(num_env_steps=10).validate()
    EnvArgs().validate()


def test_header_is_plain_c_abi():
    """include/lsm_rollout.h compiles as C99 and C++11 on its own: no torch or HIP types at the boundary."""
    import shutil
    import subprocess
    hdr = os.path.join(ROOT, "include", "lsm_rollout.h")
    for cc, std, lang in (("gcc", "-std=c99", "c"), ("g++", "-std=c++11", "c++")):
        if shutil.which(cc) is None:
            pytest.skip("%s not available" % cc)
        subprocess.check_call([cc, std, "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-x", lang, hdr])


# ---- Philox fast-reset stream (LSM_RNG_PHILOX) ---------------------------------------------------
# Random123 known-answer vectors for philox4x32_R(10, ctr, key) (kat_vectors: ctr, key, expected)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(lib, ctr, key, want):
    c = np.array(ctr, dtype=np.uint32)
    k = np.array(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    assert lib.lsm_host_philox4x32(c.ctypes.data, k.ctypes.data, out.ctypes.data) == 0
    assert tuple(int(x) for x in out) == want


def test_philox_uniforms_are_uniform_and_counter_based(lib):
    n = 200000
    a = np.zeros(n)
    b = np.zeros(n)
    lib.lsm_host_philox_uniforms(12345, 0, n, -2.0, 3.0, a.ctypes.data)
    lib.lsm_host_philox_uniforms(12345, 1, n, -2.0, 3.0, b.ctypes.data)
    assert a.min() >= -2.0 and a.max() < 3.0
    assert abs(a.mean() - 0.5) < 0.02 and abs(a.std() - 5 / np.sqrt(12)) < 0.02
    hist = np.histogram(a, bins=20, range=(-2, 3))[0]
    assert hist.min() > 0.9 * n / 20 and hist.max() < 1.1 * n / 20
    assert not np.array_equal(a[:100], b[:100])          # another reset index, another stream
    c = np.zeros(100)
    lib.lsm_host_philox_uniforms(12345, 0, 100, -2.0, 3.0, c.ctypes.data)
    np.testing.assert_array_equal(a[:100], c)             # same (key, reset) -> same draws


@pytest.mark.parametrize("dyn,n", [("double_integrator", 8), ("airtaxi", 16)])
def test_host_scenario_philox_distribution(lib, dyn, n):
    """The fast mode draws the same scenario distribution: agents / goals in the reference's
    boxes, goals separated as randomly_generate_separated_positions requires (utils.py:39-68)."""
    ws = 4 if dyn == "double_integrator" else 6
    cfg = capi.LsmConfig(dynamics=0 if dyn == "double_integrator" else 1, num_envs=1, num_agents=n,
                         num_landmarks=2, episode_length=250, world_size=ws, rng=capi.LSM_RNG_PHILOX)
    args = EnvArgs(dynamics_type=dyn, num_agents=n, world_size=ws, num_env_steps=250 * 4, use_safety_filter=True)
    cur = curriculum.to_struct(curriculum.curriculum_block(args, 4))
    seen = []
    for seed in range(40):
        st = np.zeros((n, 4))
        lm = np.zeros((2 * n, 4))
        assert lib.lsm_host_scenario(cfg, cur, seed * 1000 + 7, st.ctypes.data, lm.ctypes.data) == 0
        if dyn == "double_integrator":
            assert np.all(np.abs(st[:, :2]) <= 0.8 * ws) and np.all(st[:, 2:] == 0)
            dmin, dmax = 0.25 * 4.0, 0.75 * 4.0
        else:
            assert np.all(st[:, 0] >= -0.5 * ws) and np.all(st[:, 0] <= 0.25 * ws)
            assert np.all(np.abs(st[:, 1]) <= 0.5 * ws) and np.all((st[:, 2] >= 0) & (st[:, 2] < 2 * np.pi))
            dmin, dmax = 0.5 * 3 * 1.60934, 3 * 1.60934
        # agent 0's two goals (later agents may reuse the previous agent's goals, :1296-1300)
        seen.append(np.linalg.norm(lm[0, :2] - lm[n, :2]))
    d = np.array(seen)
    # the separation draw retries up to 1000 times: essentially every pair satisfies it
    assert np.mean((d > dmin) & (d < dmax)) > 0.95


def test_product_source_reads_no_environment_knobs():
    """Kernel choice is lsm_create_select's explicit lsm_kernel_select (tests, A/B runs), never an
    environment variable: every getenv in the rollout sources sits inside a diagnostic-build block
    (LSM_STAMPS / LSM_DIAGNOSTIC_BUILD, which product builds refuse)."""
    import os
    import re
    csrc = os.path.join(os.path.dirname(__file__), "..", "layered-safe-marl_amd", "csrc")
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".hip", ".h")):
            continue
        stack = []
        for ln, line in enumerate(open(os.path.join(csrc, name)), 1):
            t = line.strip()
            if re.match(r"#\s*if", t):
                stack.append(t)
            elif re.match(r"#\s*endif", t):
                stack.pop()
            elif re.match(r"#\s*else", t) and stack:
                stack[-1] = "else of " + stack[-1]
            if "getenv(" in line and not t.startswith("//"):
                guards = [g for g in stack if not g.startswith("else of") and
                          ("LSM_STAMPS" in g or "LSM_DIAGNOSTIC_BUILD" in g)]
                assert guards, "%s:%d reads the environment outside a diagnostic block" % (name, ln)
