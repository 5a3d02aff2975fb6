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
