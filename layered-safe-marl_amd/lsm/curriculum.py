"""Curriculum block computed on the host with the reference's own float64 expressions.

Mirrors ``SafeAamScenario.update_curriculum`` (navigation_graph_safe.py:324-366),
``get_effective_curriculum_ratio_sloped/stair`` (:1101-1122) and the
``curriculum_ratio_airtaxi`` / ``curriculum_ratio`` locals of
``Scenario.random_scenario`` (:1216-1218,1299-1302). The result is passed to the
reset kernel as an ``lsm_curriculum`` struct and stored per env.
"""
from __future__ import annotations

import numpy as np

from .config import AirTaxiConfig, DoubleIntegratorConfig, RewardBinaryConfig


def _sloped(r, start=0.25, end=0.75):
    return np.clip(r - start, 0, end - start) / (end - start)


def _stair(r, num_steps=4, start=0.2, end=0.75):
    if r < start:
        return 0
    if r > end:
        return 1
    cv = (num_steps - 1) * np.clip(r - start, 0, end - start) / (end - start)
    return (1 + np.floor(cv)) / num_steps


def curriculum_block(args, num_current_episode: int) -> dict:
    """All curriculum-derived quantities for one reset call (float64, reference order)."""
    di = args.dynamics_type == "double_integrator"
    C = DoubleIntegratorConfig if di else AirTaxiConfig
    total = int(args.num_env_steps) // args.episode_length // args.n_rollout_threads
    r = np.clip(num_current_episode / total, 0.0, 1.0)
    sl = _sloped(r)
    st = _stair(r)
    ghe0 = 0.5 - 0.5 * np.cos(C.GOAL_HEADING_THRESHOLD)
    ghe = ghe0 * (1.0 - sl) + ghe0 * sl
    gse = C.GOAL_SPEED_THRESHOLD * (1.0 - st) + C.GOAL_SPEED_THRESHOLD * st
    mdt = C.DISTANCE_TO_GOAL_THRESHOLD * (1.0 - st) + C.DISTANCE_TO_GOAL_THRESHOLD * st
    phase = _stair(r, start=0.2, end=0.75, num_steps=4) * 0.5 * np.pi
    rsd = 1 - np.cos(phase)
    use_filter = bool(args.use_safety_filter)
    world_filter = use_filter
    if (not (use_filter and RewardBinaryConfig.INITIAL_PHASE_USE_SAFETY_FILTER)) and use_filter:
        world_filter = bool(sl > 0)
    sep_t = C.SEPARATION_DISTANCE
    sep_i = args.initial_separation() if hasattr(args, "initial_separation") else (
        0 if RewardBinaryConfig.SEPARATION_DISTANCE_CURRICULUM else sep_t)
    sep = sep_i * (1.0 - rsd) + sep_t * rsd
    eng = C.ENGAGEMENT_DISTANCE + (sep - C.ENGAGEMENT_DISTANCE_REFERENCE_SEPARATION_DISTANCE)
    cra = 1 if use_filter else _sloped(r, start=0.25, end=0.75)
    crs = 1 if use_filter else _sloped(r)
    return dict(curriculum_ratio=float(r), sloped=float(sl), stair=float(st), ratio_airtaxi=float(cra),
                ratio_scenario=float(crs), goal_heading_error_thresh=float(ghe),
                goal_speed_error_thresh=float(gse), min_dist_thresh=float(mdt),
                separation_distance=float(sep), engagement_distance=float(eng),
                world_use_safety_filter=1.0 if world_filter else 0.0,
                # _stair returns the Python int 0 / 1 outside its ramp (:1115-1118): the scaled reward
                # weights (:340-345) are then ints, which keeps reward_hj_value's products float32
                stair_is_int=1.0 if isinstance(st, int) else 0.0)


def to_struct(block: dict):
    from .capi import LsmCurriculum
    c = LsmCurriculum()
    for k, v in block.items():
        setattr(c, k, float(v))
    return c
