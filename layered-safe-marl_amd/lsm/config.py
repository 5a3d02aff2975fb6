"""Physical / reward constants and env arguments of the navigation_graph_safe path.

Mirrors ``multiagent/config.py:3-83`` (same class and attribute names, same
expressions, so float64 values are bit-identical) and the env-side argparse
fields the reference's ``make_world`` reads (``scripts/train_mpe.py:73-107``,
``onpolicy/config.py``; canonical values from ``train.sh:15-30``).
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass, asdict
from typing import Optional

import numpy as np


class AirTaxiConfig:
    V_MIN = 60 * 0.514444 * 0.001
    V_MAX = 175 * 0.514444 * 0.001
    V_NOMINAL = 110 * 0.514444 * 0.001
    ACCEL_MIN = -0.001
    ACCEL_MAX = 0.002
    ANGULAR_RATE_MAX = 0.1
    MOTION_PRIM_ACCEL_OPTIONS = 5
    MOTION_PRIM_ANGRATE_OPTIONS = 5
    CBF_RATE = 3.0
    ENGAGEMENT_DISTANCE = 1.4
    ENGAGEMENT_DISTANCE_REFERENCE_SEPARATION_DISTANCE = 2200 * 0.0003048
    DT = 1.0
    DISTANCE_TO_GOAL_THRESHOLD = 0.35
    GOAL_HEADING_THRESHOLD = np.pi / 4
    GOAL_SPEED_THRESHOLD = 0.03
    SEPARATION_DISTANCE = 1500 * 0.0003048
    COORDINATION_RANGE = 3 * 1.60934


class DoubleIntegratorConfig:
    VX_MIN = -0.5
    VX_MAX = 0.5
    VY_MIN = -0.5
    VY_MAX = 0.5
    V_MIN = 0.1
    V_NOMINAL = 0.5
    V_MAX = np.sqrt(VX_MAX ** 2 + VY_MAX ** 2)
    ACCELX_MIN = -0.5
    ACCELX_MAX = 0.5
    ACCELY_MIN = -0.5
    ACCELY_MAX = 0.5
    ACCELX_OPTIONS = 5
    ACCELY_OPTIONS = 5
    CBF_RATE = 3.0
    ENGAGEMENT_DISTANCE = 1.0
    ENGAGEMENT_DISTANCE_REFERENCE_SEPARATION_DISTANCE = 0.5
    DT = 0.1
    DISTANCE_TO_GOAL_THRESHOLD = 0.3
    GOAL_HEADING_THRESHOLD = np.pi / 4
    GOAL_SPEED_THRESHOLD = 0.15
    SEPARATION_DISTANCE = 0.5
    COORDINATION_RANGE = 4


class RewardWeightConfig:
    MIN_REWARD = -40
    MAX_REWARD = 50
    GOAL_REACH = 50
    SAFETY_VIOLATION = -20
    HJ_VALUE = -2
    POTENTIAL_CONFLICT = -1
    DIFF_FROM_FILTERED_ACTION = -1


class RewardBinaryConfig:
    SAFETY_VIOLATION = False
    HJ_VALUE = False
    POTENTIAL_CONFLICT = False
    SEPARATION_DISTANCE_CURRICULUM = False
    INITIAL_PHASE_USE_SAFETY_FILTER = False
    DIFF_FROM_FILTERED_ACTION = False


REWARD_TERMS = {   # EnvArgs.reward_terms names -> RewardBinaryConfig switch (config.py:78-83)
    "safety_violation": "SAFETY_VIOLATION",
    "potential_conflict": "POTENTIAL_CONFLICT",
    "diff_from_filtered_action": "DIFF_FROM_FILTERED_ACTION",
    "hj_value": "HJ_VALUE",
}

ENTITY_SIZE = 0.050          # multiagent/core.py:261
EPS_HJ = 0.4                 # multiagent/safety_filter.py:235,410


# scenario_name values: the training scenario and the evaluation scenarios whose layouts
# lsm.layouts restates (navigation_graph_safe_eval.py, navigation_graph_safe_bayarea_*.py)
SCENARIOS = ("navigation_graph_safe", "navigation_graph_safe_eval", "navigation_graph_safe_bayarea_merge",
             "navigation_graph_safe_bayarea_cross")
EVAL_SCENARIO_TYPE = "left_to_right_merge_and_land"   # multiagent/config.py:86


@dataclass
class EnvArgs:
    """The env-side flags of ``all_args`` that the path reads."""
    scenario_name: str = "navigation_graph_safe"
    dynamics_type: str = "double_integrator"
    num_agents: int = 3
    num_landmarks: int = 2
    num_obstacles: int = 0
    num_walls: int = 0
    num_scripted_agents: int = 0
    world_size: float = 4
    episode_length: int = 250
    num_env_steps: int = 1000
    n_rollout_threads: int = 1
    use_safety_filter: bool = False
    num_internal_step: int = 1
    use_masking: bool = True
    use_dones: bool = False
    collaborative: bool = False
    graph_feat_type: str = "relative"
    discrete_action: bool = True
    seed: int = 0
    # RewardBinaryConfig.SEPARATION_DISTANCE_CURRICULUM (a hand-edited class constant in the
    # reference, config.py:81); None = that constant, True / False override it per env handle
    separation_distance_curriculum: Optional[bool] = None
    # RewardBinaryConfig's optional reward terms (config.py:78-83, class constants the reference's
    # users edit): None = those constants; else the names of the terms switched on, a subset of
    # REWARD_TERMS (navigation_graph_safe.py:793-850)
    reward_terms: Optional[tuple] = None
    # evaluation scenarios: multiagent.config.eval_scenario_type (a module constant in the
    # reference) and the Bay Area map's (width, height) in pixels (the image is not in the reference)
    eval_scenario_type: str = EVAL_SCENARIO_TYPE
    bayarea_image_size: Optional[tuple] = None

    def active_reward_terms(self) -> tuple:
        """The optional reward terms in effect (names, REWARD_TERMS order)."""
        if self.reward_terms is None:
            return tuple(k for k in REWARD_TERMS if getattr(RewardBinaryConfig, REWARD_TERMS[k]))
        return tuple(k for k in REWARD_TERMS if k in self.reward_terms)

    def uses_hj_handle(self) -> bool:
        """use_hj_handle = use_safety_filter or RewardBinaryConfig.HJ_VALUE (navigation_graph_safe.py:195)."""
        return bool(self.use_safety_filter) or "hj_value" in self.active_reward_terms()

    def sep_curriculum(self) -> bool:
        v = self.separation_distance_curriculum
        return bool(RewardBinaryConfig.SEPARATION_DISTANCE_CURRICULUM if v is None else v)

    def initial_separation(self) -> float:
        """The scenario's separation_distance_init, which HjDataHandle is built with
        (navigation_graph_safe.py:183-196, core.py:429,456)."""
        C = DoubleIntegratorConfig if self.dynamics_type == "double_integrator" else AirTaxiConfig
        return 0 if self.sep_curriculum() else C.SEPARATION_DISTANCE

    @staticmethod
    def from_namespace(ns: argparse.Namespace) -> "EnvArgs":
        kw = {k: getattr(ns, k) for k in EnvArgs.__dataclass_fields__ if hasattr(ns, k)}
        return EnvArgs(**kw)

    def to_namespace(self) -> argparse.Namespace:
        return argparse.Namespace(**asdict(self))

    def validate(self):
        if self.scenario_name not in SCENARIOS:
            raise ValueError("scenario_name must be one of %s (the training scenario and its evaluation "
                             "layouts, lsm.layouts)" % (SCENARIOS,))
        if self.num_obstacles != 0 or self.num_walls != 0 or self.num_scripted_agents != 0:
            raise ValueError("obstacles/walls/scripted agents are not supported by the graph mask "
                             "(navigation_graph_safe.py:976-989)")
        if self.dynamics_type not in ("double_integrator", "airtaxi"):
            raise ValueError("dynamics_type must be 'double_integrator' or 'airtaxi'")
        if self.graph_feat_type != "relative":
            raise ValueError("only graph_feat_type='relative' is on the path (train.sh)")
        if self.num_landmarks < 1 and self.scenario_name == "navigation_graph_safe":
            raise ValueError("num_landmarks must be >= 1")
        if not 1 <= int(self.num_internal_step) <= 64:
            raise ValueError("num_internal_step must be in [1, 64] (World.step's inner loop, core.py:607)")
        if not self.discrete_action:
            raise ValueError("only the Discrete(25) action space is on the path")
        if self.reward_terms is not None:
            bad = sorted(set(self.reward_terms) - set(REWARD_TERMS))
            if bad:
                raise ValueError("unknown reward_terms %s (RewardBinaryConfig has %s)" % (bad, sorted(REWARD_TERMS)))
        if not isinstance(self.collaborative, (bool, int)) or int(self.collaborative) not in (0, 1):
            raise ValueError("collaborative must be a bool (MultiAgentGraphEnv.shared_reward)")
        total = int(self.num_env_steps) // self.episode_length // self.n_rollout_threads
        if total == 0:
            raise ValueError("num_env_steps // episode_length // n_rollout_threads == 0: the "
                             "reference's update_curriculum divides by it (navigation_graph_safe.py:326)")
        n_lm = self.num_agents * self.num_landmarks
        if n_lm - 1 > 127:
            raise ValueError("landmark ids are addressed through np.int8 (navigation_graph_safe.py:581)")
