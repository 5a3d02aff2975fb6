"""Evaluation scenario layouts computed on the host (``lsm_reset_layout``).

The evaluation Scenarios replace only ``random_scenario`` of the training scenario: they place
agents and landmarks by hand (and by a few draws from the env's numpy stream), then the rollout
is the same ``SafeAamScenario`` step -- plus, for ``RealisticScenario`` (the Bay Area maps),
per-agent departure timers. The reference computes these layouts in Python once per reset with
``n_rollout_threads = 1`` (``scripts/eval_mpe.py:101,121``); so does this module, and the device
does everything else of the reset and every step (``include/lsm_rollout.h``,
``LSM_SCENARIO_LAYOUT`` / ``LSM_SCENARIO_DEPARTURES``).

Each layout is a restatement of the reference's scenario function (cited per function) in the
same numpy operations and the same order of draws from the env's ``np.random`` stream, here an
explicit ``numpy.random.RandomState(seed + 1000 k)`` per env (the reference seeds the global
stream after ``make_world``, ``MPE_env.py:56-84`` + ``env.seed``, so the first reset's layout is the
first consumer).

Layouts:
  eval:<type>   ``navigation_graph_safe_eval.Scenario`` with ``eval_scenario_type`` = <type>
                (``navigation_graph_safe_eval.py:26-50``): circular_config, left_to_right_merge,
                bottom_to_top_merge, left_to_right_merge_and_land, bottom_to_top_merge_and_land,
                three_vehicle_conflicting_example, two_vehicle_conflicting_example.
                left_to_right_cross is not offered: it leaves every landmark's heading and speed
                None, and the reference's reward raises on its first step
                (``navigation_graph_safe.py:697-700``).
  bayarea_merge ``navigation_graph_safe_bayarea_merge.Scenario`` ("city_inbound", 8 agents,
                5 landmarks per agent, departure timers). Needs the map image's pixel size:
                the image is not in the reference (``RealisticScenario.__init__`` only reads
                its width and height, ``navigation_graph_safe.py:1125-1140``).
  bayarea_cross ``navigation_graph_safe_bayarea_cross.Scenario`` ("fixed_schedule", even N,
                6 landmarks per agent, departure timers).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import capi

# multiagent/config.py
DI_V_MIN = 0.1            # DoubleIntegratorConfig.V_MIN (goal speed min)
DI_V_NOMINAL = 0.5        # DoubleIntegratorConfig.V_NOMINAL
AT_V_MIN = 60 * 0.514444 * 0.001
AT_V_NOMINAL = 110 * 0.514444 * 0.001
AT_SEPARATION = 1500 * 0.0003048
DI_SEPARATION = 0.5
KM_IN_PIXEL = 73.6        # navigation_graph_safe_bayarea_*.py: super().__init__(..., km_in_pixel=73.6)

EVAL_TYPES = ("circular_config", "left_to_right_merge", "bottom_to_top_merge", "left_to_right_merge_and_land",
              "bottom_to_top_merge_and_land", "three_vehicle_conflicting_example",
              "two_vehicle_conflicting_example")


# ---- custom_scenarios/utils.py ------------------------------------------------------------------
def map_each_agent_landmarks_to_entire_landmarks(lst):
    """utils.py:10-25: agent-major lists -> order-major (landmark k of agent j at k * N + j)."""
    assert len(set(len(a) for a in lst)) == 1, "Number of landmarks for each agent should be the same"
    out = []
    for i in range(len(lst[0])):
        for j in range(len(lst)):
            out.append(lst[j][i])
    return out


def creat_relative_heading_list_from_goal_position_list(goal_position):
    """utils.py:27-37."""
    assert len(goal_position) > 1, "Goal position list should have more than 1 element"
    out = []
    for i in range(len(goal_position) - 1):
        h = goal_position[i + 1] - goal_position[i]
        out.append(np.arctan2(h[1], h[0]))
    return out


def randomly_generate_separated_positions(rng, n, x_range, y_range, min_distance=0.0, max_distance=np.inf):
    """utils.py:39-68 on the env's stream `rng`."""
    positions = []
    for i in range(n):
        if i > 0:
            for _ in range(1000):
                x = rng.uniform(x_range[0], x_range[1])
                y = rng.uniform(y_range[0], y_range[1])
                d = np.min(np.linalg.norm(np.array(positions) - np.array([x, y]), axis=1))
                if d > min_distance and d < max_distance:
                    break
        else:
            x = rng.uniform(x_range[0], x_range[1])
            y = rng.uniform(y_range[0], y_range[1])
        positions.append(np.asarray([x, y]))
    return positions


@dataclass
class Layout:
    """One env's reset layout: agent states [N][4] (x, y, v_x|theta, v_y|speed), landmarks
    [N*L][4] (x, y, heading, speed) and, for RealisticScenario, departed / timer / init_theta."""
    state: np.ndarray
    landmarks: np.ndarray
    departed: Optional[np.ndarray] = None
    timer: Optional[np.ndarray] = None
    init_theta: Optional[np.ndarray] = None
    # every layout sets agent.done = False except circular_config (navigation_graph_safe_eval.py:
    # 100-121), which leaves done agents of the previous episode done (packed as the keep-done
    # word the device reset honours, include/lsm_rollout.h lsm_reset_layout)
    clears_done: bool = True

    def pack(self) -> np.ndarray:
        parts = [self.state.reshape(-1), self.landmarks.reshape(-1)]
        if self.departed is not None:
            parts += [self.departed.astype(np.float64), self.timer.astype(np.float64),
                      self.init_theta.astype(np.float64)]
        parts.append(np.array([0.0 if self.clears_done else 1.0]))
        return np.concatenate(parts)


class ScenarioLayout:
    """A layout scenario: its landmark count, world size and per-reset layout draw.

    name: "eval:<type>", "bayarea_merge" or "bayarea_cross"; dynamics: "double_integrator" /
    "airtaxi"; num_landmarks: args.num_landmarks (0 = the scenario's default,
    ``init_landmarks``, navigation_graph_safe.py:37-44); image_size: (width, height) in pixels of
    the Bay Area map (RealisticScenario only)."""

    def __init__(self, name: str, dynamics: str, num_agents: int, num_landmarks: int = 0,
                 world_size: float = 2.0, image_size: Optional[Tuple[int, int]] = None):
        self.name = name
        self.di = dynamics == "double_integrator"
        self.N = int(num_agents)
        self.goal_speed_min = DI_V_MIN if self.di else AT_V_MIN
        self.goal_speed_max = DI_V_NOMINAL if self.di else AT_V_NOMINAL
        self.separation_distance = DI_SEPARATION if self.di else AT_SEPARATION
        self.departures = False
        if name.startswith("eval:"):
            self.kind = name[5:]
            if self.kind not in EVAL_TYPES:
                raise ValueError("eval layout must be one of %s" % (EVAL_TYPES,))
            default_l = {"circular_config": 1, "left_to_right_merge": 2, "bottom_to_top_merge": 2,
                         "left_to_right_merge_and_land": 3, "bottom_to_top_merge_and_land": 3,
                         "three_vehicle_conflicting_example": 1, "two_vehicle_conflicting_example": 1}[self.kind]
            aspect = {"circular_config": 1.0, "left_to_right_merge": 2.0, "bottom_to_top_merge": 0.5,
                      "left_to_right_merge_and_land": 2.0, "bottom_to_top_merge_and_land": 1.0,
                      "three_vehicle_conflicting_example": 1.0, "two_vehicle_conflicting_example": 1.0}[self.kind]
            self.world_size = float(world_size)
            self.world_aspect_ratio = aspect   # navigation_graph_safe_eval.py:75-98
        elif name in ("bayarea_merge", "bayarea_cross"):
            if dynamics != "airtaxi":
                raise ValueError("the Bay Area scenarios are airtaxi scenarios (RealisticScenario departures call "
                                 "KinematicVehicleXYState.reset_velocity(theta, speed))")
            if image_size is None:
                raise ValueError("RealisticScenario needs the map image's (width, height) in pixels")
            self.kind = name
            self.W, self.H = int(image_size[0]), int(image_size[1])
            self.world_size = 0.5 * self.H / KM_IN_PIXEL        # navigation_graph_safe.py:1139
            self.world_aspect_ratio = self.W / self.H            # bayarea_*.py get_aspect_ratio_for_scenario
            default_l = 5 if name == "bayarea_merge" else 6
            self.departures = True
        else:
            raise ValueError("unknown layout %r" % name)
        self.L = int(num_landmarks) if num_landmarks else default_l
        self.NL = self.N * self.L
        self.scenario_code = capi.LSM_SCENARIO_DEPARTURES if self.departures else capi.LSM_SCENARIO_LAYOUT

    # ---- helpers ------------------------------------------------------------------------------------
    def px(self, p):
        """RealisticScenario.convert_pixel_to_world_coordinates (navigation_graph_safe.py:1142-1151)."""
        x, y = p
        return np.array([(x - 0.5 * self.W) / KM_IN_PIXEL, (0.5 * self.H - y) / KM_IN_PIXEL])

    def _reset_velocity(self, theta):
        """state.reset_velocity(theta=...): DI zero velocity (core.py:215-217); airtaxi heading
        theta and speed = min_speed (core.py:137-145)."""
        if self.di:
            return np.array([0.0, 0.0])
        return np.array([theta, AT_V_MIN])

    def _landmarks(self, pos, head, speed):
        lm = np.zeros((self.NL, 4))
        # the reference assigns world.landmarks[k] for k < N * L from these (order-major) lists:
        # longer lists are truncated -- e.g. a Bay Area map run with a smaller --num_landmarks
        # keeps each agent's first L waypoints -- and shorter ones raise its IndexError
        if len(pos) < self.NL or len(head) < self.NL or len(speed) < self.NL:
            raise ValueError("layout has %d landmarks, the env %d (num_landmarks per agent = %d): the "
                             "reference raises IndexError" % (len(pos), self.NL, self.L))
        for k in range(self.NL):
            lm[k, 0:2] = pos[k]
            lm[k, 2] = head[k]
            lm[k, 3] = speed[k]
        return lm

    def draw(self, rng: np.random.RandomState, prev_state: Optional[np.ndarray] = None) -> Layout:
        """The layout of one reset. prev_state: the env's agent states before the reset (the Bay
        Area cross layout keeps their heading and speed)."""
        st = np.zeros((self.N, 4)) if prev_state is None else np.array(prev_state, dtype=np.float64).copy()
        fn = getattr(self, "_" + self.kind)
        return fn(rng, st)

    # ---- navigation_graph_safe_eval.py ----------------------------------------------------------
    def _circular_config(self, rng, st):
        """scenario_circular_config (navigation_graph_safe_eval.py:100-121)."""
        N = self.N
        agent_theta = np.linspace(0, 2 * np.pi, N, endpoint=False)
        radius = 0.92 * self.world_size / 2
        pos = []
        for i in range(N):
            p = np.array([radius * np.cos(agent_theta[i]), radius * np.sin(agent_theta[i])])
            st[i, :2] = p
            st[i, 2:] = self._reset_velocity(agent_theta[i] + np.pi)
            pos.append(p)
        lp = [-pos[i] for i in range(N)]
        lh = [agent_theta[i] + np.pi for i in range(N)]
        ls = [0.5 * (self.goal_speed_max + self.goal_speed_min)] * N
        return Layout(st, self._landmarks(lp, lh, ls), clears_done=False)

    def _merge_common(self, goal_positions, st, init_positions, theta):
        goal_headings = creat_relative_heading_list_from_goal_position_list(goal_positions)
        goal_headings.append(goal_headings[-1])
        if not self.di:
            goal_speeds = [self.goal_speed_max, self.goal_speed_max]
        else:
            goal_speeds = [self.goal_speed_max, self.goal_speed_min]
        for i in range(self.N):
            st[i, :2] = init_positions[i]
            st[i, 2:] = self._reset_velocity(theta)
        lp = map_each_agent_landmarks_to_entire_landmarks([goal_positions for _ in range(self.N)])
        lh = map_each_agent_landmarks_to_entire_landmarks([goal_headings for _ in range(self.N)])
        ls = map_each_agent_landmarks_to_entire_landmarks([goal_speeds for _ in range(self.N)])
        return Layout(st, self._landmarks(lp, lh, ls))

    def _left_to_right_merge(self, rng, st):
        """scenario_random_left_to_right_merge (navigation_graph_safe_eval.py:137-176): the
        separated-position draw is made (and discarded) before the even spacing."""
        u_h = 0.25 * self.world_size
        u_w = 0.25 * self.world_size * self.world_aspect_ratio
        randomly_generate_separated_positions(rng, self.N, (-2 * u_w, -u_w), (-2 * u_h, 2 * u_h),
                                              1.5 * self.separation_distance)
        pos_y = np.linspace(-2 * u_h, 2 * u_h, self.N)
        init = [np.array([-1.5 * u_w, pos_y[i]]) for i in range(self.N)]
        return self._merge_common([np.array([0, 0]), np.array([u_w, 0])], st, init, 0)

    def _bottom_to_top_merge(self, rng, st):
        """scenario_random_bottom_to_top_merge (navigation_graph_safe_eval.py:277-318)."""
        u_h = 0.25 * self.world_size
        u_w = 0.25 * self.world_size * self.world_aspect_ratio
        pos_x = np.linspace(2 * u_w, -2 * u_w, self.N)
        init = [np.array([pos_x[i], -1.5 * u_h]) for i in range(self.N)]
        return self._merge_common([np.array([0, 0]), np.array([0, u_h])], st, init, np.pi / 2)

    def _per_agent_landmarks(self, st, init_positions, theta, common, landing, speeds_of):
        lpl, lhl, lsl = [], [], []
        for i in range(self.N):
            lm_i = common + [landing[i]]
            lpl.append(lm_i)
            h = creat_relative_heading_list_from_goal_position_list(lm_i)
            h.append(h[-1])
            lhl.append(h)
            lsl.append(speeds_of(i))
        lp = map_each_agent_landmarks_to_entire_landmarks(lpl)
        lh = map_each_agent_landmarks_to_entire_landmarks(lhl)
        ls = map_each_agent_landmarks_to_entire_landmarks(lsl)
        for i in range(self.N):
            st[i, :2] = init_positions[i]
            st[i, 2:] = self._reset_velocity(theta)
        return Layout(st, self._landmarks(lp, lh, ls))

    def _left_to_right_merge_and_land(self, rng, st):
        """scenario_random_left_to_right_merge_and_land (navigation_graph_safe_eval.py:178-228)."""
        u_h = 0.25 * self.world_size
        u_w = 0.25 * self.world_size * self.world_aspect_ratio
        even_y = np.linspace(-2 * u_h, 2 * u_h, self.N)
        init = randomly_generate_separated_positions(rng, self.N, (-2 * u_w, -0.5 * u_w), (-2 * u_h, 2 * u_h),
                                                     1.5 * self.separation_distance)
        common = [np.array([0, 0]), np.array([u_w, 0])]
        landing = [np.array([2 * u_w, even_y[i]]) for i in range(self.N)]
        mid = 0.5 * (self.goal_speed_max + self.goal_speed_min)
        return self._per_agent_landmarks(st, init, 0, common, landing,
                                         lambda i: [mid, mid, self.goal_speed_min])

    def _bottom_to_top_merge_and_land(self, rng, st):
        """scenario_random_bottom_to_top_merge_and_land (navigation_graph_safe_eval.py:230-275)."""
        interval, first_y, land_w, init_y, init_w, shift = 1.5, 1.0, 3.0, -1.0, 2.0, 1.5
        common = [np.array([0.0, first_y + interval * i - shift]) for i in range(self.L - 1)]
        land_y = first_y + (self.L - 1) * interval
        land_x = np.linspace(-land_w / 2, land_w / 2, self.N)
        landing = [np.array([x, land_y - shift]) for x in land_x]
        init = randomly_generate_separated_positions(rng, self.N, (-init_w / 2, init_w / 2),
                                                     (init_y - shift, init_y + 0.5 - shift), self.separation_distance)
        return self._per_agent_landmarks(st, init, 0, common, landing,
                                         lambda i: [0.5 for _ in range(self.L - 1)] + [0.1])

    def _conflict(self, st, agents, landmark_distance):
        """scenario_{three,two}_vehicle_conflicting_example (navigation_graph_safe_eval.py:320-431):
        states set directly; landmark j at landmark_distance along agent j's heading (agent 0: +x)."""
        if self.di or self.L != 1:
            raise ValueError("the conflicting examples are airtaxi scenarios with 1 landmark per agent")
        lp, lh, ls = [], [], []
        for j, (p, th, v) in enumerate(agents):
            st[j] = [p[0], p[1], th, v]
            if j == 0:
                lp.append(np.array([p[0] + landmark_distance, 0.0]))
                lh.append(0.0)
            else:
                lp.append(p + np.array([np.cos(th), np.sin(th)]) * landmark_distance)
                lh.append(th)
            ls.append(self.goal_speed_max)
        return Layout(st, self._landmarks(lp, lh, ls))

    def _three_vehicle_conflicting_example(self, rng, st):
        if self.N != 3:
            raise ValueError("This scenario is only for 3 agents.")
        v = AT_V_NOMINAL
        agents = [(np.array([0.4, 0.0]), 0.0, v), (np.array([1.7, 0.3]), 4 * np.pi / 3, v),
                  (np.array([1.6, -0.6]), -np.pi, self.goal_speed_min)]
        return self._conflict(st, agents, 4.0)

    def _two_vehicle_conflicting_example(self, rng, st):
        if self.N != 2:
            raise ValueError("This scenario is only for 2 agents.")
        v = AT_V_NOMINAL
        agents = [(np.array([0.4, 0.0]), 0.0, v), (np.array([1.7, 0.3]), 4 * np.pi / 3, v)]
        return self._conflict(st, agents, 3.5)

    # ---- navigation_graph_safe_bayarea_merge.py: scenario_city_inbound (:84-198) --------------------
    def _bayarea_merge(self, rng, st):
        o = (13, 12)   # offset_x, offset_y (:25-26)
        P = lambda x, y: self.px((x + o[0], y + o[1]))
        depart = [P(260, 444), P(170, 243), P(1466, 160), P(1287, 525), P(1189, 695), P(1562, 937),
                  P(1916, 1032), P(1573, 1125)]   # CORTE_MADERA .. BERKELEY_MARINA
        goals = [P(1046, 1698)]                    # EMBARCADERO
        inter = [P(662, 597), P(910.5, 862), P(1159, 1127), P(1102.5, 1412.5)]
        san_pablo_mid = self.px((1106, 494))      # INTERMEDIATE_POINT_FOR_SAN_PABLO (no offset)
        landing = [np.arctan2(g[1] - inter[-1][1], g[0] - inter[-1][0]) for g in goals]
        dang = []
        for i, d in enumerate(depart):
            w = 0 if i < 2 else (2 if i < 6 else 3)
            dang.append(np.arctan2(inter[w][1] - d[1], inter[w][0] - d[0]))
        dang[2] = np.arctan2(san_pablo_mid[1] - depart[2][1], san_pablo_mid[0] - depart[2][0])
        if self.N != len(depart) * len(goals):
            raise ValueError("Number of agents should be equal to the product of number of depart positions and "
                             "goal positions (8)")
        dep = np.zeros(self.N)
        tmr = np.zeros(self.N)
        ith = np.zeros(self.N)
        lpl, lhl, lsl = [], [], []
        for i, d in enumerate(depart):
            for j, g in enumerate(goals):
                k = i * len(goals) + j
                st[k, :2] = d
                ith[k] = dang[i]
                tmr[k] = j * 150 + rng.randint(-30, 30)
                st[k, 3] = 0.0   # freeze_agent (:140)
                la = landing[j]
                if i < 2:
                    lm = [inter[0], inter[1], inter[2], inter[3], g]
                    h = creat_relative_heading_list_from_goal_position_list(lm)
                    h.append(la)
                elif i == 2:
                    lm = [san_pablo_mid, inter[1], inter[2], inter[3], g]
                    h = creat_relative_heading_list_from_goal_position_list(lm)
                    h.append(la)
                elif i < 6:
                    lm = [inter[2], inter[3], g, g, g]
                    h = creat_relative_heading_list_from_goal_position_list(lm)
                    h[-2] = la
                    h[-1] = la
                    h.append(la)
                else:
                    lm = [inter[3], g, g, g, g]
                    h = creat_relative_heading_list_from_goal_position_list(lm)
                    h[-3] = la
                    h[-2] = la
                    h[-1] = la
                    h.append(la)
                lpl.append(lm)
                lhl.append(h)
                lsl.append([self.goal_speed_max] * 5)
        lp = map_each_agent_landmarks_to_entire_landmarks(lpl)
        lh = map_each_agent_landmarks_to_entire_landmarks(lhl)
        ls = map_each_agent_landmarks_to_entire_landmarks(lsl)
        return Layout(st, self._landmarks(lp, lh, ls), dep, tmr, ith)

    # ---- navigation_graph_safe_bayarea_cross.py: scenario_fixed_schedule (:74-128) -----------------
    def _bayarea_cross(self, rng, st):
        c1 = [(611, 558), (1016, 1015), (1421, 1472), (1794, 1678), (2114, 1840), (2550, 2048), (3106, 2340)]
        c1.reverse()
        c2 = [(1569, 908), (1556, 1320), (1536, 1692), (1536, 2048), (1535, 2420), (1535, 2764)]
        if self.N % 2:
            raise ValueError("Number of agents should be even")
        depart = [self.px(c1[0]), self.px(c2[0])]
        w1 = [self.px(w) for w in c1][1:]
        last1 = np.arctan2(w1[-1][1] - w1[-2][1], w1[-1][0] - w1[-2][0])
        w2 = [self.px(w) for w in c2][1:]
        last2 = np.arctan2(w2[-1][1] - w2[-2][1], w2[-1][0] - w2[-2][0])
        w2.append(w2[-1])
        dh1 = np.arctan2(w1[0][1] - depart[0][1], w1[0][0] - depart[0][0])
        dh2 = np.arctan2(w2[0][1] - depart[1][1], w2[0][0] - depart[1][0])
        dep = np.zeros(self.N)
        tmr = np.zeros(self.N)
        ith = np.zeros(self.N)
        lpl, lhl, lsl = [], [], []
        for i in range(self.N):
            st[i, :2] = depart[i % 2]     # heading / speed kept from before the reset
            ith[i] = dh1 if i % 2 == 0 else dh2
            t = (i // 2) * 90 + rng.randint(-15, 15)
            if i % 2 == 1:
                t += 250
            tmr[i] = t
            lm = w1 if i % 2 == 0 else w2
            h = creat_relative_heading_list_from_goal_position_list(lm)
            if i % 2 == 1:
                h[-1] = last2
            h.append(last1 if i % 2 == 0 else last2)
            lpl.append(lm)
            lhl.append(h)
            lsl.append([self.goal_speed_max] * 7)
        lp = map_each_agent_landmarks_to_entire_landmarks(lpl)
        lh = map_each_agent_landmarks_to_entire_landmarks(lhl)
        ls = map_each_agent_landmarks_to_entire_landmarks(lsl)
        return Layout(st, self._landmarks(lp, lh, ls), dep, tmr, ith)


def from_args(args) -> Optional[ScenarioLayout]:
    """The layout of an evaluation scenario_name (None for the training scenario)."""
    name = args.scenario_name
    if name == "navigation_graph_safe":
        return None
    kind = {"navigation_graph_safe_eval": "eval:" + str(getattr(args, "eval_scenario_type", "")),
            "navigation_graph_safe_bayarea_merge": "bayarea_merge",
            "navigation_graph_safe_bayarea_cross": "bayarea_cross"}[name]
    return ScenarioLayout(kind, args.dynamics_type, int(args.num_agents), int(args.num_landmarks),
                          float(args.world_size), getattr(args, "bayarea_image_size", None))

