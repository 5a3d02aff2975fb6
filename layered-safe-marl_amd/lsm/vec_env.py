"""``GpuGraphVecEnv`` -- drop-in for GraphSubprocVecEnv / GraphDummyVecEnv on one MI355X.

Mirrors the reference's vec-env surface for the navigation_graph_safe path
(``onpolicy/envs/env_wrappers.py:29-140,851-1029``):

* ``reset(num_current_episode=0)`` -> ``(obs, agent_id, node_obs, adj, ep_info)``
* ``step(actions, num_current_episode=None)`` -> the 7-tuple of
  ``GraphSubprocVecEnv`` (auto-reset when every agent of an env is done, ep_info
  appended as the (N+1)-th info entry) or, with ``auto_reset=False``, the 8-tuple
  of ``GraphDummyVecEnv`` (``reset_count = 0``, no auto-reset)
* ``step_async`` / ``step_wait`` / ``close`` and the space attributes the runner
  sizes its buffers from.

All computation happens in ``liblsm_rollout.so`` (C ABI, HIP kernels). This
class only allocates the device output buffers (torch tensors), computes the
per-call curriculum block with the reference's float64 expressions, and converts
outputs: ``return_numpy=True`` gives host numpy arrays with the reference's dtypes
(float64 obs/node_obs/adj/rewards holding the kernel's float32 values -- the runner's buffer
stores float32 anyway); ``return_numpy=False`` keeps everything as device tensors.

Evaluation scenarios (``layout=lsm.layouts.ScenarioLayout(...)``): the reset's layout is
computed on the host from each env's numpy stream and handed to ``lsm_reset_layout``; every
step (and, for the Bay Area maps, the departure timers) runs on the device.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import capi
from .config import EnvArgs
from .curriculum import curriculum_block, to_struct
from .hj_tables import HjTable, default_tables
from .layouts import ScenarioLayout
from .share_vec_env import ShareVecEnv
from .spaces import Box, Discrete

EPKEYS = ("travel_time_mean", "travel_distance_mean", "done_percentage", "num_reached_goal_mean",
          "conflict_percentage", "min_distance_mean", "min_distance_min", "multiple_engagement_percentage")


def _torch():
    import torch
    return torch


class EnvInfos(list):
    """Per-env info list built lazily from the device info tensor (host copy)."""


def infos_from_arrays(info, reset, ep_info, auto_reset=True, departed=None):
    """The reference's per-env info lists from the device arrays: per agent the
    ``info_callback`` dict (navigation_graph_safe.py:386-450) plus the keys
    ``MultiAgentGraphEnv.step`` adds (environment.py:1025-1029), then the episode summary as
    the (N+1)-th entry when the worker auto-reset (env_wrappers.py:866-871).

    info [n][N][LSM_INFO_FIELDS] float64 (capi.INFO_FIELDS), reset [n], ep_info [n][8] or None.
    """
    fields = capi.INFO_FIELDS
    n, N = info.shape[0], info.shape[1]
    out = []
    for e in range(n):
        lst = EnvInfos()
        for i in range(N):
            d = {k: float(info[e, i, j]) for j, k in enumerate(fields) if not k.startswith("position_")}
            d["Safety filtered"] = bool(d["Safety filtered"])
            d["Safety violated"] = bool(d["Safety violated"])
            d["id"] = i
            d["position"] = np.array([info[e, i, fields.index("position_x")],
                                      info[e, i, fields.index("position_y")]], dtype=np.float64)
            d["Num_obst_collisions"] = 0.0
            d["Mean_by_variance"] = d["Distance_mean"] / (d["Distance_variance"] + 0.0001)
            d["Time_taken"] = d["Time_req_to_goal"]
            d["Time_mean_by_stddev"] = d["Time_mean"] / (d["Time_stddev"] + 0.0001)
            d["Departed"] = True if departed is None else bool(departed[e, i])
            lst.append(d)
        if auto_reset and reset[e]:
            lst.append({k: float(ep_info[e, j]) for j, k in enumerate(EPKEYS)})
        out.append(lst)
    return tuple(out)


def expand_compact_adj(adj, mask, E):
    """adj[e][r][c] = (M[e] bit r | M[e] bit c) ? 0 : A[r][c] for the compact layout
    (A: [n, E, E] float32, M: [n, N, W] int64 words of disconnect bits)."""
    torch = _torch()
    n, N, W = mask.shape
    sh = torch.arange(64, device=mask.device, dtype=torch.int64)
    bits = ((mask.unsqueeze(-1) >> sh) & 1).reshape(n, N, W * 64)[..., :E].bool()
    keep = ~(bits.unsqueeze(-1) | bits.unsqueeze(-2))
    # a select, not a product: masked entries are assigned 0 in the reference (in-place zeroing,
    # navigation_graph_safe.py:976-989), whatever the table holds
    return torch.where(keep, adj.unsqueeze(1), torch.zeros((), dtype=adj.dtype, device=adj.device))


class GpuGraphVecEnv(ShareVecEnv):
    """rng: "mt19937" (the reference's draws, default) or "philox" (fast device resets, same
    scenario distribution). layout: an evaluation ScenarioLayout (needs auto_reset=False).
    kernel_select: tests / A/B runs only, fields of lsm_kernel_select (include/lsm_rollout.h), e.g.
    {"workgroup_per_env": 1} or {"team": 0}; None = the library's own choice.
    emit_edge_counts: the step also writes each ego graph's adjacency nonzeros (LSM_OUT_ADJ_NNZ, E <= 64
    kernels), and edge_list() builds the learner's edge list in one pass over the adjacency."""

    def __init__(self, all_args, num_envs: Optional[int] = None, device=None,
                 value_table: Optional[HjTable] = None, ttr_table: Optional[HjTable] = None,
                 auto_reset: bool = True, env_offset: int = 0, emit_edges: bool = False,
                 return_numpy: bool = True, build_infos: bool = True, small_tables: bool = False,
                 adj_layout: str = "reference", collision_forces: bool = False,
                 layout: Optional[ScenarioLayout] = None, rng: str = "mt19937",
                 kernel_select: Optional[dict] = None, emit_edge_counts: bool = False):
        torch = _torch()
        self.args = EnvArgs.from_namespace(all_args) if not isinstance(all_args, EnvArgs) else all_args
        self.args.validate()
        a = self.args
        if layout is None and a.scenario_name != "navigation_graph_safe":
            from .layouts import from_args
            layout = from_args(a)
        self.layout = layout
        if layout is not None:
            if auto_reset:
                raise ValueError("evaluation layouts run with GraphDummyVecEnv semantics (auto_reset=False), "
                                 "as scripts/eval_mpe.py does")
            if layout.N != int(a.num_agents):
                raise ValueError("layout built for %d agents, args.num_agents = %d" % (layout.N, a.num_agents))
            a.num_landmarks = layout.L
        elif a.num_landmarks < 2:
            raise ValueError("num_landmarks must be >= 2 (reference asserts, utils.py:31)")
        if rng not in ("mt19937", "philox"):
            raise ValueError("rng must be 'mt19937' or 'philox'")
        self.num_envs = int(num_envs if num_envs is not None else a.n_rollout_threads)
        self.env_offset = int(env_offset)   # global index of this handle's env 0 (seed + 1000 k)
        self.device = torch.device(device if device is not None else "cuda:%d" % torch.cuda.current_device())
        if self.device.type != "cuda":
            raise capi.LsmError("GpuGraphVecEnv needs a HIP device; there is no CPU fallback")
        torch.cuda.set_device(self.device)
        self.lib = capi.load_library()
        self.auto_reset = bool(auto_reset)
        self.return_numpy = bool(return_numpy)
        self.build_infos = bool(build_infos)
        di = a.dynamics_type == "double_integrator"
        self.N = int(a.num_agents)
        if adj_layout not in ("reference", "compact"):
            raise ValueError("adj_layout must be 'reference' or 'compact'")
        self.adj_layout = adj_layout
        cfg = capi.LsmConfig(dynamics=capi.LSM_DOUBLE_INTEGRATOR if di else capi.LSM_AIRTAXI,
                             num_envs=self.num_envs, num_agents=self.N, num_landmarks=int(a.num_landmarks),
                             episode_length=int(a.episode_length), use_safety_filter=int(bool(a.use_safety_filter)),
                             use_masking=int(bool(a.use_masking)), auto_reset=int(self.auto_reset),
                             emit_edges=int(bool(emit_edges)),
                             adj_layout=capi.ADJ_COMPACT if adj_layout == "compact" else capi.ADJ_REFERENCE,
                             world_size=float(a.world_size),
                             seed=int(a.seed), env_offset=int(env_offset),
                             collision_forces=int(bool(collision_forces)),
                             scenario=layout.scenario_code if layout is not None else capi.LSM_SCENARIO_TRAIN,
                             rng=capi.LSM_RNG_PHILOX if rng == "philox" else capi.LSM_RNG_MT19937,
                             num_internal_step=int(a.num_internal_step),
                             reward_terms=sum(capi.REWARD_BITS[k] for k in a.active_reward_terms()),
                             collaborative=int(bool(a.collaborative)))
        self.collaborative = bool(a.collaborative)
        if int(a.seed) + 1000 * (int(env_offset) + self.num_envs - 1) >= 2 ** 32:
            raise ValueError("numpy seeds must be < 2**32 (seed + 1000 * env index)")
        h = C.c_void_p()
        if kernel_select:   # tests / A/B runs: an explicit kernel (capi.KERNEL_SELECT_DEFAULTS)
            rc = self.lib.lsm_create_select(C.byref(cfg), C.byref(capi.kernel_select(**kernel_select)), C.byref(h))
        else:
            rc = self.lib.lsm_create(C.byref(cfg), C.byref(h))
        self.h = h
        capi.check(rc, h)
        # HJ / TTR tables (synthetic stand-ins for the absent pickles unless given); the HJ handle exists
        # with the filter on or RewardBinaryConfig.HJ_VALUE (navigation_graph_safe.py:195)
        if a.uses_hj_handle() or not di:
            vt, tt = default_tables(a.dynamics_type, small=small_tables, target_separation=a.initial_separation())
            value_table = value_table if value_table is not None else vt
            ttr_table = ttr_table if ttr_table is not None else tt
        self.value_table = value_table if a.uses_hj_handle() else None
        self.ttr_table = ttr_table if not di else None
        if self.value_table is not None:
            self._upload_value_table()
        if self.ttr_table is not None:
            t = self.ttr_table
            self._set_table(self.lib.lsm_set_ttr_table, t, t.values_hj, None, extra=(float(t.ttr_max),))
        # outputs
        self.E = int(self.lib.lsm_num_entities(h))
        self.F = int(self.lib.lsm_node_features(h))
        self.OBS = int(self.lib.lsm_obs_dim(h))
        n, N, E, F = self.num_envs, self.N, self.E, self.F
        dev = self.device
        self.t_obs = torch.zeros((n, N, self.OBS), dtype=torch.float32, device=dev)
        self.t_node = torch.zeros((n, N, E, F), dtype=torch.float32, device=dev)
        if adj_layout == "compact":
            # unmasked E x E table per env + per-ego disconnect bits (include/lsm_rollout.h)
            self.t_adj = torch.zeros((n, E, E), dtype=torch.float32, device=dev)
            self.t_adj_mask = torch.zeros((n, N, (E + 63) // 64), dtype=torch.int64, device=dev)
        else:
            self.t_adj = torch.zeros((n, N, E, E), dtype=torch.float32, device=dev)
            self.t_adj_mask = None
        self.t_rew = torch.zeros((n, N), dtype=torch.float32, device=dev)
        self.t_done = torch.zeros((n, N), dtype=torch.bool, device=dev)   # u8 buffer, 0/1
        self.t_reset = torch.zeros((n,), dtype=torch.bool, device=dev)
        self.t_epinfo = torch.zeros((n, 8), dtype=torch.float64, device=dev)
        self.t_info = torch.zeros((n, N, len(capi.INFO_FIELDS)), dtype=torch.float64, device=dev)
        self.t_state = torch.zeros((n, N, 4), dtype=torch.float64, device=dev)
        self.t_edges = torch.zeros((n, E, E), dtype=torch.uint8, device=dev) if emit_edges else None
        # per-ego adjacency nonzeros (LSM_OUT_ADJ_NNZ): edge_list() then reads the adjacency once
        self.t_adj_nnz = torch.zeros((n, N), dtype=torch.int64, device=dev) if emit_edge_counts else None
        # World.get_entity_collision_force per agent (optional report; never applied, like the reference)
        self.t_cforce = torch.zeros((n, N, 2), dtype=torch.float64, device=dev) if collision_forces else None
        # info 'Departed' (RealisticScenario departure timers)
        self.t_departed = (torch.zeros((n, N), dtype=torch.bool, device=dev)
                           if layout is not None and layout.departures else None)
        for slot, t in ((capi.OUT_OBS, self.t_obs), (capi.OUT_NODE_OBS, self.t_node),
                        (capi.OUT_ADJ, self.t_adj), (capi.OUT_REWARD, self.t_rew),
                        (capi.OUT_DONE, self.t_done), (capi.OUT_RESET_FLAG, self.t_reset),
                        (capi.OUT_EP_INFO, self.t_epinfo), (capi.OUT_INFO, self.t_info),
                        (capi.OUT_STATE, self.t_state), (capi.OUT_EDGES, self.t_edges),
                        (capi.OUT_ADJ_MASK, self.t_adj_mask), (capi.OUT_COLLISION_FORCE, self.t_cforce),
                        (capi.OUT_DEPARTED, self.t_departed), (capi.OUT_ADJ_NNZ, self.t_adj_nnz)):
            if t is None:
                continue
            capi.check(self.lib.lsm_bind_output(h, slot, C.c_void_p(t.data_ptr()),
                                                t.numel() * t.element_size()), h)
        self.agent_id = torch.arange(N, device=dev, dtype=torch.int64).view(1, N, 1).expand(n, N, 1).contiguous()
        # spaces (environment.py:143-202, 928-960)
        self.action_space = [Discrete(25) for _ in range(N)]
        self.observation_space = [Box(-np.inf, np.inf, (self.OBS,)) for _ in range(N)]
        self.share_observation_space = [Box(-np.inf, np.inf, (self.OBS * N,)) for _ in range(N)]
        self.node_observation_space = [Box(-np.inf, np.inf, (E, F)) for _ in range(N)]
        self.adj_observation_space = [Box(-np.inf, np.inf, (E, E)) for _ in range(N)]
        self.edge_observation_space = [Box(-np.inf, np.inf, (1,)) for _ in range(N)]
        self.agent_id_observation_space = [Box(-np.inf, np.inf, (1,)) for _ in range(N)]
        self.share_agent_id_observation_space = [Box(-np.inf, np.inf, (N,)) for _ in range(N)]
        self._pending = None
        self._cur_cache = {}
        self._last_ep = 0
        self.closed = False
        # evaluation layouts draw from each env's numpy stream on the host (np.random.seed(seed +
        # 1000 k) after make_world, MPE_env.py:56-84)
        self._rngs = ([np.random.RandomState(int(a.seed) + 1000 * (int(env_offset) + k)) for k in range(n)]
                      if layout is not None else None)
        self.kernel_name = self.lib.lsm_kernel_name(h).decode()

    # -- tables ------------------------------------------------------------------------
    def _set_table(self, fn, t: HjTable, values, grads, extra=()):
        nd = t.ndim
        lo = (C.c_double * nd)(*[float(x) for x in t.lo])
        hi = (C.c_double * nd)(*[float(x) for x in t.hi])
        shape = (C.c_int32 * nd)(*[int(x) for x in t.shape])
        per = (C.c_int32 * nd)(*[1 if d in t.periodic else 0 for d in range(nd)])
        v = np.ascontiguousarray(values, dtype=np.float32)
        args = [self.h, nd, lo, hi, shape, per, v.ctypes.data_as(C.c_void_p)]
        if grads is not None:
            g = np.ascontiguousarray(grads, dtype=np.float32)
            args.append(g.ctypes.data_as(C.c_void_p))
        args.extend(extra)
        capi.check(fn(*args), self.h)

    def _upload_value_table(self):
        """HjDataHandle.__init__ (safety_filter.py:155-168): the table is read-only after this;
        each env's own `update_separation_distance` history (safety_filter.py:170-174) is applied
        on the device at its resets."""
        t = self.value_table
        self._set_table(self.lib.lsm_set_value_table, t, t.values_hj, t.device_grads(),
                        extra=(float(t.separation_distance),))

    # -- vec-env API -------------------------------------------------------------------------
    def _stream(self):
        return C.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def reset(self, num_current_episode: int = 0):
        block = curriculum_block(self.args, num_current_episode)
        self._last_ep = num_current_episode
        cur = to_struct(block)
        if self.layout is None:
            capi.check(self.lib.lsm_reset(self.h, C.byref(cur), self._stream()), self.h)
        else:
            torch = _torch()
            prev = self.t_state.cpu().numpy()
            lay = np.stack([self.layout.draw(self._rngs[k], prev[k]).pack() for k in range(self.num_envs)])
            assert lay.shape[1] == self.lib.lsm_layout_doubles(self.h)
            self._layout_dev = torch.as_tensor(lay, dtype=torch.float64, device=self.device).contiguous()
            capi.check(self.lib.lsm_reset_layout(self.h, C.byref(cur), C.c_void_p(self._layout_dev.data_ptr()),
                                                 self._stream()), self.h)
        ep = self._ep_info_all()
        if self.return_numpy:
            return (self._host64(self.t_obs), self.agent_id.cpu().numpy(), self._host64(self.t_node),
                    self._host64(self.reference_adj()), ep)
        return self.t_obs, self.agent_id, self.t_node, self.t_adj, ep

    @staticmethod
    def _host64(t):
        """Host copy with the reference's float64 dtype (values are the kernel's float32 ones)."""
        return t.cpu().numpy().astype(np.float64)

    def _ep_info_all(self):
        e = self.t_epinfo.cpu().numpy()
        return tuple({k: float(e[i, j]) for j, k in enumerate(EPKEYS)} for i in range(self.num_envs))

    def _actions_device(self, actions):
        torch = _torch()
        # fast path, no torch op calls: the runner's (n, N) int32 device tensor as it already is
        # (each .to() / .contiguous() is a dispatcher round with device guards on the host; a
        # 20-step window's first step paid ~100 us of host time before its launch:
        # profiles/r05_s28_window_attrib.txt)
        if isinstance(actions, torch.Tensor) and actions.dtype == torch.int32 and actions.dim() == 2 and \
                actions.device == self.device and actions.is_contiguous():
            return actions, capi.LSM_ACTIONS_INDEX_I32
        if isinstance(actions, torch.Tensor):
            t = actions.to(self.device)
        else:
            host = np.asarray(actions)
            if host.ndim == 2 and host.size and (host.min() < 0 or host.max() > 24):
                raise ValueError("action indices must be in [0, 25) (Discrete(25))")
            t = torch.as_tensor(host, device=self.device)
        if t.dim() == 2:
            return t.to(torch.int32).contiguous(), capi.LSM_ACTIONS_INDEX_I32
        if t.dim() == 3 and t.shape[-1] == 25:
            if t.dtype == torch.float64:
                return t.contiguous(), capi.LSM_ACTIONS_ONEHOT_F64
            return t.to(torch.float32).contiguous(), capi.LSM_ACTIONS_ONEHOT_F32
        raise ValueError("actions must be (n_envs, N) indices or (n_envs, N, 25) one-hot")

    def _curriculum(self, ep):
        c = self._cur_cache.get(ep)
        if c is None:
            block = curriculum_block(self.args, ep)
            c = self._cur_cache[ep] = (block, to_struct(block))
        return c

    def step_async(self, actions, num_current_episode: Optional[int] = None):
        ep = self._last_ep if num_current_episode is None else num_current_episode
        block, cur = self._curriculum(ep)
        act, kind = self._actions_device(actions)
        capi.check(self.lib.lsm_step(self.h, C.c_void_p(act.data_ptr()), kind, C.byref(cur), self._stream()),
                   self.h)
        self._pending = (act, block)

    def step_wait(self):
        self._pending = None
        # shared reward (collaborative): each worker returns [[sum]] * N, stacked (n, N, 1)
        # (environment.py:1031-1037, env_wrappers.py:988-996); else (n, N)
        t_rew = self.t_rew.unsqueeze(-1) if self.collaborative else self.t_rew
        if not self.return_numpy:
            out = (self.t_obs, self.agent_id, self.t_node, self.t_adj, t_rew, self.t_done,
                   (self.t_info, self.t_reset, self.t_epinfo))
            return out + (0,) if not self.auto_reset else out
        self.check_actions()   # the host copies below synchronise anyway
        obs = self._host64(self.t_obs)
        node = self._host64(self.t_node)
        adj = self._host64(self.reference_adj())
        rew = self._host64(t_rew)
        dones = self.t_done.cpu().numpy().astype(bool)
        infos = self._infos() if self.build_infos else None
        aid = self.agent_id.cpu().numpy()
        if self.auto_reset:
            return obs, aid, node, adj, rew, dones, infos
        return obs, aid, node, adj, rew, dones, infos, 0

    def check_actions(self):
        """Raise if a step since the last check got an index action outside [0, 25) from a device
        tensor (the kernel clamps it to stay in bounds and flags it). Synchronises."""
        v = self.lib.lsm_action_errors(self.h, self._stream())
        if v < 0:
            raise capi.LsmError("lsm_action_errors failed")
        if v:
            raise ValueError("an action index outside [0, 25) (Discrete(25)) reached the rollout")

    def step(self, actions, num_current_episode: Optional[int] = None):
        self.step_async(actions, num_current_episode)
        return self.step_wait()

    def _infos(self):
        reset = self.t_reset.cpu().numpy()
        return infos_from_arrays(self.t_info.cpu().numpy(), reset,
                                 self.t_epinfo.cpu().numpy() if reset.any() else None, self.auto_reset,
                                 None if self.t_departed is None else self.t_departed.cpu().numpy())

    def reference_adj(self):
        """The adjacency in the reference layout [n, N, E, E] (device tensor). In the compact
        layout it is expanded from the table and the per-ego masks (torch ops on the device)."""
        if self.t_adj_mask is None:
            return self.t_adj
        return expand_compact_adj(self.t_adj, self.t_adj_mask, self.E)

    def edge_list(self):
        """The learner's graph input for the current per-ego adjacencies, as GNNBase.process_adj
        (gnn.py:376-407) returns it for the runner's (n*N, E, E) batch: (edge_index int64 [2, nnz],
        edge_attr float32 [nnz, 1]), built on the GPU from either adjacency layout."""
        from . import edges
        if self.t_adj_mask is None:
            return edges.process_adj(self.t_adj.view(-1, self.E, self.E), counts=self.t_adj_nnz)
        return edges.process_adj_compact(self.t_adj, self.t_adj_mask, self.N, counts=self.t_adj_nnz)

    def set_agent_state(self, env_index: int, agent_state, reached=None):
        """Overwrite one env's agent states ([N][4]) and optionally reached_goal ([N])."""
        st = np.ascontiguousarray(agent_state, dtype=np.float64).reshape(self.N, 4)
        rp = None if reached is None else np.ascontiguousarray(reached, dtype=np.int32).reshape(self.N)
        capi.check(self.lib.lsm_set_agent_state(
            self.h, int(env_index), st.ctypes.data_as(C.c_void_p),
            None if rp is None else rp.ctypes.data_as(C.c_void_p), self._stream()), self.h)

    def state(self):
        """Agent states [n, N, 4] (float64) after the last call (positions/velocities)."""
        return self.t_state

    def close_extras(self):
        self.close()

    def close(self):
        if not self.closed and getattr(self, "h", None):
            _torch().cuda.synchronize(self.device)
            self.lib.lsm_destroy(self.h)
            self.h = None
        self.closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
