"""Device-resident ``GraphReplayBuffer`` rows filled by the rollout with no copies.

Mirrors the env-produced fields of ``onpolicy/utils/graph_buffer.py:84-163`` (share_obs, obs,
node_obs, adj, agent_id, share_agent_id, rewards, masks, bad_masks, active_masks; same shapes and
dtypes, as torch tensors on the env's GPU) and the env-side halves of ``GMPERunner.warmup``
(``graph_mpe_runner.py:253-283``), ``GMPERunner.insert`` (``:444-487``) and
``GraphReplayBuffer.after_update`` (``graph_buffer.py:253-283``).

The rollout kernel writes obs / node_obs / adj into row t+1 and rewards into row t directly: the
env's output slots are ring-bound to the buffer (``lsm_bind_output_ring``), one ring index per
buffer row, so selecting a row is a host-side pointer choice. With a centralized critic
(``use_centralized_V``, the reference default) the kernel also writes that row's share_obs, masks and
active_masks (optional output slots); otherwise ``lsm_buffer_insert`` (HIP) derives them from the
step's obs and dones. agent_id / share_agent_id rows are constant and filled once. Policy-side fields (rnn states, actions, values, log-probs) stay with the learner.
"""
from __future__ import annotations

import ctypes as C

from . import capi


class BufferError(RuntimeError):
    pass


class DeviceGraphBuffer:
    def __init__(self, env, episode_length=None, use_centralized_V: bool = True):
        import torch
        if env.return_numpy:
            # ring-bound outputs are never written to the env's own tensors: host copies of them
            # would be stale and cost a sync per step
            raise BufferError("DeviceGraphBuffer needs an env built with return_numpy=False")
        self.env = env
        self.lib = capi.load_library()
        self.T = int(episode_length or env.args.episode_length)
        self.centralized = bool(use_centralized_V)
        n, N, E, F, OBS = env.num_envs, env.N, env.E, env.F, env.OBS
        dev = env.device
        f32, i32 = torch.float32, torch.int32
        T1 = self.T + 1
        self.share_obs = torch.zeros((T1, n, N, N * OBS if self.centralized else OBS), dtype=f32, device=dev)
        self.obs = torch.zeros((T1, n, N, OBS), dtype=f32, device=dev)
        self.node_obs = torch.zeros((T1, n, N, E, F), dtype=f32, device=dev)
        if env.t_adj_mask is None:
            self.adj = torch.zeros((T1, n, N, E, E), dtype=f32, device=dev)
            self.adj_mask = None
        else:   # compact layout: one table per env + per-ego masks (expand with vec_env.expand_compact_adj)
            self.adj = torch.zeros((T1, n, E, E), dtype=f32, device=dev)
            self.adj_mask = torch.zeros((T1,) + tuple(env.t_adj_mask.shape), dtype=torch.int64, device=dev)
        self.agent_id = torch.zeros((T1, n, N, 1), dtype=i32, device=dev)
        self.share_agent_id = torch.zeros((T1, n, N, N if self.centralized else 1), dtype=i32, device=dev)
        self.rewards = torch.zeros((self.T, n, N, 1), dtype=f32, device=dev)
        self.masks = torch.ones((T1, n, N, 1), dtype=f32, device=dev)
        self.bad_masks = torch.ones_like(self.masks)
        self.active_masks = torch.ones_like(self.masks)
        self.step = 0
        # agent ids are the same every row (the env returns agent index j for agent j)
        ids = torch.arange(N, dtype=i32, device=dev)
        self.agent_id.copy_(ids.view(1, 1, N, 1).expand_as(self.agent_id))
        self.share_agent_id.copy_((ids.view(1, 1, 1, N) if self.centralized else ids.view(1, 1, N, 1))
                                  .expand_as(self.share_agent_id))
        # centralized critic: the rollout kernel also writes share_obs / masks / active_masks rows
        # (LSM_OUT_SHARE_OBS / _MASKS / _ACTIVE_MASKS); otherwise lsm_buffer_insert derives them
        self.fused = self.centralized
        self._bind()
        # per-row kernel arguments, built once (the per-step host path is two ctypes calls)
        self._rows = [tuple(C.c_void_p(t[r].data_ptr()) for t in (self.obs, self.share_obs, self.agent_id,
                                                                  self.share_agent_id, self.masks,
                                                                  self.active_masks))
                      for r in range(T1)]
        self._done_ptr = C.c_void_p(env.t_done.data_ptr())

    # ring index i = buffer row i: obs-like rows at i, rewards at i - 1 (rewards[t] for step t)
    def _bind(self):
        rings = [(capi.OUT_OBS, self.obs, 0), (capi.OUT_NODE_OBS, self.node_obs, 0),
                 (capi.OUT_ADJ, self.adj, 0), (capi.OUT_REWARD, self.rewards, -1)]
        if self.adj_mask is not None:
            rings.append((capi.OUT_ADJ_MASK, self.adj_mask, 0))
        if self.fused:
            rings += [(capi.OUT_SHARE_OBS, self.share_obs, 0), (capi.OUT_MASKS, self.masks, 0),
                      (capi.OUT_ACTIVE_MASKS, self.active_masks, 0)]
        for slot, t, off in rings:
            stride = t[0].numel() * t.element_size()
            capi.check(self.lib.lsm_bind_output_ring(self.env.h, slot, C.c_void_p(t.data_ptr()), stride,
                                                     t.shape[0], off), self.env.h)

    def detach(self):
        """Unbind the rings: the env writes its own output tensors again."""
        for slot in (capi.OUT_OBS, capi.OUT_NODE_OBS, capi.OUT_ADJ, capi.OUT_REWARD, capi.OUT_ADJ_MASK,
                     capi.OUT_SHARE_OBS, capi.OUT_MASKS, capi.OUT_ACTIVE_MASKS):
            capi.check(self.lib.lsm_bind_output_ring(self.env.h, slot, None, 0, 0, 0), self.env.h)
        capi.check(self.lib.lsm_select_ring(self.env.h, -1), self.env.h)

    def _select(self, i):
        capi.check(self.lib.lsm_select_ring(self.env.h, int(i)), self.env.h)

    def _insert(self, row, with_dones):
        env = self.env
        o, so, aid, said, m, am = self._rows[row]
        rc = self.lib.lsm_buffer_insert(o, self._done_ptr if with_dones else None, env.num_envs, env.N, env.OBS,
                                        int(self.centralized), so, aid, said, m, am, env._stream())
        if rc != 0:
            raise BufferError(self.lib.lsm_buffer_last_error().decode())

    def warmup(self, num_current_episode: int = 0):
        """GMPERunner.warmup (graph_mpe_runner.py:253-283): reset into row 0. Returns ep_info."""
        self._select(0)
        ep = self.env.reset(num_current_episode)[-1]
        if not self.fused:
            self._insert(0, False)
        self.step = 0
        return ep

    def insert_step(self, actions, num_current_episode=None):
        """env.step + GMPERunner.insert's env-side rows for buffer step t = self.step: obs,
        node_obs, adj, share_obs, agent_id, share_agent_id, masks, active_masks at t+1 and
        rewards at t. Returns (dones [n, N] u8, (info, reset_flag, ep_info)) device tensors."""
        t = self.step
        self._select(t + 1)
        self.env.step_async(actions, num_current_episode)
        self.env.step_wait()
        if not self.fused:
            self._insert(t + 1, True)
        self.step = (t + 1) % self.T
        return self.env.t_done, (self.env.t_info, self.env.t_reset, self.env.t_epinfo)

    def after_update(self):
        """GraphReplayBuffer.after_update (graph_buffer.py:253-283), env-side fields."""
        fields = [self.share_obs, self.obs, self.node_obs, self.adj, self.agent_id, self.share_agent_id,
                  self.masks, self.active_masks, self.bad_masks]
        if self.adj_mask is not None:
            fields.append(self.adj_mask)
        for f in fields:
            f[0].copy_(f[-1])
