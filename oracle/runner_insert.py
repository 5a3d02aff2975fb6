"""TEST INFRASTRUCTURE ONLY (checker, never the product path): numpy restatement of the env-side
rows of ``GMPERunner.warmup`` / ``insert`` and ``GraphReplayBuffer.insert`` / ``after_update``.

References: ``onpolicy/runner/shared/graph_mpe_runner.py:253-283`` (warmup: buffer row 0),
``:444-487`` (insert: masks / active_masks / share_obs / share_agent_id), and
``onpolicy/utils/graph_buffer.py:223-249`` (rows t+1, rewards at t), ``:253-283`` (after_update).
"""
from __future__ import annotations

import numpy as np


def insert_rows(obs, agent_id, dones=None, centralized=True):
    """Returns dict of the derived rows for one buffer index (graph_mpe_runner.py:449-484)."""
    n, N = obs.shape[:2]
    out = {}
    if dones is not None:
        dones = np.asarray(dones, dtype=bool)
        dones_env = np.all(dones, axis=1)
        masks = np.ones((n, N, 1), dtype=np.float32)
        masks[dones] = np.zeros(((dones).sum(), 1), dtype=np.float32)
        active = np.ones((n, N, 1), dtype=np.float32)
        active[dones] = np.zeros((dones.astype(int).sum(), 1), dtype=np.float32)
        active[dones_env] = np.ones((dones_env.astype(int).sum(), N, 1), dtype=np.float32)
        out["masks"], out["active_masks"] = masks, active
    if centralized:
        so = obs.reshape(n, -1)
        out["share_obs"] = np.expand_dims(so, 1).repeat(N, axis=1).astype(np.float32)
        sa = agent_id.reshape(n, -1)
        out["share_agent_id"] = np.expand_dims(sa, 1).repeat(N, axis=1).astype(np.int32)
    else:
        out["share_obs"] = obs.astype(np.float32)
        out["share_agent_id"] = agent_id.astype(np.int32)
    out["agent_id"] = agent_id.astype(np.int32)
    return out
