"""TEST INFRASTRUCTURE ONLY (checker, never the product path): numpy restatement of
``GNNBase.process_adj`` (reference ``onpolicy/algorithms/utils/gnn.py:376-407``).

gnn.py:392-399 (batched): ``edge_index = adj.nonzero()`` (row-major over (b, r, c)),
``edge_attr = adj[b, r, c]``, ``edge_index = stack([b*E + r, b*E + c])``; gnn.py:400-403 (2-D):
the same with b = 0; gnn.py:406: ``edge_attr.unsqueeze(1)``. numpy's ``nonzero`` has the same
C-order semantics as torch's (NaN counts as nonzero, -0.0 does not).
"""
from __future__ import annotations

import numpy as np


def process_adj(adj: np.ndarray):
    adj = np.asarray(adj)
    assert 2 <= adj.ndim <= 3 and adj.shape[-1] == adj.shape[-2]
    if adj.ndim == 3:
        b, r, c = np.nonzero(adj)
        attr = adj[b, r, c]
        E = adj.shape[1]
        ei = np.stack([b.astype(np.int64) * E + r, b.astype(np.int64) * E + c])
    else:
        r, c = np.nonzero(adj)
        attr = adj[r, c]
        ei = np.stack([r, c]).astype(np.int64)
    return ei.astype(np.int64), attr[:, None]


def expand_compact(table: np.ndarray, masks: np.ndarray) -> np.ndarray:
    """Reference-layout [n, N, E, E] from the compact layout (include/lsm_rollout.h
    LSM_ADJ_COMPACT): adj[e][r][c] = (M[e] bit r | M[e] bit c) ? 0 : A[r][c]."""
    n, E, _ = table.shape
    N = masks.shape[1]
    bits = np.zeros((n, N, E), dtype=bool)
    m = masks.view(np.uint64)
    for k in range(E):
        bits[:, :, k] = (m[:, :, k >> 6] >> np.uint64(k & 63)) & np.uint64(1)
    keep = ~(bits[:, :, :, None] | bits[:, :, None, :])
    return np.where(keep, table[:, None, :, :], np.float32(0))   # assignment semantics (NaN-safe)
