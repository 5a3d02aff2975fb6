"""Restated semantics of the absent third-party HJ grid (TEST INFRASTRUCTURE ONLY).

ORACLE -- test infrastructure. Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module. The product path
never routes through it.

The reference calls ``hj_reachability`` 0.5.0 (``requirements.txt:5``, not
installed here, no network) for three things:

* ``Grid.interpolate(values, state)`` -- ``multiagent/safety_filter.py:195,245,348,418``,
  ``multiagent/core.py:463``, ``multiagent/custom_scenarios/navigation_graph_safe.py:751``;
* ``Grid.grad_values(values)`` -- ``safety_filter.py:167`` (precomputed once);
* ``sets.Box.extreme_point(direction)`` -- via ``optimal_control``
  (``safety_filter.py:70-77,250,423``).

None of these is pinned by anything in the reference repository, so this module
*defines* the semantics the build follows ("parity unpinned" for the numerics
below; the reference's own control flow around them is pinned by
``tests/golden``):

Interpolation (float32 throughout, like JAX with x64 disabled):
  ``p_d = (f32(s_d) - f32(lo_d)) / f32(spacing_d)``;
  non-periodic dims: out of domain (NaN, i.e. ``state_in_hj_range == False``)
  unless ``0 <= p_d <= n_d - 1``; ``i_d = min(floor(p_d), n_d - 2)``;
  periodic dims: ``i_d = floor(p_d) mod n_d``, upper neighbour ``(i_d+1) mod n_d``;
  ``w_hi = p_d - i_d`` (before the modulo), ``w_lo = 1 - w_hi``;
  corner weight ``((w_0 * w_1) * w_2) * ...`` (the ``jnp.ix_`` outer-product
  reduce), corners summed sequentially in lexicographic order (dim 0 slowest).
Gradient table: central difference of the one-sided (upwind) first differences,
  i.e. ``(left + right) / 2`` with one-sided differences at non-periodic edges
  and wrap-around on periodic dims, computed in float64 and stored float32.
Box.extreme_point(direction): ``where(direction < 0, lo, hi)`` in float32.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


class Grid:
    """Regular grid with optional periodic dims (restated ``hj.Grid``)."""

    def __init__(self, lo, hi, shape, periodic_dims=()):
        self.lo = np.asarray(lo, dtype=np.float64)
        self.hi = np.asarray(hi, dtype=np.float64)
        self.shape = tuple(int(s) for s in shape)
        self.ndim = len(self.shape)
        self.periodic = np.zeros(self.ndim, dtype=bool)
        for d in periodic_dims:
            self.periodic[d] = True
        # hj_reachability lattice convention: periodic dims exclude the upper bound.
        n = np.asarray(self.shape, dtype=np.float64)
        self.spacings = np.where(self.periodic, (self.hi - self.lo) / n,
                                 (self.hi - self.lo) / (n - 1.0))
        self.lo32 = self.lo.astype(F32)
        self.sp32 = self.spacings.astype(F32)

    @property
    def strides(self):
        s = [1] * self.ndim
        for d in range(self.ndim - 2, -1, -1):
            s[d] = s[d + 1] * self.shape[d + 1]
        return s

    # -- interpolation -------------------------------------------------------
    def corners(self, state):
        """Return (flat_indices[2^d], weights[2^d] float32) or None if out of domain."""
        s32 = np.asarray(state, dtype=np.float64).astype(F32)
        pos = (s32 - self.lo32) / self.sp32          # float32 arithmetic
        idx_lo = np.zeros(self.ndim, dtype=np.int64)
        idx_hi = np.zeros(self.ndim, dtype=np.int64)
        w_hi = np.zeros(self.ndim, dtype=F32)
        for d in range(self.ndim):
            p = pos[d]
            if not np.isfinite(p):
                return None
            n = self.shape[d]
            f = int(np.floor(p))
            if self.periodic[d]:
                w_hi[d] = F32(p - F32(f))
                idx_lo[d] = f % n
                idx_hi[d] = (f + 1) % n
            else:
                if p < F32(0.0) or p > F32(n - 1):
                    return None
                f = min(f, n - 2)
                w_hi[d] = F32(p - F32(f))
                idx_lo[d] = f
                idx_hi[d] = f + 1
        w_lo = (F32(1.0) - w_hi).astype(F32)
        # corner c takes dim d's upper neighbour iff bit (ndim-1-d) of c is set; its weight is
        # the sequential float32 product over dims (vectorised over corners, same roundings)
        bits = self._bits()
        wsel = np.where(bits, w_hi[None, :], w_lo[None, :]).astype(F32)
        w = wsel[:, 0].copy()
        for d in range(1, self.ndim):
            w = (w * wsel[:, d]).astype(F32)
        flat = (np.where(bits, idx_hi[None, :], idx_lo[None, :]) * np.asarray(self.strides)[None, :]).sum(axis=1)
        return flat.astype(np.int64), w

    def _bits(self):
        b = getattr(self, "_bits_cache", None)
        if b is None:
            c = np.arange(1 << self.ndim)[:, None]
            b = ((c >> (self.ndim - 1 - np.arange(self.ndim))[None, :]) & 1).astype(bool)
            self._bits_cache = b
        return b

    def interpolate(self, values, state):
        """Interpolate ``values`` (grid.shape [+ trailing dims]) at ``state``.

        Returns float32 scalar / vector, NaN(s) when out of domain. The weighted corners are
        summed sequentially in float32 (np.cumsum is a running sum).
        """
        values = np.asarray(values)
        trailing = values.shape[self.ndim:]
        cw = self.corners(state)
        if cw is None:
            return np.full(trailing, np.nan, dtype=F32) if trailing else F32(np.nan)
        flat, wts = cw
        vflat = values.reshape((-1,) + trailing)[flat]
        prod = (wts.reshape((-1,) + (1,) * len(trailing)) * vflat).astype(F32)
        acc = np.cumsum(prod, axis=0, dtype=F32)[-1]
        return acc if trailing else F32(acc)

    # -- gradients -------------------------------------------------------------
    def grad_values(self, values):
        """Central average of upwind first differences, float64 math, float32 out."""
        v = np.asarray(values, dtype=np.float64)
        grads = []
        for d in range(self.ndim):
            h = self.spacings[d]
            if self.periodic[d]:
                left = (v - np.roll(v, 1, axis=d)) / h
                right = (np.roll(v, -1, axis=d) - v) / h
            else:
                diff = np.diff(v, axis=d) / h
                pad_first = np.take(diff, [0], axis=d)
                pad_last = np.take(diff, [diff.shape[d] - 1], axis=d)
                left = np.concatenate([pad_first, diff], axis=d)
                right = np.concatenate([diff, pad_last], axis=d)
            grads.append(0.5 * (left + right))
        return np.stack(grads, axis=-1).astype(F32)


def box_extreme_point(lo, hi, direction):
    """Restated ``hj.sets.Box.extreme_point``: where(direction < 0, lo, hi), float32."""
    d = np.asarray(direction)
    return np.where(d < 0, np.asarray(lo, dtype=F32), np.asarray(hi, dtype=F32)).astype(F32)
