"""HJ value-function / TTR tables: synthetic builders, pickle ingestion, gradients.

Host-side setup code (runs once, not on the per-step path). Mirrors what
``HjDataHandle`` does at load time (``multiagent/safety_filter.py:154-174``):

* ``values_hj = -stored_values - shift`` with ``shift = target_separation -
  stored_separation`` (float32 arithmetic, like the reference's numpy/JAX array);
* ``grads_hj = grid.grad_values(values_hj)`` -- the gradient scheme of the absent
  ``hj_reachability`` 0.5.0 is not pinned offline; this build uses the central
  average of the upwind first differences (one-sided at non-periodic edges,
  wrap-around on periodic dims), see DESIGN.md "Parity".

The real pickles (``data/crazyflies_value_function.pkl`` ...) live on Google
Drive and are absent; synthetic tables with the SURVEY §8(d) shapes stand in.
Device layout: values float32 [n_nodes]; grads float32 [n_nodes][4] for 4-D
tables (one 16-byte load per corner) and [n_nodes][5] padded to [n_nodes][8]
for 5-D tables (two 16-byte loads per corner).
"""
from __future__ import annotations

import math
import pickle
from dataclasses import dataclass, field

import numpy as np

from .config import AirTaxiConfig, DoubleIntegratorConfig

F32 = np.float32


@dataclass
class HjTable:
    lo: np.ndarray
    hi: np.ndarray
    shape: tuple
    periodic: tuple
    values_hj: np.ndarray            # float32, grid.shape (already negated/shifted)
    grads_hj: np.ndarray = None      # float32, grid.shape + (ndim,)
    separation_distance: float = 0.0
    ttr_max: float = float("nan")
    extra: dict = field(default_factory=dict)

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def spacings(self):
        n = np.asarray(self.shape, dtype=np.float64)
        per = np.zeros(self.ndim, dtype=bool)
        for d in self.periodic:
            per[d] = True
        return np.where(per, (self.hi - self.lo) / n, (self.hi - self.lo) / (n - 1.0))

    def device_grads(self):
        """Grads padded to 4 or 8 float32 per node for 16-byte corner loads."""
        g = np.ascontiguousarray(self.grads_hj, dtype=F32).reshape(-1, self.ndim)
        width = 4 if self.ndim <= 4 else 8
        out = np.zeros((g.shape[0], width), dtype=F32)
        out[:, :self.ndim] = g
        return out


def grad_values(values, lo, hi, shape, periodic=()):
    """Central average of upwind first differences (float64 math, float32 out)."""
    v = np.asarray(values, dtype=np.float64)
    ndim = len(shape)
    n = np.asarray(shape, dtype=np.float64)
    lo = np.asarray(lo, dtype=np.float64)
    hi = np.asarray(hi, dtype=np.float64)
    per = [d in periodic for d in range(ndim)]
    grads = []
    for d in range(ndim):
        h = (hi[d] - lo[d]) / n[d] if per[d] else (hi[d] - lo[d]) / (n[d] - 1.0)
        if per[d]:
            left = (v - np.roll(v, 1, axis=d)) / h
            right = (np.roll(v, -1, axis=d) - v) / h
        else:
            diff = np.diff(v, axis=d) / h
            left = np.concatenate([np.take(diff, [0], axis=d), diff], axis=d)
            right = np.concatenate([diff, np.take(diff, [diff.shape[d] - 1], axis=d)], axis=d)
        grads.append(0.5 * (left + right))
    return np.stack(grads, axis=-1).astype(F32)


def _axes(lo, hi, shape, periodic):
    axes = []
    for d, n in enumerate(shape):
        if d in periodic:
            axes.append(lo[d] + (hi[d] - lo[d]) / n * np.arange(n))
        else:
            axes.append(np.linspace(lo[d], hi[d], n))
    return axes


# -- synthetic tables ------------------------------
DI_SHAPE_FULL = (61, 61, 41, 41)
AT_SHAPE_FULL = (41, 41, 36, 9, 9)
TTR_SHAPE_FULL = (41, 41, 36, 9)


def synthetic_di_stored(shape=DI_SHAPE_FULL, separation=0.5, brake=1.0):
    """Stored DI table (values = -V): V = |p| - sep - max(0, -rdot)^2 / (2 brake)."""
    lo = np.array([-4.5, -4.5, -1.0, -1.0])
    hi = np.array([4.5, 4.5, 1.0, 1.0])
    x, y, dvx, dvy = np.meshgrid(*_axes(lo, hi, shape, ()), indexing="ij")
    r = np.sqrt(x * x + y * y)
    rdot = np.where(r > 0, (x * dvx + y * dvy) / np.where(r > 0, r, 1.0), 0.0)
    V = r - separation - np.maximum(0.0, -rdot) ** 2 / (2.0 * brake)
    return dict(values=(-V).astype(F32), lo=lo, hi=hi, shape=tuple(shape), periodic=(),
                separation_distance=separation)


def synthetic_airtaxi_stored(shape=AT_SHAPE_FULL, separation=None, horizon=15.0):
    """Stored airtaxi table (values = -V) over (x_r, y_r, dtheta, v_a, v_b), dtheta periodic."""
    if separation is None:
        separation = AirTaxiConfig.SEPARATION_DISTANCE
    vlo, vhi = 0.95 * AirTaxiConfig.V_MIN, 1.05 * AirTaxiConfig.V_MAX
    lo = np.array([-6.0, -6.0, -math.pi, vlo, vlo])
    hi = np.array([6.0, 6.0, math.pi, vhi, vhi])
    x, y, th, va, vb = np.meshgrid(*_axes(lo, hi, shape, (2,)), indexing="ij")
    r = np.sqrt(x * x + y * y)
    rvx = vb * np.cos(th) - va
    rvy = vb * np.sin(th)
    rdot = np.where(r > 0, (x * rvx + y * rvy) / np.where(r > 0, r, 1.0), 0.0)
    V = r - separation - np.maximum(0.0, -rdot) * horizon
    return dict(values=(-V).astype(F32), lo=lo, hi=hi, shape=tuple(shape), periodic=(2,),
                separation_distance=separation)


def synthetic_ttr(shape=TTR_SHAPE_FULL, ttr_max=200.0):
    """Synthetic airtaxi time-to-reach table: ttr = |p_rel| / V_MAX, clipped at ttr_max."""
    vlo, vhi = 0.95 * AirTaxiConfig.V_MIN, 1.05 * AirTaxiConfig.V_MAX
    lo = np.array([-6.0, -6.0, -math.pi, vlo])
    hi = np.array([6.0, 6.0, math.pi, vhi])
    x, y, th, v = np.meshgrid(*_axes(lo, hi, shape, (2,)), indexing="ij")
    ttr = np.minimum(np.sqrt(x * x + y * y) / AirTaxiConfig.V_MAX + 5.0 * (1.0 - np.cos(th)), ttr_max)
    return dict(values=ttr.astype(F32), lo=lo, hi=hi, shape=tuple(shape), periodic=(2,),
                ttr_max=float(ttr_max))


def value_table_from_stored(stored: dict, target_separation: float) -> HjTable:
    """``HjDataHandle.__init__`` (safety_filter.py:155-168)."""
    shift = target_separation - stored["separation_distance"]
    values_hj = (-stored["values"] - shift).astype(F32)
    t = HjTable(lo=np.asarray(stored["lo"], np.float64), hi=np.asarray(stored["hi"], np.float64),
                shape=tuple(stored["shape"]), periodic=tuple(stored["periodic"]),
                values_hj=values_hj, separation_distance=target_separation)
    t.grads_hj = grad_values(values_hj, t.lo, t.hi, t.shape, t.periodic)
    return t


def ttr_table_from_stored(stored: dict) -> HjTable:
    return HjTable(lo=np.asarray(stored["lo"], np.float64), hi=np.asarray(stored["hi"], np.float64),
                   shape=tuple(stored["shape"]), periodic=tuple(stored["periodic"]),
                   values_hj=np.ascontiguousarray(stored["values"], dtype=F32),
                   ttr_max=float(stored["ttr_max"]))


# ---- pickle ingestion that executes nothing from the file ----------------------------------
# The reference's value/TTR pickles hold hj_reachability / hj_reachability_utils objects
# (HjDataHandle, safety_filter.py:154-168; navigation_graph_safe.py:128-138) whose classes are absent
# here. The unpickler below resolves only numpy's array/dtype reconstructors, codecs.encode and inert
# builtin containers; every other global (a class or ANY callable, e.g. os.system) becomes an inert
# stand-in that merely records its arguments and state. Arrays are then found by attribute name.

_NP_OK = {"_reconstruct", "ndarray", "dtype", "scalar", "_frombuffer"}
_BUILTIN_OK = {"dict", "list", "tuple", "set", "frozenset", "slice", "complex", "float", "int",
               "bytearray", "bytes", "str", "bool", "range"}


class _Inert:
    """Stand-in for any global the safe unpickler will not resolve: calling it (REDUCE) or
    constructing it (NEWOBJ) only stores the arguments; BUILD stores the state."""

    def __init__(self, *args, **kwargs):
        self._args, self._kwargs = args, kwargs

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2 and isinstance(state[1], dict):
            state = {**(state[0] or {}), **state[1]}   # (dict, slotstate)
        if isinstance(state, dict):
            self.__dict__.update(state)
        else:
            self._state = state

    def __getattr__(self, name):   # missing attributes of a stand-in are absent, never computed
        raise AttributeError(name)


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        top = module.split(".")[0]
        if top == "numpy" and name in _NP_OK:
            return super().find_class(module, name)
        if module == "_codecs" and name == "encode":
            return super().find_class(module, name)
        if module == "builtins" and name in _BUILTIN_OK:
            return super().find_class(module, name)
        return type(name, (_Inert,), {"__module__": "lsm.hj_tables.inert." + module})


def _find_array(x, depth=0):
    """First ndarray inside x (an array, an array-like stand-in such as a pickled jax Array, or a
    container of them)."""
    if isinstance(x, np.ndarray):
        return x
    if depth > 6:
        return None
    if isinstance(x, (list, tuple)):
        items = x
    elif isinstance(x, dict):
        items = list(x.values())
    elif isinstance(x, _Inert):
        items = list(getattr(x, "_args", ())) + list(x.__dict__.values())
        if "_state" in x.__dict__:
            items.append(x.__dict__["_state"])
    else:
        return None
    for it in items:
        a = _find_array(it, depth + 1)
        if a is not None:
            return a
    return None


def _get(obj, name, default=None):
    if isinstance(obj, dict):
        return obj.get(name, default)
    return obj.__dict__.get(name, default) if hasattr(obj, "__dict__") else getattr(obj, name, default)


def safe_load_pickle(path: str):
    """Unpickle ``path`` without executing anything it names (see _SafeUnpickler)."""
    with open(path, "rb") as f:
        return _SafeUnpickler(f).load()


def load_stored_pickle(path: str) -> dict:
    """Read a value / TTR pickle (``.values``, ``.grid_meta_data`` {lo, hi, shape, periodic_dims},
    ``.info['separation_distance']``, ``.ttr_max``) through the non-executing unpickler."""
    obj = safe_load_pickle(path)
    meta = _get(obj, "grid_meta_data")
    if meta is None:
        raise ValueError("%s: no grid_meta_data" % path)
    vals = _find_array(_get(obj, "values"))
    if vals is None:
        raise ValueError("%s: no values array" % path)
    lo, hi = _find_array(_get(meta, "lo")), _find_array(_get(meta, "hi"))
    lo = np.asarray(lo if lo is not None else _get(meta, "lo"), dtype=np.float64)
    hi = np.asarray(hi if hi is not None else _get(meta, "hi"), dtype=np.float64)
    shape = _get(meta, "shape")
    shape = tuple(int(v) for v in (shape if shape is not None else vals.shape))
    per = _get(meta, "periodic_dims", ()) or ()
    per = _find_array(per) if not isinstance(per, (list, tuple)) else per
    d = dict(values=np.asarray(vals, dtype=F32), lo=lo, hi=hi, shape=shape,
             periodic=tuple(int(v) for v in np.asarray(per).reshape(-1)) if per is not None else ())
    info = _get(obj, "info")
    if info is not None and _get(info, "separation_distance") is not None:
        d["separation_distance"] = float(_get(info, "separation_distance"))
    if _get(obj, "ttr_max") is not None:
        d["ttr_max"] = float(_get(obj, "ttr_max"))
    return d


def default_tables(dynamics: str, small: bool = False, target_separation=None):
    """(value_table, ttr_table) for a dynamics type; ``small`` shrinks the grids for tests.
    ``target_separation``: what HjDataHandle is built with (the scenario's
    separation_distance_init; default the config's SEPARATION_DISTANCE)."""
    if dynamics == "double_integrator":
        shape = (31, 31, 21, 21) if small else DI_SHAPE_FULL
        st = synthetic_di_stored(shape)
        sep = DoubleIntegratorConfig.SEPARATION_DISTANCE if target_separation is None else target_separation
        return value_table_from_stored(st, sep), None
    shape = (25, 25, 24, 7, 7) if small else AT_SHAPE_FULL
    tshape = (25, 25, 24, 7) if small else TTR_SHAPE_FULL
    st = synthetic_airtaxi_stored(shape)
    sep = AirTaxiConfig.SEPARATION_DISTANCE if target_separation is None else target_separation
    return (value_table_from_stored(st, sep), ttr_table_from_stored(synthetic_ttr(tshape)))
