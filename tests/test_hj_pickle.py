"""Value / TTR pickle ingestion (HjDataHandle, safety_filter.py:154-168; TTR load,
navigation_graph_safe.py:128-138) through lsm.hj_tables' non-executing unpickler: arrays and grid
meta come back from pickles of classes that do not exist here, and nothing a pickle names runs."""
import os
import pickle
import sys
import types

import numpy as np

from lsm import hj_tables


def _fake_module(name):
    parts = name.split(".")
    for k in range(1, len(parts) + 1):   # the package chain must import
        sys.modules.setdefault(".".join(parts[:k]), types.ModuleType(".".join(parts[:k])))
    return sys.modules[name]


def _write_reference_like_pickle(path, values, lo, hi, periodic, sep=None, ttr_max=None):
    """Pickle objects of classes living in modules absent at load time (like the reference's
    hj_reachability_utils objects), then drop the modules."""
    mod = _fake_module("hj_reachability_utils_fake.common")

    class GridMetaData:
        pass

    class ValueData:
        pass

    for c in (GridMetaData, ValueData):
        c.__module__ = mod.__name__
        c.__qualname__ = c.__name__
        setattr(mod, c.__name__, c)
    meta = GridMetaData()
    meta.lo, meta.hi, meta.shape, meta.periodic_dims = np.asarray(lo), np.asarray(hi), values.shape, list(periodic)
    obj = ValueData()
    obj.values, obj.grid_meta_data = values, meta
    if sep is not None:
        obj.info = {"separation_distance": sep}
    if ttr_max is not None:
        obj.ttr_max = ttr_max
    with open(path, "wb") as f:
        pickle.dump(obj, f)
    for k in [k for k in sys.modules if k.startswith("hj_reachability_utils_fake")]:
        del sys.modules[k]


def test_reference_like_value_pickle_round_trip(tmp_path):
    st = hj_tables.synthetic_di_stored((9, 9, 5, 5))
    p = tmp_path / "vf.pkl"
    _write_reference_like_pickle(p, st["values"], st["lo"], st["hi"], (), sep=0.5)
    d = hj_tables.load_stored_pickle(str(p))
    np.testing.assert_array_equal(d["values"], st["values"])
    np.testing.assert_array_equal(d["lo"], st["lo"])
    np.testing.assert_array_equal(d["hi"], st["hi"])
    assert d["shape"] == (9, 9, 5, 5) and d["periodic"] == () and d["separation_distance"] == 0.5
    vt = hj_tables.value_table_from_stored(d, 0.5)
    ref = hj_tables.value_table_from_stored(dict(st, separation_distance=0.5), 0.5)
    np.testing.assert_array_equal(vt.values_hj, ref.values_hj)
    np.testing.assert_array_equal(vt.grads_hj, ref.grads_hj)


def test_ttr_pickle_periodic_and_ttr_max(tmp_path):
    vals = np.random.default_rng(0).random((5, 5, 6, 3)).astype(np.float32)
    p = tmp_path / "ttr.pkl"
    _write_reference_like_pickle(p, vals, [-6, -6, -np.pi, 0.03], [6, 6, np.pi, 0.09], (2,), ttr_max=200.0)
    d = hj_tables.load_stored_pickle(str(p))
    np.testing.assert_array_equal(d["values"], vals)
    assert d["periodic"] == (2,) and d["ttr_max"] == 200.0


class _Evil:
    def __init__(self, marker):
        self.marker = marker

    def __reduce__(self):
        return (os.system, ("touch %s" % self.marker,))


def test_unpickler_executes_nothing(tmp_path):
    marker = tmp_path / "pwned"
    p = tmp_path / "evil.pkl"
    with open(p, "wb") as f:
        pickle.dump({"values": np.zeros(3, np.float32), "payload": _Evil(str(marker))}, f)
    obj = hj_tables.safe_load_pickle(str(p))
    assert not marker.exists()
    assert isinstance(obj["payload"], hj_tables._Inert)
    np.testing.assert_array_equal(obj["values"], np.zeros(3, np.float32))
