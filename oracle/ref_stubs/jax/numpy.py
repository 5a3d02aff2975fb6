"""float32 numpy shim standing in for ``jax.numpy`` (x64 disabled)."""
import numpy as _np

float32 = _np.float32
int32 = _np.int32


def _f32(x):
    a = _np.asarray(x)
    if a.dtype == _np.bool_:
        return a
    return a.astype(_np.float32)


def array(obj, dtype=None):
    if isinstance(obj, (list, tuple)):
        obj = [_np.asarray(o, dtype=_np.float64) if not isinstance(o, (list, tuple)) else
               [_np.asarray(p, dtype=_np.float64) for p in o] for o in obj]
        a = _np.array(obj, dtype=_np.float64)
    else:
        a = _np.asarray(obj)
    return a.astype(dtype) if dtype is not None else _f32(a)


asarray = array


def zeros(shape, dtype=None):
    return _np.zeros(shape, dtype=_np.float32)


def ones(shape, dtype=None):
    return _np.ones(shape, dtype=_np.float32)


def eye(n, dtype=None):
    return _np.eye(n, dtype=_np.float32)


def where(cond, a, b):
    return _np.where(cond, _f32(a), _f32(b)).astype(_np.float32)


def cos(x):
    return _np.cos(_f32(x)).astype(_np.float32)


def sin(x):
    return _np.sin(_f32(x)).astype(_np.float32)


def stack(xs, axis=0):
    return _np.stack([_f32(x) for x in xs], axis=axis)
