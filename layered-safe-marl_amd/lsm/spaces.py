"""Minimal gym-compatible space objects (gym is not a dependency of the product).

Same attributes the onpolicy runner reads: ``Box.shape``, ``Discrete.n``
(``onpolicy/runner/shared/base_runner.py:106-143``,
``multiagent/environment.py:143-202,928-960``).
"""
from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def __repr__(self):
        return "Discrete(%d)" % self.n


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.low = low
        self.high = high
        self.shape = tuple(shape)
        self.dtype = dtype

    def __repr__(self):
        return "Box(%s)" % (self.shape,)
