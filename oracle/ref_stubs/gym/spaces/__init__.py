"""Minimal gym.spaces stub (test infrastructure)."""
import numpy as np


class Discrete(object):
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def __repr__(self):
        return "Discrete(%d)" % self.n


class Box(object):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low = low
        self.high = high
        self.shape = tuple(shape) if shape is not None else np.shape(low)
        self.dtype = dtype

    def __repr__(self):
        return "Box(%s)" % (self.shape,)


class Tuple(object):
    def __init__(self, spaces):
        self.spaces = tuple(spaces)
