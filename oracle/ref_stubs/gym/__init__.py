"""Minimal gym stub (test infrastructure): Env base class + spaces."""
from . import spaces  # noqa: F401
from . import envs  # noqa: F401


class Env(object):
    metadata = {}

    def close(self):
        pass


class Space(object):
    def __init__(self, shape=None, dtype=None):
        self.shape = shape
        self.dtype = dtype
