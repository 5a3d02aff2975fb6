"""jax stub (test infrastructure): only ``jax.numpy`` is used by the reference
(``multiagent/safety_filter.py:4``). JAX runs with x64 disabled, so the stub's
``jax.numpy`` produces float32 arrays."""
from . import numpy  # noqa: F401
