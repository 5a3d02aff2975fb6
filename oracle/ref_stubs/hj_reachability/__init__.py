"""hj_reachability 0.5.0 stub (test infrastructure). Semantics restated in oracle/hj_grid.py."""
from . import sets  # noqa: F401
