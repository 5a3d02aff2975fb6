"""Stub of ``hj_reachability_utils.common`` (test infrastructure).

Provides the three names the reference imports
(``multiagent/safety_filter.py:6-7``, ``navigation_graph_safe.py:24``) plus the
pickle payload classes written by ``tests/golden/make_golden.py``.
"""
import numpy as _np

from oracle.hj_grid import Grid


class GridMetaData(object):
    def __init__(self, lo, hi, shape, periodic_dims=()):
        self.lo = _np.asarray(lo, dtype=_np.float64)
        self.hi = _np.asarray(hi, dtype=_np.float64)
        self.shape = tuple(int(s) for s in shape)
        self.periodic_dims = tuple(int(d) for d in periodic_dims)


class HjValueData(object):
    """Payload of ``data/*_value_function.pkl`` (fields used at safety_filter.py:158-166)."""

    def __init__(self, values, grid_meta_data, separation_distance):
        self.values = values
        self.grid_meta_data = grid_meta_data
        self.info = {'separation_distance': separation_distance}


class TtrData(object):
    """Payload of ``data/airtaxi_ttr_function.pkl`` (navigation_graph_safe.py:133-138)."""

    def __init__(self, values, grid_meta_data, ttr_max):
        self.values = values
        self.grid_meta_data = grid_meta_data
        self.ttr_max = ttr_max


def get_hj_grid_from_meta_data(meta):
    return Grid(meta.lo, meta.hi, meta.shape, meta.periodic_dims)


class ControlAndDisturbanceAffineDynamics(object):
    """Restated hj_reachability ``ControlAndDisturbanceAffineDynamics``."""

    def __init__(self, control_mode, disturbance_mode, control_space, disturbance_space):
        self.control_mode = control_mode
        self.disturbance_mode = disturbance_mode
        self.control_space = control_space
        self.disturbance_space = disturbance_space

    def __call__(self, state, control, disturbance, time):
        return (self.open_loop_dynamics(state, time)
                + self.control_jacobian(state, time) @ control
                + self.disturbance_jacobian(state, time) @ disturbance)

    def optimal_control_and_disturbance(self, state, time, grad_value):
        control_direction = grad_value @ self.control_jacobian(state, time)
        if self.control_mode == "min":
            control_direction = -control_direction
        disturbance_direction = grad_value @ self.disturbance_jacobian(state, time)
        if self.disturbance_mode == "min":
            disturbance_direction = -disturbance_direction
        return (self.control_space.extreme_point(control_direction),
                self.disturbance_space.extreme_point(disturbance_direction))

    def optimal_control(self, state, time, grad_value):
        return self.optimal_control_and_disturbance(state, time, grad_value)[0]
