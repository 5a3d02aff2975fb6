"""The double integrator's integration, bit for bit (CPU tests).

The reference integrates with scipy's ``solve_ivp(..., 'RK45')`` (multiagent/core.py:199-210). Its
last bit decides the safety filter's clip thresholds whenever a relative velocity is exactly
+-0.45 (velocities are multiples of 0.025 between filter interventions), so the kernel replays the
RK45 call itself (csrc/lsm_rk45.h) instead of the closed form. Three links are pinned here:

* oracle/csrc/rk45_ref.c (the oracle's C restatement, libm pow) == scipy solve_ivp;
* the kernel's code built for the host (``lsm_host_rk45_di``) == the oracle restatement;
* the kernel's glibc pow restatement (``lsm_host_glibc_pow``) == libm pow.
"""
import ctypes as C
import math

import numpy as np
import pytest
from scipy.integrate import solve_ivp

from oracle.lsm_oracle import _rk45_ref


def _cases(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        kind = k % 6
        if kind == 0:      # unfiltered: velocities on the 0.025 lattice, discrete accelerations
            v = rng.integers(-20, 21, 2) * 0.025
            a = rng.choice([-0.5, -0.25, 0.0, 0.25, 0.5], 2)
        elif kind == 1:    # filtered (QP) accelerations, clamped speeds
            v = rng.uniform(-0.5, 0.5, 2)
            v = v * min(1.0, 0.5 / max(np.hypot(*v), 1e-300))
            a = rng.uniform(-0.5, 0.5, 2)
        elif kind == 2:    # frozen / resting agents
            v = np.zeros(2)
            a = rng.choice([-0.5, 0.0, 0.5], 2)
        elif kind == 3:    # tiny velocities and accelerations
            v = rng.uniform(-1e-7, 1e-7, 2)
            a = rng.uniform(-1e-6, 1e-6, 2)
        elif kind == 4:    # positions near the origin (scale ~ atol)
            v = rng.integers(-20, 21, 2) * 0.025
            a = rng.choice([-0.5, -0.25, 0.0, 0.25, 0.5], 2)
        else:
            v = rng.uniform(-0.5, 0.5, 2)
            a = rng.choice([-0.5, -0.25, 0.0, 0.25, 0.5], 2)
        p = rng.uniform(-1e-5, 1e-5, 2) if kind == 4 else rng.uniform(-4, 4, 2)
        if kind == 2 and rng.random() < 0.3:
            p = np.zeros(2)
        out.append((np.array([p[0], p[1], v[0], v[1]]), np.asarray(a, dtype=np.float64)))
    # at rest with no acceleration (the kernels skip the integration there), signed zeros included
    for p0 in (0.0, -0.0, 1.5):
        for v0 in (0.0, -0.0):
            for a0 in (0.0, -0.0):
                out.append((np.array([p0, -2.25, v0, 0.0]), np.array([a0, 0.0])))
                out.append((np.array([p0, 0.0, 0.0, v0]), np.array([0.0, a0])))
    return out


def test_oracle_restatement_equals_scipy():
    lib = _rk45_ref()
    for y0, a in _cases(3000, 0):
        ref = solve_ivp(lambda t, y: np.array([y[2], y[3], a[0], a[1]]), [0, 0.1], y0, method="RK45").y[:, -1]
        y = y0.copy()
        lib.rk45_di_ref(y.ctypes.data, float(a[0]), float(a[1]), 0.1)
        np.testing.assert_array_equal(y, ref, err_msg="y0=%r a=%r" % (y0.tolist(), a.tolist()))


def test_kernel_rk45_equals_oracle_restatement():
    from lsm import capi
    lib = capi.load_library()
    ref = _rk45_ref()
    out = np.zeros(4)
    for y0, a in _cases(60000, 1):
        y = y0.copy()
        ref.rk45_di_ref(y.ctypes.data, float(a[0]), float(a[1]), 0.1)
        lib.lsm_host_rk45_di(y0.ctypes.data, float(a[0]), float(a[1]), 0.1, out.ctypes.data)
        np.testing.assert_array_equal(out, y, err_msg="y0=%r a=%r" % (y0.tolist(), a.tolist()))


def test_kernel_pow_equals_glibc():
    from lsm import capi
    lib = capi.load_library()
    rng = np.random.default_rng(2)
    xs = np.exp(rng.uniform(-45.0, 8.0, 100000))
    for k, x in enumerate(xs):
        y = 0.2 if k & 1 else -0.2
        assert lib.lsm_host_glibc_pow(float(x), y) == math.pow(float(x), y), (x, y)
    for x in (1.0, 1.0 + 2 ** -52, 1.0 - 2 ** -53, 1e-300, 1e300, 0.01):
        assert lib.lsm_host_glibc_pow(x, 0.2) == math.pow(x, 0.2), x


def test_closed_form_differs_from_rk45_at_the_last_bit():
    """Why the kernel replays RK45: on the velocity lattice the closed form and RK45 round
    differently often enough to flip exact-threshold decisions (e.g. a relative velocity of
    -0.45 against the clip threshold -0.5 - 0.1 * -0.5)."""
    from oracle.lsm_oracle import closed_form_step
    lib = _rk45_ref()
    diff = 0
    cases = _cases(600, 3)[::6]
    for y0, a in cases:
        y = y0.copy()
        lib.rk45_di_ref(y.ctypes.data, float(a[0]), float(a[1]), 0.1)
        diff += int(not np.array_equal(y, closed_form_step(y0, a, 0.1, True)))
    assert diff > 0
