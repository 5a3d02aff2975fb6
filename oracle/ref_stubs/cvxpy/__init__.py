"""cvxpy 1.4.1 stub (test infrastructure): affine expressions + closed-form QP.

The reference solves, per active agent, the single-constraint CBF-QP
``min (u-u_ref)^T W (u-u_ref)  s.t.  g^T (f(x) + G u) + gamma V >= 0``
(``multiagent/safety_filter.py:286-308,364-376``) with cvxpy's default solver.
This stub returns the exact KKT solution instead (parity against OSQP is
unpinned):

  s = a.u_ref + b  with  a = coefficient row of u, b = constant term
  s >= 0            -> u = u_ref
  a == 0 and s < 0  -> infeasible -> ``u.value = None``
  otherwise         -> u = u_ref - s / (a^T W^-1 a) * W^-1 a

All arithmetic is float64, dot products summed left to right.
"""
import numpy as _np


def _seqdot(a, b):
    acc = 0.0
    for x, y in zip(a, b):
        acc = acc + float(x) * float(y)
    return acc


class Expression(object):
    """Affine map ``A u + c`` of the single problem variable (A: m x n, c: m)."""
    __array_ufunc__ = None

    def __init__(self, A, c):
        self.A = _np.asarray(A, dtype=_np.float64)
        self.c = _np.asarray(c, dtype=_np.float64)

    # arithmetic ------------------------------------------------------------
    def __add__(self, other):
        if isinstance(other, Expression):
            return Expression(self.A + other.A, self.c + other.c)
        return Expression(self.A, self.c + _np.asarray(other, dtype=_np.float64))

    __radd__ = __add__

    def __sub__(self, other):
        if isinstance(other, Expression):
            return Expression(self.A - other.A, self.c - other.c)
        return Expression(self.A, self.c - _np.asarray(other, dtype=_np.float64))

    def __rsub__(self, other):
        return Expression(-self.A, _np.asarray(other, dtype=_np.float64) - self.c)

    def __rmatmul__(self, M):
        M = _np.asarray(M, dtype=_np.float64)
        if M.ndim == 1:
            row = _np.array([_seqdot(M, self.A[:, k]) for k in range(self.A.shape[1])])
            return Expression(row[None, :], _np.array([_seqdot(M, self.c)]))
        A = _np.array([[_seqdot(M[i], self.A[:, k]) for k in range(self.A.shape[1])]
                       for i in range(M.shape[0])])
        c = _np.array([_seqdot(M[i], self.c) for i in range(M.shape[0])])
        return Expression(A, c)

    def __rmul__(self, s):
        s = float(s)
        return Expression(s * self.A, s * self.c)

    __mul__ = __rmul__

    def __ge__(self, other):
        return Constraint(self - other)


class Variable(Expression):
    def __init__(self, n):
        super().__init__(_np.eye(n), _np.zeros(n))
        self.n = n
        self.value = None


class Constraint(object):
    def __init__(self, expr):
        self.expr = expr  # expr >= 0


class QuadForm(object):
    def __init__(self, expr, P):
        self.expr = expr
        self.P = _np.asarray(P, dtype=_np.float64)


def quad_form(expr, P):
    return QuadForm(expr, P)


class Minimize(object):
    def __init__(self, obj):
        self.obj = obj


class Problem(object):
    def __init__(self, objective, constraints):
        self.objective = objective
        self.constraints = constraints

    def solve(self, *args, **kwargs):
        q = self.objective.obj
        expr = q.expr                       # u - u_ref  (A = I, c = -u_ref)
        u_ref = -expr.c
        w = _np.diag(q.P).astype(_np.float64)
        con = self.constraints[0].expr      # a u + b >= 0
        a = con.A[0]
        b = float(con.c[0])
        var = _VARS[-1]
        s = _seqdot(a, u_ref) + b
        if s >= 0.0:
            var.value = u_ref.copy()
            return 0.0
        den = 0.0
        for k in range(len(a)):
            den = den + float(a[k]) * float(a[k]) / w[k]
        if den == 0.0:
            var.value = None
            return float('inf')
        lam = s / den
        u = _np.array([u_ref[k] - lam * (float(a[k]) / w[k]) for k in range(len(a))])
        var.value = u
        return 0.0


_VARS = []
_Variable = Variable


def Variable(n):  # noqa: F811 -- track the most recent variable for Problem.solve
    v = _Variable(n)
    _VARS.append(v)
    if len(_VARS) > 4:
        del _VARS[0]
    return v
