/* rk45_ref.c -- TEST INFRASTRUCTURE (oracle). C restatement of the reference's double-integrator
 * integration: DoubleIntegratorXYState.update_state (multiagent/core.py:199-210) calls
 *     solve_ivp(ode, [0, dt], y0, method='RK45').y[:, -1]
 * with ode(t, y) = [y2, y3, a0, a1] (core.py:187-193). This file follows scipy 1.15.3
 * (scipy/integrate/_ivp/ivp.py solve_ivp, rk.py RungeKutta._step_impl / rk_step / RK45,
 * common.py select_initial_step / norm) step by step, with numpy's arithmetic as it runs in the
 * build image:
 *   - np.dot(K[:s].T, w) is OpenBLAS 0.3.29 dgemv_n (SkylakeX kernels): column groups of 4, then 2,
 *     then 1; within a group of 4: t = fma(k0,w0,k1*w1), t = fma(k2,w2,t), t = fma(k3,w3,t);
 *     group of 2: fma(k0,w0,k1*w1); group of 1: k0*w0; each group's sum added to the result
 *     (identified with crafted inputs, tests/test_rk45.py pins it);
 *   - np.linalg.norm(x) = sqrt(ddot(x, x)), ddot an fma chain from x0*x0;
 *   - numpy scalar ** = libm pow (called directly here).
 * Pinned bit-exactly against scipy by tests/test_rk45.py; used by oracle/lsm_oracle.py's
 * integrator="restated". */
#include <math.h>
#include <string.h>

static const double RK_A[6][5] = {
    {0, 0, 0, 0, 0},
    {1.0 / 5, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
static const double RK_B[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
static const double RK_E[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525,
                               1.0 / 40};
static const double RK_C[6] = {0, 1.0 / 5, 3.0 / 10, 4.0 / 5, 8.0 / 9, 1};

/* out = np.dot(M.T, w) for M = K[:n] (n rows of 4): OpenBLAS dgemv_n column groups */
static void dot_kt(double K[][4], const double* w, int n, double* out) {
  for (int r = 0; r < 4; ++r) {
    double acc = 0.0;
    int j = 0;
    while (n - j >= 4) {
      double t = fma(K[j][r], w[j], K[j + 1][r] * w[j + 1]);
      t = fma(K[j + 2][r], w[j + 2], t);
      t = fma(K[j + 3][r], w[j + 3], t);
      acc = acc + t;
      j += 4;
    }
    if (n - j >= 2) {
      acc = acc + fma(K[j][r], w[j], K[j + 1][r] * w[j + 1]);
      j += 2;
    }
    if (n - j == 1) acc = acc + K[j][r] * w[j];
    out[r] = acc;
  }
}

/* common.norm: np.linalg.norm(x) / x.size ** 0.5 */
static double rms_norm4(const double* x) {
  double s = x[0] * x[0];
  for (int i = 1; i < 4; ++i) s = fma(x[i], x[i], s);
  return sqrt(s) / 2.0;
}

static void ode(const double* y, double a0, double a1, double* f) {
  f[0] = y[2];
  f[1] = y[3];
  f[2] = a0;
  f[3] = a1;
}

/* y <- solve_ivp(ode, [0, t_bound], y, method='RK45').y[:, -1]; returns the number of accepted
 * steps (negative: the solver stopped with TOO_SMALL_STEP; y is then where it stopped) */
int rk45_di_ref(double* y, double a0, double a1, double t_bound) {
  const double rtol = 1e-3, atol = 1e-6;
  const double SAFETY = 0.9, MIN_FACTOR = 0.2, MAX_FACTOR = 10.0, error_exponent = -1.0 / (4 + 1);
  double f[4], scale[4], tmp[4];
  ode(y, a0, a1, f);
  /* select_initial_step(fun, t0, y0, t_bound, max_step=inf, f0, direction=1, order=4, rtol, atol) */
  double h_abs;
  {
    const double interval_length = fabs(t_bound - 0.0);
    for (int i = 0; i < 4; ++i) scale[i] = atol + fabs(y[i]) * rtol;
    for (int i = 0; i < 4; ++i) tmp[i] = y[i] / scale[i];
    const double d0 = rms_norm4(tmp);
    for (int i = 0; i < 4; ++i) tmp[i] = f[i] / scale[i];
    const double d1 = rms_norm4(tmp);
    double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
    if (interval_length < h0) h0 = interval_length;
    double y1[4], f1[4];
    for (int i = 0; i < 4; ++i) y1[i] = y[i] + h0 * 1.0 * f[i];
    ode(y1, a0, a1, f1);
    for (int i = 0; i < 4; ++i) tmp[i] = (f1[i] - f[i]) / scale[i];
    const double d2 = rms_norm4(tmp) / h0;
    double h1;
    if (d1 <= 1e-15 && d2 <= 1e-15)
      h1 = (1e-6 > h0 * 1e-3) ? 1e-6 : h0 * 1e-3;
    else
      h1 = pow(0.01 / (d2 > d1 ? d2 : d1), 1.0 / (4 + 1));
    h_abs = 100 * h0;                       /* Python min(): first of the smallest */
    if (h1 < h_abs) h_abs = h1;
    if (interval_length < h_abs) h_abs = interval_length;
  }
  double t = 0.0;
  double K[7][4];
  int steps = 0;
  while (!(t == t_bound)) {                 /* OdeSolver.step until status 'finished' */
    const double min_step = 10 * fabs(nextafter(t, INFINITY) - t);
    double h_cur = h_abs;
    if (h_cur < min_step) h_cur = min_step;
    int accepted = 0, rejected = 0;
    double t_new = t, y_new[4], f_new[4], h = 0.0;
    while (!accepted) {
      if (h_cur < min_step) return -steps - 1;
      h = h_cur * 1.0;
      t_new = t + h;
      if (1.0 * (t_new - t_bound) > 0) t_new = t_bound;
      h = t_new - t;
      h_cur = fabs(h);
      /* rk_step */
      memcpy(K[0], f, sizeof f);
      for (int s = 1; s < 6; ++s) {
        double dy[4], ys[4];
        dot_kt(K, RK_A[s], s, dy);
        for (int i = 0; i < 4; ++i) ys[i] = y[i] + dy[i] * h;
        (void)RK_C[s];                      /* fun(t + c * h, .) ignores t */
        ode(ys, a0, a1, K[s]);
      }
      double g[4];
      dot_kt(K, RK_B, 6, g);
      for (int i = 0; i < 4; ++i) y_new[i] = y[i] + h * g[i];
      ode(y_new, a0, a1, f_new);
      memcpy(K[6], f_new, sizeof f_new);
      /* error norm */
      double e[4];
      dot_kt(K, RK_E, 7, e);
      for (int i = 0; i < 4; ++i) {
        const double ay = fabs(y[i]), ayn = fabs(y_new[i]);
        tmp[i] = (e[i] * h) / (atol + (ay >= ayn ? ay : ayn) * rtol);  /* np.maximum */
      }
      const double error_norm = rms_norm4(tmp);
      if (error_norm < 1) {
        double factor;
        if (error_norm == 0) {
          factor = MAX_FACTOR;
        } else {
          const double q = SAFETY * pow(error_norm, error_exponent);
          factor = (q < MAX_FACTOR) ? q : MAX_FACTOR;   /* min(MAX_FACTOR, q) */
        }
        if (rejected && factor > 1) factor = 1;
        h_cur *= factor;
        accepted = 1;
      } else {
        const double q = SAFETY * pow(error_norm, error_exponent);
        h_cur *= (q > MIN_FACTOR) ? q : MIN_FACTOR;
        rejected = 1;
      }
    }
    t = t_new;
    memcpy(y, y_new, sizeof y_new);
    memcpy(f, f_new, sizeof f_new);
    h_abs = h_cur;
    ++steps;
  }
  return steps;
}
