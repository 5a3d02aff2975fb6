// lsm_rk45.h -- the reference's double-integrator integration, operation for operation.
//
// DoubleIntegratorXYState.update_state (multiagent/core.py:199-210) calls
// scipy.integrate.solve_ivp(ode, [0, dt], y0, method='RK45') on x' = v, v' = a. The exact
// solution is p + v dt + a dt^2 / 2, but the reference's rounding is RK45's: an initial step from
// select_initial_step (scipy/integrate/_ivp/common.py), 1-3 Dormand-Prince steps whose stage sums
// are numpy dot products (OpenBLAS dgemv), and numpy's scalar `**` (glibc pow) in the step-size
// rules. Velocities are multiples of 0.025 when unfiltered, so relative velocities hit the filter's
// clip thresholds (+-0.45, safety_filter.py:328-340) exactly, and the decision there depends on
// the last bit: the closed form and RK45 differ in ~1/3 of the cases. This header restates
// scipy 1.15's RK45 for this ODE with:
//   * np.dot(K[:s].T, w) as OpenBLAS 0.3.29 dgemv_n (SkylakeX kernels, measured in the build
//     container): columns in groups of 4 (t = fma(k0, w0, k1 w1); t = fma(k2, w2, t);
//     t = fma(k3, w3, t)), then a group of 2 (fma(k0, w0, k1 w1)), then 1 (k0 w0), each group
//     sum added to the running result;
//   * np.linalg.norm of a 4-vector as ddot (fma chain) and sqrt;
//   * glibc 2.35's pow (sysdeps/ieee754/dbl-64/e_pow.c, FMA variant), with its data tables
//     (lsm_pow_tables.h, extracted from the image's libm by tools/gen_pow_tables.py): glibc's pow
//     is not correctly rounded, so its own algorithm is needed for the exact bits.
// tests/test_rk45.py checks the host build of this code against scipy and glibc bit-exactly.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "lsm_pow_tables.h"

#define LSM_RK_HD __host__ __device__ __forceinline__

namespace lsm {

LSM_RK_HD uint64_t as_u64(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
LSM_RK_HD double as_f64(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

// glibc log_inline (e_pow.c): log(x) as hi + tail, x positive normal.
LSM_RK_HD double glibc_log_inline(uint64_t ix, double* tail) {
  const uint64_t OFF = 0x3fe6955500000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> (52 - 7)) % 128);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = as_f64(iz);
  const double kd = (double)k;
  const double* e = powl_tab(i);
  const double invc = e[0], logc = e[1], logctail = e[2];
  const double r = fma(z, invc, -1.0);
  const double t1 = fma(kd, POWL_LN2HI, logc);
  const double t2 = t1 + r;
  const double lo1 = fma(kd, POWL_LN2LO, logctail);
  const double lo2 = t1 - t2 + r;
  const double* A = POWL_POLY;
  const double ar = A[0] * r;
  const double ar2 = r * ar;
  const double ar3 = r * ar2;
  const double hi = t2 + ar2;
  const double lo3 = fma(ar, r, -ar2);
  const double lo4 = t2 - hi + ar2;
  const double p = ar3 * fma(ar2, fma(ar2, fma(r, A[6], A[5]), fma(r, A[4], A[3])), fma(r, A[2], A[1]));
  const double lo = lo1 + lo2 + lo3 + lo4 + p;
  const double y = hi + lo;
  *tail = hi - y + lo;
  return y;
}

// glibc exp_inline (e_exp.c) for 2^-54 <= |x| < 512 (the range pow(x, +-0.2) reaches here);
// tiny |x| returns 1 + x as glibc does.
LSM_RK_HD double glibc_exp_inline(double x, double xtail) {
  const uint32_t abstop = (uint32_t)(as_u64(x) >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {   // top12(0x1p-54) = 0x3c9, top12(512) = 0x408
    if ((int)abstop - 0x3c9 < 0) return 1.0 + x;
    return x < 0 ? 0.0 : INFINITY;            // not reached by the step-size rules
  }
  double kd = fma(EXPD_INVLN2N, x, EXPD_SHIFT);
  const uint64_t ki = as_u64(kd);
  kd -= EXPD_SHIFT;
  double r = fma(kd, EXPD_NEGLN2LON, fma(kd, EXPD_NEGLN2HIN, x));
  r += xtail;
  const int idx = 2 * (int)(ki % 128);
  const uint64_t top = ki << (52 - 7);
  const double tl = as_f64(expd_tab(idx));
  const uint64_t sbits = expd_tab(idx + 1) + top;
  const double r2 = r * r;
  const double* C = EXPD_POLY;
  const double tmp = fma(r2 * r2, fma(r, C[3], C[2]), fma(r2, fma(r, C[1], C[0]), tl + r));
  const double scale = as_f64(sbits);
  return fma(scale, tmp, scale);
}

// glibc pow(x, y) for positive normal x and a finite non-integer y of moderate size
// (the step-size rules: y = +-0.2).
LSM_RK_HD double glibc_pow(double x, double y) {
  double lo;
  const double hi = glibc_log_inline(as_u64(x), &lo);
  const double ehi = y * hi;
  const double elo = fma(y, lo, fma(y, hi, -ehi));
  return glibc_exp_inline(ehi, elo);
}

// np.dot(K[:s].T, w) for K rows of 4 (OpenBLAS dgemv_n column groups, see above)
LSM_RK_HD void rk_gemv(const double (*K)[4], const double* w, int s, double* out) {
  for (int r = 0; r < 4; ++r) {
    double y = 0.0;
    int j = 0;
    for (; j + 4 <= s; j += 4) {
      double t = fma(K[j][r], w[j], K[j + 1][r] * w[j + 1]);
      t = fma(K[j + 2][r], w[j + 2], t);
      t = fma(K[j + 3][r], w[j + 3], t);
      y = y + t;
    }
    if ((s - j) & 2) {
      y = y + fma(K[j][r], w[j], K[j + 1][r] * w[j + 1]);
      j += 2;
    }
    if ((s - j) & 1) y = y + K[j][r] * w[j];
    out[r] = y;
  }
}

// scipy common.norm: np.linalg.norm(x) / sqrt(x.size) for a 4-vector (ddot fma chain)
LSM_RK_HD double rk_norm4(const double* x) {
  double s = x[0] * x[0];
  s = fma(x[1], x[1], s);
  s = fma(x[2], x[2], s);
  s = fma(x[3], x[3], s);
  return sqrt(s) / 2.0;
}

// Dormand-Prince 5(4) tableau (scipy RK45.A / B / C / E), as float64 literals of the same fractions
struct Rk45Tab {
  double A[6][5], B[6], E[7];
};
LSM_RK_HD const Rk45Tab& rk45_tab() {
  static constexpr Rk45Tab T = {
      {{0, 0, 0, 0, 0},
       {1.0 / 5, 0, 0, 0, 0},
       {3.0 / 40, 9.0 / 40, 0, 0, 0},
       {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
       {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
       {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}},
      {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84},
      {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525, 1.0 / 40}};
  return T;
}

// solve_ivp(x' = v, v' = a, [0, tb], y, method='RK45').y[:, -1] (rtol 1e-3, atol 1e-6, no
// max_step). Returns the number of steps; y is updated in place. A rejected step (error norm
// >= 1, which this polynomial ODE does not produce) returns -1 with y unchanged.
LSM_RK_HD int rk45_di(double* y, double a0, double a1, double tb) {
  const double rtol = 1e-3, atol = 1e-6;
  const Rk45Tab& T = rk45_tab();
  double f[4] = {y[2], y[3], a0, a1};
  double sc[4], tmp[4];
  // select_initial_step
  for (int i = 0; i < 4; ++i) sc[i] = atol + fabs(y[i]) * rtol;
  for (int i = 0; i < 4; ++i) tmp[i] = y[i] / sc[i];
  const double d0 = rk_norm4(tmp);
  for (int i = 0; i < 4; ++i) tmp[i] = f[i] / sc[i];
  const double d1 = rk_norm4(tmp);
  double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
  h0 = (tb < h0) ? tb : h0;
  const double f1[4] = {y[2] + h0 * f[2], y[3] + h0 * f[3], a0, a1};
  for (int i = 0; i < 4; ++i) tmp[i] = (f1[i] - f[i]) / sc[i];
  const double d2 = rk_norm4(tmp) / h0;
  double h1;
  if (d1 <= 1e-15 && d2 <= 1e-15) {
    h1 = (h0 * 1e-3 > 1e-6) ? h0 * 1e-3 : 1e-6;
  } else {
    h1 = glibc_pow(0.01 / ((d2 > d1) ? d2 : d1), 1.0 / 5.0);
  }
  double h_abs = 100 * h0;           // min(100 h0, h1, interval_length, max_step = inf)
  if (h1 < h_abs) h_abs = h1;
  if (tb < h_abs) h_abs = tb;
  double t = 0.0;
  double K[7][4];
  int n = 0;
  while (t < tb) {
    double t_new = t + h_abs;
    if (t_new - tb > 0) t_new = tb;
    const double h = t_new - t;
    h_abs = fabs(h);
    for (int i = 0; i < 4; ++i) K[0][i] = f[i];
    for (int s = 1; s < 6; ++s) {
      double dy[4];
      rk_gemv(K, T.A[s], s, dy);
      K[s][0] = y[2] + dy[2] * h;   // fun(t + c h, y + dy * h) = [vx, vy, a0, a1]
      K[s][1] = y[3] + dy[3] * h;
      K[s][2] = a0;
      K[s][3] = a1;
    }
    double g[4], yn[4];
    rk_gemv(K, T.B, 6, g);
    for (int i = 0; i < 4; ++i) yn[i] = y[i] + h * g[i];
    K[6][0] = yn[2]; K[6][1] = yn[3]; K[6][2] = a0; K[6][3] = a1;
    double e[4];
    rk_gemv(K, T.E, 7, e);
    for (int i = 0; i < 4; ++i) {
      const double ay = fabs(y[i]), ayn = fabs(yn[i]);
      tmp[i] = (e[i] * h) / (atol + ((ay >= ayn) ? ay : ayn) * rtol);
    }
    const double en = rk_norm4(tmp);
    if (!(en < 1)) return -1;
    double fac = 10.0;   // MAX_FACTOR
    if (en != 0) {
      const double q = 0.9 * glibc_pow(en, -1.0 / 5.0);   // SAFETY * error_norm ** error_exponent
      if (q < fac) fac = q;
    }
    h_abs *= fac;
    t = t_new;
    for (int i = 0; i < 4; ++i) { y[i] = yn[i]; f[i] = K[6][i]; }
    ++n;
  }
  return n;
}

}  // namespace lsm
