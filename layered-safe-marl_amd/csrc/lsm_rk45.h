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

// The pow tables' memory: the constant arrays (nullptr), or copies of them (the team kernel stages
// them in LDS for its agent wave: 3 KB of {invc, logc, logctail} rows, 2 KB of exp pairs).
struct PowTabs {
  const double* log = nullptr;     // [128][3]
  const uint64_t* exp = nullptr;   // [256]
};

// glibc log_inline (e_pow.c): log(x) as hi + tail, x positive normal.
LSM_RK_HD double glibc_log_inline(uint64_t ix, double* tail, PowTabs tb = PowTabs()) {
  const uint64_t OFF = 0x3fe6955500000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> (52 - 7)) % 128);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = as_f64(iz);
  const double kd = (double)k;
  const double* e = tb.log ? tb.log + 3 * i : powl_tab(i);
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
LSM_RK_HD double glibc_exp_inline(double x, double xtail, PowTabs tb = PowTabs()) {
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
  const uint64_t* et = tb.exp ? tb.exp : expd_tab_ptr();
  const double tl = as_f64(et[idx]);
  const uint64_t sbits = et[idx + 1] + top;
  const double r2 = r * r;
  const double* C = EXPD_POLY;
  const double tmp = fma(r2 * r2, fma(r, C[3], C[2]), fma(r2, fma(r, C[1], C[0]), tl + r));
  const double scale = as_f64(sbits);
  return fma(scale, tmp, scale);
}

// glibc pow(x, y) for positive normal x and a finite non-integer y of moderate size
// (the step-size rules: y = +-0.2).
LSM_RK_HD double glibc_pow(double x, double y, PowTabs tb = PowTabs()) {
  double lo;
  const double hi = glibc_log_inline(as_u64(x), &lo, tb);
  const double ehi = y * hi;
  const double elo = fma(y, lo, fma(y, hi, -ehi));
  return glibc_exp_inline(ehi, elo, tb);
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

// One velocity component's np.dot(K[:s].T, w) when every stage row holds the same value a
// (the accelerations: K[j][2] = a0, K[j][3] = a1 for all j): OpenBLAS dgemv_n column groups.
LSM_RK_HD double rk_gemv_const(double a, const double* w, int s) {
  double y = 0.0;
  int j = 0;
  for (; j + 4 <= s; j += 4) {
    double t = fma(a, w[j], a * w[j + 1]);
    t = fma(a, w[j + 2], t);
    t = fma(a, w[j + 3], t);
    y = y + t;
  }
  if ((s - j) & 2) {
    y = y + fma(a, w[j], a * w[j + 1]);
    j += 2;
  }
  if ((s - j) & 1) y = y + a * w[j];
  return y;
}

// One position component's np.dot(K[:s].T, w): K[j] = the stage velocities k[j].
LSM_RK_HD double rk_gemv_col(const double* k, const double* w, int s) {
  double y = 0.0;
  int j = 0;
  for (; j + 4 <= s; j += 4) {
    double t = fma(k[j], w[j], k[j + 1] * w[j + 1]);
    t = fma(k[j + 2], w[j + 2], t);
    t = fma(k[j + 3], w[j + 3], t);
    y = y + t;
  }
  if ((s - j) & 2) {
    y = y + fma(k[j], w[j], k[j + 1] * w[j + 1]);
    j += 2;
  }
  if ((s - j) & 1) y = y + k[j] * w[j];
  return y;
}

// solve_ivp(x' = v, v' = a, [0, tb], y, method='RK45').y[:, -1] (rtol 1e-3, atol 1e-6, no
// max_step), y updated in place, returns the number of steps. Same operations and roundings as
// scipy's generic code (dgemv over the K rows), specialised to this ODE:
//   * the right-hand side ignores positions, so the stage positions y + dy (dy[0], dy[1]) feed
//     nothing and are not formed;
//   * K[j][2..3] = a for every stage, so the velocity-component dot products depend on a only and
//     are computed once per call instead of once per step;
//   * the error factor min(10, 0.9 err^-1/5) is 10 without evaluating pow when err <= 1e-6
//     (0.9 * (1e-6)^-0.2 = 14.2 > 10); err == 0 gives 10 as in scipy; after the step that
//     reaches tb it is not evaluated at all (scipy computes the next step size, nothing reads it).
// A rejected step (err >= 1) follows _step_impl: h *= max(0.2, 0.9 err^-1/5), factor <= 1 after.
LSM_RK_HD int rk45_di(double* y, double a0, double a1, double tb) {
  const double rtol = 1e-3, atol = 1e-6;
  // At rest with no acceleration (+0.0 velocities and accelerations, no -0.0 position) every stage
  // is +-0 and every step leaves y as it is: skip the ~6 steps select_initial_step's 1e-6 start
  // takes to reach tb (the step count is not part of the result).
  if (as_u64(y[2]) == 0 && as_u64(y[3]) == 0 && as_u64(a0) == 0 && as_u64(a1) == 0 &&
      as_u64(y[0]) != 0x8000000000000000ull && as_u64(y[1]) != 0x8000000000000000ull)
    return 0;
  const Rk45Tab& T = rk45_tab();
  // velocity-component stage increments, final combination and error dot products
  double dv0[6], dv1[6];
#pragma unroll
  for (int s = 1; s < 6; ++s) {
    dv0[s] = rk_gemv_const(a0, T.A[s], s);
    dv1[s] = rk_gemv_const(a1, T.A[s], s);
  }
  const double gb0 = rk_gemv_const(a0, T.B, 6), gb1 = rk_gemv_const(a1, T.B, 6);
  const double ge0 = rk_gemv_const(a0, T.E, 7), ge1 = rk_gemv_const(a1, T.E, 7);
  // select_initial_step
  const double sc0 = atol + fabs(y[0]) * rtol, sc1 = atol + fabs(y[1]) * rtol;
  const double sc2 = atol + fabs(y[2]) * rtol, sc3 = atol + fabs(y[3]) * rtol;
  double t4[4] = {y[0] / sc0, y[1] / sc1, y[2] / sc2, y[3] / sc3};
  const double d0 = rk_norm4(t4);
  t4[0] = y[2] / sc0; t4[1] = y[3] / sc1; t4[2] = a0 / sc2; t4[3] = a1 / sc3;
  const double d1 = rk_norm4(t4);
  double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
  h0 = (tb < h0) ? tb : h0;
  // f1 - f0 = [(v + h0 a) - v, 0, 0] per axis (f1 of y0 + h0 f0)
  t4[0] = ((y[2] + h0 * a0) - y[2]) / sc0;
  t4[1] = ((y[3] + h0 * a1) - y[3]) / sc1;
  t4[2] = (a0 - a0) / sc2;
  t4[3] = (a1 - a1) / sc3;
  const double d2 = rk_norm4(t4) / h0;
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
  int n = 0;
  double v0 = y[2], v1 = y[3];       // K[0][0..1] = f[0..1] = the step's starting velocity
  while (t < tb) {
    bool rejected = false;
    for (;;) {
      double t_new = t + h_abs;
      if (t_new - tb > 0) t_new = tb;
      const double h = t_new - t;
      h_abs = fabs(h);
      double k0[7], k1[7];           // stage velocities (the position components of K)
      k0[0] = v0; k1[0] = v1;
#pragma unroll
      for (int s = 1; s < 6; ++s) {
        k0[s] = y[2] + dv0[s] * h;
        k1[s] = y[3] + dv1[s] * h;
      }
      const double yn0 = y[0] + h * rk_gemv_col(k0, T.B, 6);
      const double yn1 = y[1] + h * rk_gemv_col(k1, T.B, 6);
      const double yn2 = y[2] + h * gb0;
      const double yn3 = y[3] + h * gb1;
      k0[6] = yn2; k1[6] = yn3;
      const double e0 = rk_gemv_col(k0, T.E, 7), e1 = rk_gemv_col(k1, T.E, 7);
      const double yy[4] = {y[0], y[1], y[2], y[3]}, yn[4] = {yn0, yn1, yn2, yn3}, ee[4] = {e0, e1, ge0, ge1};
      // The error terms are rounding noise for this ODE (its stages are exact up to rounding): with
      // |e h| <= 1e-13 on all four components each scaled term is <= 1e-7 (denominators >= atol =
      // 1e-6), so the norm is < 1e-6 and the step is accepted with factor 10 (no pow) -- the branch
      // the full computation takes. NaN fails the test and takes the full computation.
      bool small = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) small = small && fabs(ee[i] * h) <= 1e-13;
      double en = 0.0;
      if (!small) {
        double r4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double ay = fabs(yy[i]), ayn = fabs(yn[i]);
          r4[i] = (ee[i] * h) / (atol + ((ay >= ayn) ? ay : ayn) * rtol);
        }
        en = rk_norm4(r4);
      }
      if (en < 1) {
        if (t_new < tb) {            // the step size after the last step is never used
          double fac = 10.0;         // MAX_FACTOR
          if (en > 1e-6) {
            const double q = 0.9 * glibc_pow(en, -1.0 / 5.0);
            if (q < fac) fac = q;
          }
          if (rejected && fac > 1) fac = 1;
          h_abs *= fac;
        }
        t = t_new;
        y[0] = yn0; y[1] = yn1; y[2] = yn2; y[3] = yn3;
        v0 = yn2; v1 = yn3;
        ++n;
        break;
      }
      const double q = 0.9 * glibc_pow(en, -1.0 / 5.0);
      h_abs *= (q > 0.2) ? q : 0.2;
      rejected = true;
    }
  }
  return n;
}

}  // namespace lsm
