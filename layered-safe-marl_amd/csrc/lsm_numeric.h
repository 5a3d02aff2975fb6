// lsm_numeric.h -- numpy-compatible float64 primitives used by both the HIP kernels and
// the host-side test entry points.
//
// The reference's arithmetic is numpy on x86-64 (OpenBLAS). To reproduce its
// decisions (goal reached / done / edge thresholds) the build compiles with
// -ffp-contract=off and re-creates, operation by operation, the few places where
// numpy does NOT evaluate a plain left-to-right expression (measured in the build
// container, see DESIGN.md "Numerics"):
//   * np.linalg.norm(v) of a 1-D vector  = sqrt(ddot): acc = v0*v0; acc = fma(vk, vk, acc)
//   * np.dot(2x2 rotation, v)            = out_r = fma(M[r][0], v0, M[r][1]*v1)
//   * np.add.reduce / np.mean / np.std   = numpy pairwise summation (8 partial sums)
//   * np.clip / np.maximum               = compare-select, NaN-free here
//   * Python min()/max()                 = "b < a ? b : a" / "b > a ? b : a"
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define LSM_HD __host__ __device__ __forceinline__

namespace lsm {

LSM_HD double np_clip(double x, double lo, double hi) {
  double t = (x > lo) ? x : lo;
  return (t < hi) ? t : hi;
}
LSM_HD double np_maximum(double a, double b) { return (a >= b) ? a : b; }
LSM_HD double py_min(double a, double b) { return (b < a) ? b : a; }
LSM_HD double py_max(double a, double b) { return (b > a) ? b : a; }

// np.linalg.norm of a 1-D float64 vector (BLAS ddot with FMA accumulation).
LSM_HD double blas_norm2(double x, double y) { return sqrt(fma(y, y, x * x)); }
LSM_HD double blas_norm3(double x, double y, double z) { return sqrt(fma(z, z, fma(y, y, x * x))); }
LSM_HD double blas_norm4(double a, double b, double c, double d) {
  return sqrt(fma(d, d, fma(c, c, fma(b, b, a * a))));
}
// np.sqrt(np.sum(np.square(d))) for a 2-vector, and np.linalg.norm(..., axis=k) (no BLAS).
LSM_HD double plain_norm2(double x, double y) { return sqrt(x * x + y * y); }

// np.dot(rot, v) with rot = [[c, s], [-s, c]] (get_relative_position_from_reference).
LSM_HD void blas_rot(double c, double s, double vx, double vy, double& ox, double& oy) {
  ox = fma(c, vx, s * vy);
  oy = fma(-s, vx, c * vy);
}

// numpy pairwise summation (pairwise_sum_DOUBLE), n <= 128 (the path never sums more),
// over an accessor so device code needs no private arrays.
template <class A>
LSM_HD double np_sum_acc(const A& a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += a(i);
    return res;
  }
  double r0 = a(0), r1 = a(1), r2 = a(2), r3 = a(3), r4 = a(4), r5 = a(5), r6 = a(6), r7 = a(7);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += a(i); r1 += a(i + 1); r2 += a(i + 2); r3 += a(i + 3);
    r4 += a(i + 4); r5 += a(i + 5); r6 += a(i + 6); r7 += a(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a(i);
  return res;
}
// np_sum_acc over a plain array with the 8-way loop kept rolled (large n, rare path)
LSM_HD double np_sum_rolled(const double* a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int i = 8;
#pragma unroll 1
  for (; i < n - (n % 8); i += 8) {
    r0 += a[i]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
    r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
#pragma unroll 1
  for (; i < n; ++i) res += a[i];
  return res;
}
LSM_HD double np_mean_rolled(const double* a, int n) { return np_sum_rolled(a, n) / (double)n; }
struct ArrAcc {
  const double* p;
  LSM_HD double operator()(int i) const { return p[i]; }
};
LSM_HD double np_sum(const double* a, int n) { return np_sum_acc(ArrAcc{a}, n); }
LSM_HD double np_mean(const double* a, int n) { return np_sum(a, n) / (double)n; }
template <class A>
struct SqDevAcc {
  A a;
  double m;
  LSM_HD double operator()(int i) const {
    const double d = a(i) - m;
    return d * d;
  }
};
// np.mean / np.std of an accessor-defined array (np.std: sqrt(mean(|x - mean|^2)))
template <class A>
LSM_HD void np_mean_std(const A& a, int n, double& mean, double& std) {
  mean = np_sum_acc(a, n) / (double)n;
  std = sqrt(np_sum_acc(SqDevAcc<A>{a, mean}, n) / (double)n);
}

// direction_alignment_error (custom_scenarios/utils.py:79-81).
LSM_HD double dae(double h, double ref) { return 0.5 - 0.5 * cos(h - ref); }

// ---- MT19937 exactly as numpy's legacy RandomState (mt19937.c / legacy distributions) ----
constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr uint32_t MT_MATRIX_A = 0x9908b0dfu;
constexpr uint32_t MT_UPPER = 0x80000000u;
constexpr uint32_t MT_LOWER = 0x7fffffffu;

LSM_HD uint32_t mt_twist1(uint32_t ki, uint32_t ki1, uint32_t km) {
  uint32_t y = (ki & MT_UPPER) | (ki1 & MT_LOWER);
  return km ^ (y >> 1) ^ ((0u - (y & 1u)) & MT_MATRIX_A);
}
LSM_HD uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
// np.random.seed(int): mt19937_seed -> init_genrand
LSM_HD void mt_seed(uint32_t seed, uint32_t* key, int stride) {
  for (int pos = 0; pos < MT_N; ++pos) {
    key[pos * stride] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)pos + 1u;
  }
}

// Host RNG (sequential twist); the device uses the wave-cooperative twist in the kernel.
struct HostMT {
  uint32_t key[MT_N];
  int pos;
  void seed(uint32_t s) { mt_seed(s, key, 1); pos = MT_N; }
  void gen() {
    int i = 0;
    for (; i < MT_N - MT_M; ++i) key[i] = mt_twist1(key[i], key[i + 1], key[i + MT_M]);
    for (; i < MT_N - 1; ++i) key[i] = mt_twist1(key[i], key[i + 1], key[i + (MT_M - MT_N)]);
    key[MT_N - 1] = mt_twist1(key[MT_N - 1], key[0], key[MT_M - 1]);
    pos = 0;
  }
  uint32_t next32() {
    if (pos >= MT_N) gen();
    return mt_temper(key[pos++]);
  }
  double next_double() {
    uint32_t a = next32() >> 5, b = next32() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  // RandomState.uniform(low, high): low + (high - low) * next_double()
  double uniform(double lo, double hi) {
    double range = hi - lo;
    return lo + range * next_double();
  }
};

}  // namespace lsm
