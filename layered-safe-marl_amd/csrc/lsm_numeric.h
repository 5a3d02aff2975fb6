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
  bool exhausted() const { return false; }
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

// ---- Philox4x32-10 (Salmon et al., SC'11): the fast reset stream (LSM_RNG_PHILOX) ----------
// Counter-based: draw block b of reset r of env key k is philox(ctr = (b, r, 0, 0), key = (k, tag)),
// so a reset needs no stored generator state (the device keeps only r). Every lane of an env
// runs the identical scalar sequence, like the MT19937 replay. Doubles take two words the
// numpy way ((a >> 5) 2^26 + (b >> 6)) / 2^53, so uniform(lo, hi) has the same form.
// The Philox4x32 block function, 10 rounds (Random123's philox4x32_R(10, ctr, key)).
LSM_HD void philox4x32_10(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], a = key[0], b = key[1];
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ a, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ b;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    a += 0x9E3779B9u; b += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Philox {
  uint32_t k0, k1, r;   // key, reset index
  uint32_t blk;         // next counter block
  uint32_t buf[4];
  int pos;
  LSM_HD void init(uint32_t key, uint32_t reset_index) {
    k0 = key; k1 = 0x4c534d31u; r = reset_index; blk = 0; pos = 4;
  }
  LSM_HD void round_all() {
    const uint32_t ctr[4] = {blk, r, 0u, 0u}, key[2] = {k0, k1};
    philox4x32_10(ctr, key, buf);
    ++blk;
    pos = 0;
  }
  LSM_HD uint32_t next32() {
    if (pos >= 4) round_all();
    return buf[pos++];
  }
  LSM_HD bool exhausted() const { return false; }
  LSM_HD double next_double() {
    uint32_t a = next32() >> 5, b = next32() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  LSM_HD double uniform(double lo, double hi) {
    double range = hi - lo;
    return lo + range * next_double();
  }
};

}  // namespace lsm
