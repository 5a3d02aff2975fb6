// rk45_latency.hip -- DIAGNOSTIC micro-benchmark (never part of the product library): the
// latency of one wave running the double integrator's RK45 restatement (lsm_rk45.h) on 32
// lanes, as the team kernel's agent wave does in its phase B, with per-operation dependent-chain
// latencies beside it (glibc_pow, FP64 div / sqrt / fma, four independent divisions), to see
// where that phase's ~8.5k cycles (stamps) go. One wave per CU (256 workgroups of 64 threads),
// s_memtime around REPS calls per lane.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o rk45_latency rk45_latency.hip
//   ./rk45_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../csrc/lsm_rk45.h"

using namespace lsm;

template <int V>
__global__ __launch_bounds__(64) void bench(const double* y0, const double* acc, double* out, unsigned long long* cyc,
                                            int reps) {
  const int lane = threadIdx.x;
  const int g = blockIdx.x * 64 + lane;
  double y[4] = {y0[4 * g], y0[4 * g + 1], y0[4 * g + 2], y0[4 * g + 3]};
  const double a0 = acc[2 * g], a1 = acc[2 * g + 1];
  double s = 0.0, x = 1.0 + fabs(y[0]), q[4] = {x, x + 1, x + 2, x + 3};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if (lane < 32) {
      if (V == 0) {
        double yy[4] = {y[0] + s * 1e-300, y[1], y[2], y[3]};
        rk45_di(yy, a0, a1, 0.1);
        s += yy[0] + yy[1] + yy[2] + yy[3];
      } else if (V == 1) {
        x = glibc_pow(x, -0.2) + 0.5;
      } else if (V == 2) {
        x = 3.0 / x + 0.25;
      } else if (V == 3) {
        x = sqrt(x) + 1.0;
      } else if (V == 4) {
        x = fma(x, 0.999, 1e-3);
      } else {
        for (int k = 0; k < 4; ++k) q[k] = 3.0 / q[k] + 0.25;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[g] = s + x + q[0] + q[1] + q[2] + q[3];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int blocks = 256, n = blocks * 64, reps = 64;
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> up(-3.2, 3.2);
  std::uniform_int_distribution<int> uv(-20, 20), ua(0, 4);
  std::vector<double> y(4 * n), a(2 * n);
  for (int i = 0; i < n; ++i) {
    y[4 * i] = up(rng); y[4 * i + 1] = up(rng);
    y[4 * i + 2] = 0.025 * uv(rng); y[4 * i + 3] = 0.025 * uv(rng);
    a[2 * i] = -0.5 + 0.25 * ua(rng); a[2 * i + 1] = -0.5 + 0.25 * ua(rng);
  }
  double *dy = nullptr, *da = nullptr, *dout = nullptr;
  unsigned long long* dc = nullptr;
  if (hipMalloc(&dy, 8 * y.size()) || hipMalloc(&da, 8 * a.size()) || hipMalloc(&dout, 8 * n) ||
      hipMalloc(&dc, 8 * blocks))
    return 1;
  if (hipMemcpy(dy, y.data(), 8 * y.size(), hipMemcpyHostToDevice) ||
      hipMemcpy(da, a.data(), 8 * a.size(), hipMemcpyHostToDevice))
    return 1;
  std::vector<unsigned long long> c(blocks);
  auto run = [&](auto kern, const char* name) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, dy, da, dout, dc, reps);
    if (hipDeviceSynchronize() || hipMemcpy(c.data(), dc, 8 * blocks, hipMemcpyDeviceToHost)) {
      printf("%s failed\n", name);
      return;
    }
    std::vector<unsigned long long> s(c);
    std::sort(s.begin(), s.end());
    printf("%-28s median %8.1f cycles per call (p10 %.1f, p90 %.1f)\n", name, s[blocks / 2] / (double)reps,
           s[blocks / 10] / (double)reps, s[9 * blocks / 10] / (double)reps);
  };
  run(bench<0>, "rk45_di exact");
  run(bench<1>, "glibc_pow (dependent)");
  run(bench<2>, "FP64 div (dependent)");
  run(bench<3>, "FP64 sqrt (dependent)");
  run(bench<4>, "FP64 fma (dependent)");
  run(bench<5>, "4 independent FP64 divs");
  return 0;
}
