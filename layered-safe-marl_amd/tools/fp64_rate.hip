// fp64_rate.hip -- DIAGNOSTIC micro-benchmark (never part of the product library): latency and
// throughput of the float64 operations the rollout's per-agent phases are made of, on gfx950.
//   latency:    one wave per SIMD, one dependent chain per lane (cycles per operation)
//   throughput: W waves per SIMD, 8 independent chains per lane (SIMD cycles per wave-instruction
//               of the operation, i.e. per 64 lanes)
// s_memtime around the timed loop of each wave; medians over the waves.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o fp64_rate fp64_rate.hip
//   ./fp64_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

enum { OP_FMA64, OP_FMA32, OP_DIV64, OP_SQRT64, OP_RSQ64, OP_SIN64, OP_COS64, OP_ATAN2_64, OP_LDS64, OP_CVT };

template <int OP>
__device__ __forceinline__ double step(double x, double c, double* lds) {
  if (OP == OP_FMA64) return fma(x, 0.999999, c);
  if (OP == OP_FMA32) return (double)fmaf((float)x, 0.999999f, (float)c);
  if (OP == OP_DIV64) return c / x + 0.5;
  if (OP == OP_SQRT64) return sqrt(x) + c;
  if (OP == OP_RSQ64) return __builtin_amdgcn_rsq(x) + c;
  if (OP == OP_SIN64) return sin(x) + c;
  if (OP == OP_COS64) return cos(x) + c;
  if (OP == OP_ATAN2_64) return atan2(x, c) + 1.5;
  if (OP == OP_LDS64) {
    const int k = ((int)x) & 63;
    return lds[(threadIdx.x + k) & 255] + c;
  }
  return (double)(float)(x - c) + 1.25;   // OP_CVT: f64 sub, round to f32 and back
}

template <int OP, int CH>
__global__ __launch_bounds__(256) void bench(double* out, unsigned long long* cyc, int reps) {
  __shared__ double lds[256];
  lds[threadIdx.x] = 1.0 + threadIdx.x * 1e-3;
  __syncthreads();
  double x[CH];
  const double c = 1.0 + (threadIdx.x & 7) * 1e-3;
#pragma unroll
  for (int k = 0; k < CH; ++k) x[k] = 1.25 + k * 0.01 + threadIdx.x * 1e-5;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int k = 0; k < CH; ++k) x[k] = step<OP>(x[k], c, lds);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  const int reps = 64;
  double* dout = nullptr;
  unsigned long long* dc = nullptr;
  const int maxw = 1024 * 4;
  if (hipMalloc(&dout, 8 * 64 * maxw) || hipMalloc(&dc, 8 * maxw)) return 1;
  std::vector<unsigned long long> c(maxw);
  auto run = [&](auto kern, const char* name, int threads, int chains) {
    // 256 CUs x 4 SIMDs: 1024 workgroups of `threads` -> threads / 64 waves per SIMD
    const int blocks = 1024, nw = blocks * threads / 64;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, dout, dc, reps);
    if (hipDeviceSynchronize() || hipMemcpy(c.data(), dc, 8 * nw, hipMemcpyDeviceToHost)) {
      printf("%s failed\n", name);
      return;
    }
    std::vector<unsigned long long> s(c.begin(), c.begin() + nw);
    std::sort(s.begin(), s.end());
    const double per = s[nw / 2] / (double)(reps * 8 * chains);
    const int wps = threads / 64;
    if (chains == 1)
      printf("%-10s latency    %7.1f cycles per dependent op (1 wave/SIMD)\n", name, per);
    else
      printf("%-10s throughput %7.1f SIMD cycles per wave-op (%d waves/SIMD, %d chains)\n", name, per / wps, wps,
             chains);
  };
#define RUN(OP, NAME)                               \
  run(bench<OP, 1>, NAME, 64, 1);                   \
  run(bench<OP, 8>, NAME, 256, 8);
  RUN(OP_FMA64, "fma f64");
  RUN(OP_FMA32, "fma f32");
  RUN(OP_DIV64, "div f64");
  RUN(OP_SQRT64, "sqrt f64");
  RUN(OP_RSQ64, "rsq f64");
  RUN(OP_SIN64, "sin f64");
  RUN(OP_COS64, "cos f64");
  RUN(OP_ATAN2_64, "atan2 f64");
  RUN(OP_LDS64, "lds f64");
  RUN(OP_CVT, "f64-f32");
  return 0;
}
