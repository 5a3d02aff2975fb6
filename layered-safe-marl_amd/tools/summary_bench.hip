// DIAGNOSTIC microbenchmark (not part of the product): variants of the episode-summary reduction
// (lsm_metrics.hip) on n x 8 float64 rows -> 8 column sums, n, min of column 6 (NaN-propagating).
// Times back-to-back launches with HIP events and checks every variant's sums against the first.
//   hipcc --offload-arch=gfx950 -O3 -o tools/summary_bench tools/summary_bench.hip && tools/summary_bench 4096
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef double f64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double nanmin(double m, double v) {
  if (v != v) return v;
  return (m == m && v < m) ? v : m;
}

// BT threads, RB rows per load batch; wave butterfly, then the BT/64 wave partials combined either
// serially by 9 threads (TREE = 0, the shipped kernel) or by a butterfly over the partials (TREE = 1)
template <int BT, int RB, int TREE>
__global__ __launch_bounds__(BT) void summary_kernel(const double* __restrict__ ep, int n, double* __restrict__ out) {
  constexpr int NW = BT / 64;
  __shared__ double part[NW][9];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double mn = INFINITY;
  for (int r0 = t; r0 < n; r0 += RB * BT) {
    f64x2 v[RB][4];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int r = r0 + q * BT;
      const f64x2* row = (const f64x2*)(ep + (size_t)(r < n ? r : 0) * 8);
#pragma unroll
      for (int c = 0; c < 4; ++c) v[q][c] = row[c];
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      if (r0 + q * BT >= n) break;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[2 * c] += v[q][c].x;
        acc[2 * c + 1] += v[q][c].y;
      }
      mn = nanmin(mn, v[q][3].x);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = acc[k] + __shfl_xor(acc[k], off);
    mn = nanmin(mn, __shfl_xor(mn, off));
  }
  if (NW == 1) {
    if (lane < 8) out[lane] = acc[lane];   // (register array indexed by lane: small select chain)
    if (lane == 8) out[9] = mn;
    if (lane == 9) out[8] = (double)n;
    return;
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) part[wv][k] = acc[k];
    part[wv][8] = mn;
  }
  __syncthreads();
  if (TREE == 0) {
    if (t < 9) {
      double s = part[0][t];
      for (int w = 1; w < NW; ++w) s = (t == 8) ? nanmin(s, part[w][t]) : s + part[w][t];
      out[t == 8 ? 9 : t] = s;
    }
    if (t == 9) out[8] = (double)n;
  } else {
    // wave 0: lane l < 9 * NW holds partial (w = l / 9, k = l % 9)... simpler: lanes k + 16 w? use
    // lanes w (< NW) per column k, 9 butterflies of log2(NW) levels
    if (wv == 0) {
      const int w = lane & (NW - 1);
      double s[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) s[k] = part[w][k];
#pragma unroll
      for (int off = NW / 2; off > 0; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = s[k] + __shfl_xor(s[k], off);
        s[8] = nanmin(s[8], __shfl_xor(s[8], off));
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = s[k];
        out[9] = s[8];
        out[8] = (double)n;
      }
    }
  }
}

// Coalesced: lane l of the block loads 16-B chunk q = t, t + BT, ... of the row-major array, so a
// wave's load is 1 KB contiguous; BT % 4 == 0 keeps thread t on columns 2c, 2c + 1 (c = t % 4).
// Wave butterfly over lanes of equal c (xor 4 .. 32), then the NW x 4 wave partials by 4 lanes.
template <int BT, int RB>
__global__ __launch_bounds__(BT) void summary_coal(const double* __restrict__ ep, int n, double* __restrict__ out) {
  constexpr int NW = BT / 64;
  __shared__ double part[NW][4][3];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, c = t & 3;
  const f64x2* src = (const f64x2*)ep;
  const int nq = 4 * n;
  double a0 = 0.0, a1 = 0.0, mn = INFINITY;
  for (int q0 = t; q0 < nq; q0 += RB * BT) {
    f64x2 v[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int q = q0 + r * BT;
      v[r] = src[q < nq ? q : 0];
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (q0 + r * BT >= nq) break;
      a0 += v[r].x;
      a1 += v[r].y;
      if (c == 3) mn = nanmin(mn, v[r].x);
    }
  }
#pragma unroll
  for (int off = 4; off < 64; off <<= 1) {
    a0 = a0 + __shfl_xor(a0, off);
    a1 = a1 + __shfl_xor(a1, off);
    mn = nanmin(mn, __shfl_xor(mn, off));
  }
  if (lane < 4) {
    part[wv][lane][0] = a0;
    part[wv][lane][1] = a1;
    part[wv][lane][2] = mn;
  }
  __syncthreads();
  if (t < 4) {
    double s0 = part[0][t][0], s1 = part[0][t][1], m = part[0][t][2];
    for (int w = 1; w < NW; ++w) {
      s0 += part[w][t][0];
      s1 += part[w][t][1];
      m = nanmin(m, part[w][t][2]);
    }
    out[2 * t] = s0;
    out[2 * t + 1] = s1;
    if (t == 3) out[9] = m;
    if (t == 0) out[8] = (double)n;
  }
}

template <class F>
static float time_us(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) f();
  CHK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

__global__ void empty_kernel() {}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  std::vector<double> h((size_t)n * 8);
  srand(7);
  for (auto& x : h) x = (double)rand() / RAND_MAX;
  double *ep, *out;
  CHK(hipMalloc(&ep, h.size() * 8));
  CHK(hipMalloc(&out, 16 * 8 * 32));   // 16 doubles per variant, up to 32 variants
  CHK(hipMemcpy(ep, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  struct V { const char* name; void (*k)(const double*, int, double*); int bt; };
  const V vs[] = {
      {"1024 thr RB4 serial (shipped)", summary_kernel<1024, 4, 0>, 1024},
      {"1024 thr RB4 tree", summary_kernel<1024, 4, 1>, 1024},
      {"512 thr RB8 tree", summary_kernel<512, 8, 1>, 512},
      {"256 thr RB8 tree", summary_kernel<256, 8, 1>, 256},
      {"256 thr RB4 tree", summary_kernel<256, 4, 1>, 256},
      {"64 thr RB8 (one wave)", summary_kernel<64, 8, 1>, 64},
      {"coal 1024 RB16", summary_coal<1024, 16>, 1024},
      {"coal 1024 RB4", summary_coal<1024, 4>, 1024},
      {"coal 512 RB8", summary_coal<512, 8>, 512},
      {"coal 512 RB32", summary_coal<512, 32>, 512},
      {"coal 256 RB16", summary_coal<256, 16>, 256},
      {"coal 256 RB64", summary_coal<256, 64>, 256},
      {"coal 128 RB32", summary_coal<128, 32>, 128},
  };
  const int NV = sizeof(vs) / sizeof(vs[0]);
  static_assert(sizeof(vs) / sizeof(vs[0]) <= 32, "out holds 32 variants");
  printf("{\"envs\": %d, \"empty_kernel_us\": %.2f", n,
         time_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0); }, 200));
  std::vector<double> ref(10), got(10);
  for (int i = 0; i < NV; ++i) {
    double* o = out + 16 * i;
    const float us = time_us([&] { hipLaunchKernelGGL(vs[i].k, dim3(1), dim3(vs[i].bt), 0, 0, ep, n, o); }, 200);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(got.data(), o, 80, hipMemcpyDeviceToHost));
    if (i == 0) ref = got;
    double md = 0;
    for (int k = 0; k < 10; ++k) md = fmax(md, fabs(got[k] - ref[k]) / fmax(1e-300, fabs(ref[k])));
    printf(", \"%s\": {\"us\": %.2f, \"max_rel_diff_vs_shipped\": %.2e}", vs[i].name, us, md);
  }
  printf("}\n");
  return 0;
}
