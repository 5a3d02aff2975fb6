// lsm_metrics.hip -- the episode-summary reduction behind the runner's per-episode log.
//
// Reference: GMPERunner's episode parse (onpolicy/runner/shared/graph_mpe_runner.py:222-251)
// averages seven fields of the per-thread ep_info dicts over threads and takes the minimum of
// `min_distance_min`. Here one rank's [n][8] float64 ep_info (LSM_OUT_EP_INFO) becomes
//   out[0..7] = column sums, out[8] = n, out[9] = min of column 6 (NaN-propagating, like np.min)
// in ONE launch (one 1024-thread workgroup), with no host synchronisation: out[0..8] then goes through an all_reduce(SUM) and
// out[9] through an all_reduce(MIN) over RCCL (lsm/dist.py), and mean = sum / count on the host
// after the rollout. The order of the float64 additions is fixed (below), so the result is
// reproducible run to run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace {

constexpr int BT = 1024;   // one workgroup of 16 waves
constexpr int RB = 16;     // 16-B chunks loaded per batch per thread (issued together: 4096 rows in one batch)

__device__ __forceinline__ double nanmin(double m, double v) {   // np.min: NaN propagates
  if (v != v) return v;
  return (m == m && v < m) ? v : m;
}

// The [n][8] rows as 4n 16-B chunks (columns 2c, 2c + 1 of a row in chunk c): thread t adds chunks
// t, t + BT, ... in order (a wave's load is 1 KB contiguous, and with BT % 4 == 0 thread t always
// holds columns 2c, 2c + 1, c = t % 4); then a butterfly over the 16 lanes of a wave with equal c
// (xor 4, 8, 16, 32) and the 16 wave partials in wave order on threads 0-3. Fixed order: the result
// is reproducible run to run. (The round-5 kernel, a row per thread with a 64-lane butterfly over
// all 9 values and a serial 16-partial combine: 9.1 us per launch at 4096 envs against 5.2 for
// this one, back to back, profiles/r06_s17_summary_bench.json, tools/summary_bench.hip.)
__global__ __launch_bounds__(BT) void episode_summary_kernel(const double* __restrict__ ep, int32_t n,
                                                             double* __restrict__ out) {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  __shared__ double part[BT / 64][4][3];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, c = t & 3;
  const f64x2* src = (const f64x2*)ep;
  const int64_t nq = 4 * (int64_t)n;
  double a0 = 0.0, a1 = 0.0, mn = INFINITY;
  for (int64_t q0 = t; q0 < nq; q0 += RB * BT) {
    f64x2 v[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int64_t q = q0 + r * BT;
      v[r] = src[q < nq ? q : 0];
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (q0 + r * BT >= nq) break;
      a0 += v[r].x;
      a1 += v[r].y;
      if (c == 3) mn = nanmin(mn, v[r].x);   // column 6 (min_distance_min)
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
    for (int w = 1; w < BT / 64; ++w) {
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

}  // namespace

extern "C" {

// See include/lsm_rollout.h.
int lsm_episode_summary(const double* ep_info, int32_t n, double* out, void* stream) {
  if (n < 0 || !out || (n > 0 && !ep_info)) return 1;
  if (((uintptr_t)ep_info & 15) != 0) return 1;   // 16-B row loads
  hipLaunchKernelGGL(episode_summary_kernel, dim3(1), dim3(BT), 0, (hipStream_t)stream, ep_info, n, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
