// lsm_metrics.hip -- the episode-summary reduction behind the runner's per-episode log.
//
// Reference: GMPERunner's episode parse (onpolicy/runner/shared/graph_mpe_runner.py:222-251)
// averages seven fields of the per-thread ep_info dicts over threads and takes the minimum of
// `min_distance_min`. Here one rank's [n][8] float64 ep_info (LSM_OUT_EP_INFO) becomes
//   out[0..7] = column sums, out[8] = n, out[9] = min of column 6 (NaN-propagating, like np.min)
// in ONE launch (one 1024-thread workgroup), with no host synchronisation: out[0..8] then goes through an all_reduce(SUM) and
// out[9] through an all_reduce(MIN) over RCCL (lsm/dist.py), and mean = sum / count on the host
// after the rollout. The order of the float64 additions is fixed (per-thread strided rows, then a
// wave butterfly and the 16 wave partials in order), so the result is reproducible run to run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace {

constexpr int BT = 1024;   // one workgroup of 16 waves: 4 rows per thread at 4096 envs
constexpr int RB = 4;      // rows loaded per batch (their 16 loads are issued together)

__device__ __forceinline__ double nanmin(double m, double v) {   // np.min: NaN propagates
  if (v != v) return v;
  return (m == m && v < m) ? v : m;
}

// Fixed order: thread t adds rows t, t + BT, ... in row order; then a butterfly over the 64 lanes
// of each wave (xor 32, 16, ..., 1) and the 16 wave partials in wave order on lane 0 of wave 0.
// The loads of RB rows are issued before their additions (one memory round trip per batch; the
// former 256-thread loop waited for every row in turn: 9.6 us per launch at 4096 envs).
__global__ __launch_bounds__(BT) void episode_summary_kernel(const double* __restrict__ ep, int32_t n,
                                                             double* __restrict__ out) {
  __shared__ double part[BT / 64][9];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double mn = INFINITY;
  typedef double f64x2 __attribute__((ext_vector_type(2)));
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
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) part[wv][k] = acc[k];
    part[wv][8] = mn;
  }
  __syncthreads();
  if (t < 9) {
    double s = part[0][t];
    for (int w = 1; w < BT / 64; ++w) s = (t == 8) ? nanmin(s, part[w][t]) : s + part[w][t];
    out[t == 8 ? 9 : t] = s;
  }
  if (t == 9) out[8] = (double)n;
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
