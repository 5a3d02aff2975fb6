// lsm_metrics.hip -- the episode-summary reduction behind the runner's per-episode log.
//
// Reference: GMPERunner's episode parse (onpolicy/runner/shared/graph_mpe_runner.py:222-251)
// averages seven fields of the per-thread ep_info dicts over threads and takes the minimum of
// `min_distance_min`. Here one rank's [n][8] float64 ep_info (LSM_OUT_EP_INFO) becomes
//   out[0..7] = column sums, out[8] = n, out[9] = min of column 6 (NaN-propagating, like np.min)
// in ONE launch, with no host synchronisation: out[0..8] then goes through an all_reduce(SUM) and
// out[9] through an all_reduce(MIN) over RCCL (lsm/dist.py), and mean = sum / count on the host
// after the rollout. The order of the float64 additions is fixed (per-thread strided rows, then a
// fixed LDS tree), so the result is reproducible run to run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace {

constexpr int BT = 256;

__global__ __launch_bounds__(BT) void episode_summary_kernel(const double* __restrict__ ep, int32_t n,
                                                             double* __restrict__ out) {
  __shared__ double part[9][BT];
  const int t = threadIdx.x;
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double mn = INFINITY;
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  for (int r = t; r < n; r += BT) {
    const f64x2* row = (const f64x2*)(ep + (size_t)r * 8);
    const f64x2 a = row[0], b = row[1], c = row[2], d = row[3];
    acc[0] += a.x; acc[1] += a.y; acc[2] += b.x; acc[3] += b.y;
    acc[4] += c.x; acc[5] += c.y; acc[6] += d.x; acc[7] += d.y;
    const double v = d.x;
    if (v != v) mn = v;
    else if (mn == mn && v < mn) mn = v;
  }
  for (int k = 0; k < 8; ++k) part[k][t] = acc[k];
  part[8][t] = mn;
  __syncthreads();
  for (int s = BT / 2; s > 0; s >>= 1) {
    if (t < s) {
      for (int k = 0; k < 8; ++k) part[k][t] = part[k][t] + part[k][t + s];
      const double o = part[8][t + s], m = part[8][t];
      if (o != o) part[8][t] = o;
      else if (m == m && o < m) part[8][t] = o;
    }
    __syncthreads();
  }
  if (t < 8) out[t] = part[t][0];
  if (t == 8) out[8] = (double)n;
  if (t == 9) out[9] = part[8][0];
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
