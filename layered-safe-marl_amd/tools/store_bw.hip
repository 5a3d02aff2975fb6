// store_bw.hip -- achievable HBM write rate for the rollout's output pattern (diagnostic tool,
// not part of the library). Each wave writes `chunk` contiguous bytes per stream with 16-B
// stores, `streams` separate output arrays (as an env's wave writes adjacency, node features,
// info rows, ... to different tensors), over `waves` waves resident at once; plus a plain
// grid-stride stream of the same total as the reference point.
//   hipcc --offload-arch=gfx950 -O3 -o store_bw store_bw.hip && ./store_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

struct Streams {
  f32x4* p[8];
  unsigned n16[8];   // 16-B words per wave in stream s
};

// one wave per env: for each stream, the env's contiguous chunk
__global__ __launch_bounds__(256) void chunks_kernel(Streams S, int nstreams, int waves, int nt) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= waves) return;
  const f32x4 v = {1.0f, 2.0f, 3.0f, (float)w};
  for (int s = 0; s < nstreams; ++s) {
    f32x4* d = S.p[s] + (size_t)w * S.n16[s];
    const unsigned n = S.n16[s];
    if (nt) {
      for (unsigned k = lane; k < n; k += 64) __builtin_nontemporal_store(v, d + k);
    } else {
      for (unsigned k = lane; k < n; k += 64) d[k] = v;
    }
  }
}

__global__ __launch_bounds__(256) void stride_kernel(f32x4* d, size_t n16) {
  const f32x4 v = {1.0f, 2.0f, 3.0f, 4.0f};
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n16; k += (size_t)gridDim.x * blockDim.x)
    d[k] = v;
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 4096;
  // config 3's per-env output streams (bytes): adjacency, node features, info rows, obs, record
  const std::vector<unsigned> per_env = {18432, 7680, 1152, 224, 3936};
  Streams S;
  size_t total = 0;
  for (size_t s = 0; s < per_env.size(); ++s) {
    S.n16[s] = per_env[s] / 16;
    CK(hipMalloc(&S.p[s], (size_t)per_env[s] * waves));
    total += (size_t)per_env[s] * waves;
  }
  f32x4* flat;
  CK(hipMalloc(&flat, total));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200;
  for (int mode = 0; mode < 4; ++mode) {
    for (int i = 0; i < 20; ++i) {
      if (mode < 2) chunks_kernel<<<(waves + 3) / 4, 256>>>(S, (int)per_env.size(), waves, mode);
      else if (mode == 2) stride_kernel<<<1024 * 4, 256>>>(flat, total / 16);
      else chunks_kernel<<<(waves + 3) / 4, 256>>>(S, 1, waves, 0);
    }
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) {
      if (mode < 2) chunks_kernel<<<(waves + 3) / 4, 256>>>(S, (int)per_env.size(), waves, mode);
      else if (mode == 2) stride_kernel<<<1024 * 4, 256>>>(flat, total / 16);
      else chunks_kernel<<<(waves + 3) / 4, 256>>>(S, 1, waves, 0);
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = 1000.0 * ms / reps;
    const size_t bytes = mode == 3 ? (size_t)per_env[0] * waves : total;
    const char* name[] = {"env chunks, 5 streams", "env chunks, 5 streams, nontemporal", "grid-stride, one stream",
                          "env chunks, adjacency only"};
    printf("%-40s %8.2f us  %7.1f MB  %6.2f TB/s\n", name[mode], us, bytes / 1e6, bytes / us / 1e6);
  }
  return 0;
}
