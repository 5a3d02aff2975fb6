// movb64_hazard.hip -- does a v_mov_b32 to the low half of a register pair that a v_mov_b64 wrote
// just before take effect on gfx950? (WAW ordering of the 64-bit move and a 32-bit VALU write)
//
// The compiler emitted exactly this pair in edge_emit_kernel<4> (the compact layout's masked value:
// `v_mov_b64 v[34:35], v[4:5]` ... `v_mov_b32 v34, 0`), and that build miscounted edges. Each
// variant below runs the sequence with 0..3 independent instructions between the two writes and
// checks the low word is the 32-bit move's. Build and run:
//   hipcc --offload-arch=gfx950 -O2 -o movb64_hazard movb64_hazard.hip && ./movb64_hazard
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

template <int GAP>
__global__ void waw_kernel(const uint64_t* in, uint64_t* out, int n, int reps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = in[i];
  uint64_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    uint64_t y;
    if (GAP == 0) {
      asm volatile("v_mov_b64 v[40:41], %1\n\tv_mov_b32 v40, 0\n\tv_mov_b64 %0, v[40:41]"
                   : "=v"(y) : "v"(x) : "v40", "v41");
    } else if (GAP == 1) {
      asm volatile("v_mov_b64 v[40:41], %1\n\tv_mov_b32 v42, 1\n\tv_mov_b32 v40, 0\n\tv_mov_b64 %0, v[40:41]"
                   : "=v"(y) : "v"(x) : "v40", "v41", "v42");
    } else if (GAP == 2) {
      asm volatile("v_mov_b64 v[40:41], %1\n\tv_mov_b32 v42, 1\n\tv_mov_b32 v43, 2\n\tv_mov_b32 v40, 0\n\t"
                   "v_mov_b64 %0, v[40:41]"
                   : "=v"(y) : "v"(x) : "v40", "v41", "v42", "v43");
    } else {
      // the compiler's own shape: 64-bit moves of two pairs, then the 32-bit write of the low half
      asm volatile("v_mov_b64 v[44:45], %1\n\tv_and_b32 v42, 1, v42\n\tv_mov_b32 v43, 0\n\t"
                   "v_mov_b64 v[40:41], %1\n\tv_cmp_eq_u64 vcc, 0, v[42:43]\n\tv_mov_b32 v40, 0\n\t"
                   "v_mov_b64 %0, v[40:41]"
                   : "=v"(y) : "v"(x) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
    }
    acc += (y & 0xffffffffull) != 0 ? 1 : 0;   // the low word must be 0
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    if ((x & 0xffffffffull) == 0) x |= 1;
  }
  out[i] = acc;
}

template <int GAP>
static long run(int n, int reps) {
  std::vector<uint64_t> h(n);
  for (int i = 0; i < n; ++i) h[i] = 0x9e3779b97f4a7c15ull * (i + 1) | 1ull;
  uint64_t *din, *dout;
  hipMalloc(&din, n * 8);
  hipMalloc(&dout, n * 8);
  hipMemcpy(din, h.data(), n * 8, hipMemcpyHostToDevice);
  waw_kernel<GAP><<<(n + 255) / 256, 256>>>(din, dout, n, reps);
  hipMemcpy(h.data(), dout, n * 8, hipMemcpyDeviceToHost);
  hipFree(din);
  hipFree(dout);
  long bad = 0;
  for (int i = 0; i < n; ++i) bad += (long)h[i];
  return bad;
}

int main() {
  const int n = 1 << 20, reps = 64;
  printf("gap 0: %ld of %ld low words not overwritten\n", run<0>(n, reps), (long)n * reps);
  printf("gap 1: %ld of %ld\n", run<1>(n, reps), (long)n * reps);
  printf("gap 2: %ld of %ld\n", run<2>(n, reps), (long)n * reps);
  printf("compiler shape: %ld of %ld\n", run<3>(n, reps), (long)n * reps);
  return 0;
}
