// lsm_edges.hip -- device-side GNNBase.process_adj: dense per-ego adjacency -> (edge_index, edge_attr).
//
// Reference: onpolicy/algorithms/utils/gnn.py:376-407 (GNNBase.process_adj). For a batch of B
// adjacency matrices adj[B][E][E] the reference computes
//     idx        = adj.nonzero()                       (row-major order over (b, r, c))
//     edge_attr  = adj[idx[:,0], idx[:,1], idx[:,2]].unsqueeze(1)        float [nnz][1]
//     edge_index = stack([b*E + r, b*E + c])                             int64 [2][nnz]
// and the 2-D case (B = 1) is the same thing with b = 0. SURVEY §8(f) row 2: emit the learner's
// graph input straight from the rollout's device buffers instead of the dense (n, N, E, E) tensor.
//
// Two adjacency sources:
//   reference layout  adj[b][r][c]                     (LSM_ADJ_REFERENCE, b = env*N + ego)
//   compact layout    A[env][r][c] + M[env][ego][W]    (LSM_ADJ_COMPACT): the reference value is
//                     (M bit r | M bit c) ? 0 : A[r][c]; expanded on the fly, never materialised.
//
// Three launches, all HBM/L2-streaming integer work (no MFMA):
//   edge_count_kernel   one wave per graph: nonzero count via 64-lane ballots -> counts[b]
//   scan (hipcub)       inclusive sum of counts -> offsets[1..B], offsets[0] = 0, offsets[B] = nnz
//   edge_emit_kernel    one wave per graph: re-reads its E*E values (L2 / MALL resident after the
//                       count pass) and writes its edges at offsets[b] in row-major order; the
//                       in-chunk position is the popcount of the ballot below the lane (mbcnt), so
//                       the output order is exactly nonzero()'s; edges are compacted in LDS and
//                       stored by consecutive lanes. The _dev entry reads nnz = offsets[B] on the
//                       device (outputs sized by an upper bound), so the three launches run back to
//                       back with the one host sync after all of them.
// A graph's E*E values are walked as one flat index k = r*E + c in 64-lane chunks (4 elements per
// lane with one 16-B load when E is even), so every lane is busy whatever E is (E = 24 rows would
// leave 40 of 64 lanes idle per row).
#include <hip/hip_runtime.h>
#include <hipcub/device/device_scan.hpp>

#include <cstdint>

namespace {

constexpr int WAVE = 64;
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int GRAPHS_PER_BLOCK = 4;   // 256-thread workgroups, one wave per graph

struct AdjSrc {
  const float* adj;         // reference: [B][E][E]; compact: [B / N][E][E]
  const uint64_t* masks;    // compact only: [B][W] (== [n][N][W]); nullptr for reference
  int64_t B;
  int32_t E, N, W;
  float inv_e;              // 1 / E for the flat-index row split
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Row of flat index k (< E*E <= 65536): floor((k + 0.5) / E) in fp32 is exact here -- the
// distance of (k + 0.5) / E from an integer is >= 0.5 / E >= 1/512, far above fp32 rounding.
__device__ __forceinline__ int row_of(int k, float inv_e) { return (int)(((float)k + 0.5f) * inv_e); }

// The compact layout's disconnect words of one graph (W = ceil(E / 64) <= 4), loaded once per wave
// before its element loads and held in registers. Round 5's kernels read the word of every element
// from global memory next to the element's own load; a 4-chunk variant of them undercounted one
// edge in a few graphs of some calls on unchanged inputs (profiles/r05_s21_edges_diag.txt). With
// the words in registers the only global loads left in the element loop are the adjacency values.
struct MaskRegs {
  uint64_t w0, w1, w2, w3;
  bool on;   // compact layout
};

__device__ __forceinline__ MaskRegs load_masks(const uint64_t* m, int W) {
  MaskRegs M;
  M.on = m != nullptr;
  M.w0 = M.w1 = M.w2 = M.w3 = 0ull;
  if (M.on) {
    // wave-uniform address: one load per word for the wave, complete before the first use
    M.w0 = m[0];
    if (W > 1) M.w1 = m[1];
    if (W > 2) M.w2 = m[2];
    if (W > 3) M.w3 = m[3];
  }
  return M;
}

// bit r of the graph's disconnect words, by selects (no branch on the lane-varying word index)
__device__ __forceinline__ uint32_t mbit(const MaskRegs& M, int r) {
  const uint32_t q = (uint32_t)r >> 6;
  uint64_t x = M.w0;
  x = q == 1u ? M.w1 : x;
  x = q == 2u ? M.w2 : x;
  x = q == 3u ? M.w3 : x;
  return (uint32_t)(x >> (r & 63)) & 1u;
}

// v, or +0.0 when row r or column c is disconnected (the reference assigns 0 to those entries,
// navigation_graph_safe.py:976-989): an AND with an all-ones / all-zeros word, branch-free
__device__ __forceinline__ float mask_val(float v, const MaskRegs& M, int r, int c) {
  const uint32_t drop = mbit(M, r) | mbit(M, c);
  return __uint_as_float(__float_as_uint(v) & (drop - 1u));
}

// Value of element k of graph b (0 where masked in the compact layout).
__device__ __forceinline__ float load_val(const AdjSrc& s, const float* g, const MaskRegs& M, int k) {
  const float v = __builtin_nontemporal_load(g + k);
  if (!M.on) return v;
  const int r = row_of(k, s.inv_e);
  return mask_val(v, M, r, k - r * s.E);
}

__device__ __forceinline__ const float* graph_ptr(const AdjSrc& s, int64_t b) {
  const int64_t EE = (int64_t)s.E * s.E;
  return s.adj + (s.masks ? (b / s.N) : b) * EE;
}

// VEC = 4 (E even, so every graph and row pair is 16-B aligned): each lane takes 4 consecutive
// elements with one 16-B load; its nonzero count c in [0, 4] is spread over 3 ballots (bit k of c),
// so the exclusive prefix over lanes is sum_k 2^k * popcount(ballot_k below the lane).
template <int VEC>
__device__ __forceinline__ int lane_vals(const AdjSrc& s, const float* g, const MaskRegs& M, int k, int EE,
                                         float (&v)[VEC]) {
  int c = 0;
  if (VEC == 1) {
    v[0] = k < EE ? load_val(s, g, M, k) : 0.0f;
    c = v[0] != 0.0f;
  } else {
    if (k < EE) {
      const f32x4 q = __builtin_nontemporal_load((const f32x4*)(g + k));
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      if (M.on) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int r = row_of(k + i, s.inv_e);
          v[i] = mask_val(v[i], M, r, k + i - r * s.E);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) v[i] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) c += v[i] != 0.0f;   // NaN counts, -0.0 does not (torch)
  }
  return c;
}

__device__ __forceinline__ uint32_t below(uint64_t bal) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

template <int VEC>
__global__ __launch_bounds__(256) void edge_count_kernel(AdjSrc s, int64_t* __restrict__ counts,
                                                         int64_t* __restrict__ offsets) {
  const int64_t b = (int64_t)blockIdx.x * GRAPHS_PER_BLOCK + (threadIdx.x >> 6);
  if (b >= s.B) return;   // whole wave exits together
  const float* g = graph_ptr(s, b);
  const MaskRegs M = load_masks(s.masks ? s.masks + b * s.W : nullptr, s.W);
  const int EE = s.E * s.E;
  int cnt = 0;
  for (int k0 = 0; k0 < EE; k0 += WAVE * VEC) {
    float v[VEC];
    const int c = lane_vals<VEC>(s, g, M, k0 + VEC * lane_id(), EE, v);
    if (VEC == 1) {
      cnt += __popcll(__ballot(c != 0));
    } else {
      cnt += __popcll(__ballot(c & 1)) + 2 * __popcll(__ballot(c & 2)) + 4 * __popcll(__ballot(c & 4));
    }
  }
  if (lane_id() == 0) counts[b] = cnt;
  if (b == 0 && lane_id() == 0) offsets[0] = 0;   // the scan fills offsets[1..B]
}

// The chunk's edges are first compacted into the wave's LDS slice (flat index + value at their
// exclusive-prefix slot), then written out by consecutive lanes: every store instruction covers
// consecutive edge slots (full 512-B / 256-B lines), where storing straight from the lane that found
// the edge would scatter each instruction over partial lines.
// nnz < 0: read it on the device (offsets[B]); the outputs then hold `cap` edges, and nothing is
// written when nnz > cap (the caller sees nnz and reports it).
// bad != nullptr: the offsets came from counts the caller supplied (the step kernel's
// LSM_OUT_ADJ_NNZ), not from this file's count pass; a graph whose nonzeros differ from its slot
// (offsets[b + 1] - offsets[b]) increments *bad, and its slot is zero-filled rather than left unset.
template <int VEC>
__global__ __launch_bounds__(256) void edge_emit_kernel(AdjSrc s, const int64_t* __restrict__ offsets,
                                                        int64_t nnz, int64_t cap, int64_t* __restrict__ edge_index,
                                                        float* __restrict__ edge_attr, int64_t* __restrict__ bad) {
  __shared__ int32_t sk[GRAPHS_PER_BLOCK][WAVE * VEC];
  __shared__ float sv[GRAPHS_PER_BLOCK][WAVE * VEC];
  const int w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * GRAPHS_PER_BLOCK + w;
  if (b >= s.B) return;
  if (nnz < 0) {
    nnz = offsets[s.B];
    if (nnz > cap) return;
  }
  const float* g = graph_ptr(s, b);
  const MaskRegs M = load_masks(s.masks ? s.masks + b * s.W : nullptr, s.W);
  const int EE = s.E * s.E;
  const int lane = lane_id();
  const int64_t node0 = b * s.E;
  const int64_t pos0 = offsets[b];
  int64_t pos = pos0;
  const int64_t end = offsets[b + 1];
  if (end > nnz || pos0 > end) {   // caller's nnz is stale / bad counts: write nothing out of bounds
    if (bad && lane == 0) atomicAdd((unsigned long long*)bad, 1ull);
    return;
  }
  int64_t found = 0;   // the graph's nonzeros (checked against its slot when the counts are given)
  for (int k0 = 0; k0 < EE && (bad || pos < end); k0 += WAVE * VEC) {
    const int k = k0 + VEC * lane;
    float v[VEC];
    const int c = lane_vals<VEC>(s, g, M, k, EE, v);
    uint32_t pre;
    int tot;
    if (VEC == 1) {
      const uint64_t bal = __ballot(c != 0);
      pre = below(bal);
      tot = __popcll(bal);
    } else {
      const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
      pre = below(b0) + 2 * below(b1) + 4 * below(b2);
      tot = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    }
    found += tot;
    if (c) {
      int o = (int)pre;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        if (v[i] != 0.0f) {
          sk[w][o] = k + i;
          sv[w][o] = v[i];
          ++o;
        }
      }
    }
    // intra-wave LDS hand-off (the block's waves run different graphs: no block barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int room = (int)(end - pos < (int64_t)tot ? end - pos : (int64_t)tot);   // never past the slot
    for (int t = lane; t < room; t += WAVE) {
      const int kk = sk[w][t];
      const int r = row_of(kk, s.inv_e);
      edge_index[pos + t] = node0 + r;
      edge_index[nnz + pos + t] = node0 + (kk - r * s.E);
      edge_attr[pos + t] = sv[w][t];
    }
    __builtin_amdgcn_wave_barrier();   // slots are rewritten by the next chunk
    pos += room;
  }
  if (bad && found != end - pos0) {
    for (int64_t t = pos + lane; t < end; t += WAVE) {   // a short graph: its slot's tail zeroed
      edge_index[t] = 0;
      edge_index[nnz + t] = 0;
      edge_attr[t] = 0.0f;
    }
    if (lane == 0) atomicAdd((unsigned long long*)bad, 1ull);
  }
}

// offsets[0] = 0 and the error word offsets[B + 1] = 0 before the scan / emit of the counts path
__global__ void offsets_init_kernel(int64_t* offsets, int64_t B) {
  if (threadIdx.x == 0) {
    offsets[0] = 0;
    offsets[B + 1] = 0;
  }
}

thread_local char g_err[256];

int fail(const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return 1;
}

int make_src(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N, AdjSrc* s) {
  if (!adj) return fail("adj is null");
  if (B < 0) return fail("B < 0");
  if (E <= 0 || E > 256) return fail("E must be in [1, 256]");
  if (masks && (N <= 0 || B % N != 0)) return fail("compact layout: B must be a multiple of N > 0");
  s->adj = adj;
  s->masks = masks;
  s->B = B;
  s->E = E;
  s->N = masks ? N : 1;
  s->W = (E + 63) / 64;
  s->inv_e = 1.0f / (float)E;
  return 0;
}

size_t scan_temp_bytes(int64_t B) {
  size_t bytes = 0;
  if (hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr, (int)B) !=
      hipSuccess)
    return 0;   // lsm_edges_count then reports "scan failed"
  return bytes;
}

}  // namespace

extern "C" {

const char* lsm_edges_last_error(void) { return g_err; }

size_t lsm_edges_workspace_bytes(int64_t B) {
  const size_t counts = ((size_t)B * sizeof(int64_t) + 255) & ~(size_t)255;
  return counts + scan_temp_bytes(B) + 256;
}

int lsm_edges_count(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                    int64_t* offsets, void* workspace, size_t workspace_bytes, void* stream) {
  AdjSrc s;
  if (make_src(adj, masks, B, E, N, &s)) return 1;
  if (B > INT32_MAX) return fail("B exceeds the scan's int32 item count");
  if (!offsets) return fail("offsets is null");
  if (workspace_bytes < lsm_edges_workspace_bytes(B)) return fail("workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (B == 0) return hipMemsetAsync(offsets, 0, sizeof(int64_t), st) == hipSuccess ? 0 : fail("memset failed");
  int64_t* counts = (int64_t*)workspace;
  const size_t cbytes = ((size_t)B * sizeof(int64_t) + 255) & ~(size_t)255;
  void* temp = (char*)workspace + cbytes;
  size_t tbytes = workspace_bytes - cbytes;
  const int64_t blocks = (B + GRAPHS_PER_BLOCK - 1) / GRAPHS_PER_BLOCK;
  if (E % 2 == 0) edge_count_kernel<4><<<dim3((unsigned)blocks), 256, 0, st>>>(s, counts, offsets);
  else edge_count_kernel<1><<<dim3((unsigned)blocks), 256, 0, st>>>(s, counts, offsets);
  if (hipcub::DeviceScan::InclusiveSum(temp, tbytes, counts, offsets + 1, (int)B, st) != hipSuccess)
    return fail("scan failed");
  return hipGetLastError() == hipSuccess ? 0 : fail("launch failed");
}

int lsm_edges_emit(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                   const int64_t* offsets, int64_t nnz, int64_t* edge_index, float* edge_attr,
                   void* stream) {
  AdjSrc s;
  if (make_src(adj, masks, B, E, N, &s)) return 1;
  if (!offsets) return fail("offsets is null");
  if (nnz < 0) return fail("nnz < 0");
  if (nnz > 0 && (!edge_index || !edge_attr)) return fail("edge_index / edge_attr is null");
  if (B == 0 || nnz == 0) return 0;
  const int64_t blocks = (B + GRAPHS_PER_BLOCK - 1) / GRAPHS_PER_BLOCK;
  if (E % 2 == 0)
    edge_emit_kernel<4><<<dim3((unsigned)blocks), 256, 0, (hipStream_t)stream>>>(s, offsets, nnz, nnz, edge_index,
                                                                                 edge_attr, nullptr);
  else
    edge_emit_kernel<1><<<dim3((unsigned)blocks), 256, 0, (hipStream_t)stream>>>(s, offsets, nnz, nnz, edge_index,
                                                                                 edge_attr, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : fail("launch failed");
}

int lsm_edges_emit_dev(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                       const int64_t* offsets, int64_t cap, int64_t* edge_index, float* edge_attr,
                       void* stream) {
  AdjSrc s;
  if (make_src(adj, masks, B, E, N, &s)) return 1;
  if (!offsets) return fail("offsets is null");
  if (cap < 0) return fail("cap < 0");
  if (cap > 0 && (!edge_index || !edge_attr)) return fail("edge_index / edge_attr is null");
  if (B == 0 || cap == 0) return 0;
  const int64_t blocks = (B + GRAPHS_PER_BLOCK - 1) / GRAPHS_PER_BLOCK;
  if (E % 2 == 0)
    edge_emit_kernel<4><<<dim3((unsigned)blocks), 256, 0, (hipStream_t)stream>>>(s, offsets, -1, cap, edge_index,
                                                                                 edge_attr, nullptr);
  else
    edge_emit_kernel<1><<<dim3((unsigned)blocks), 256, 0, (hipStream_t)stream>>>(s, offsets, -1, cap, edge_index,
                                                                                 edge_attr, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : fail("launch failed");
}

int lsm_edges_scan_emit(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                        const int64_t* counts, int64_t* offsets, void* workspace, size_t workspace_bytes, int64_t cap,
                        int64_t* edge_index, float* edge_attr, void* stream) {
  AdjSrc s;
  if (make_src(adj, masks, B, E, N, &s)) return 1;
  if (B > INT32_MAX) return fail("B exceeds the scan's int32 item count");
  if (!counts || !offsets) return fail("counts / offsets is null");
  if (cap < 0) return fail("cap < 0");
  if (cap > 0 && (!edge_index || !edge_attr)) return fail("edge_index / edge_attr is null");
  if (workspace_bytes < lsm_edges_workspace_bytes(B)) return fail("workspace too small");
  hipStream_t st = (hipStream_t)stream;
  offsets_init_kernel<<<1, 64, 0, st>>>(offsets, B);
  if (B == 0) return hipGetLastError() == hipSuccess ? 0 : fail("launch failed");
  const size_t cbytes = ((size_t)B * sizeof(int64_t) + 255) & ~(size_t)255;
  void* temp = (char*)workspace + cbytes;
  size_t tbytes = workspace_bytes - cbytes;
  if (hipcub::DeviceScan::InclusiveSum(temp, tbytes, counts, offsets + 1, (int)B, st) != hipSuccess)
    return fail("scan failed");
  if (cap > 0) {
    const int64_t blocks = (B + GRAPHS_PER_BLOCK - 1) / GRAPHS_PER_BLOCK;
    // the scan above rewrote offsets[B]; the error word offsets[B + 1] was cleared before it
    if (E % 2 == 0)
      edge_emit_kernel<4><<<dim3((unsigned)blocks), 256, 0, st>>>(s, offsets, -1, cap, edge_index, edge_attr,
                                                                  offsets + B + 1);
    else
      edge_emit_kernel<1><<<dim3((unsigned)blocks), 256, 0, st>>>(s, offsets, -1, cap, edge_index, edge_attr,
                                                                  offsets + B + 1);
  }
  return hipGetLastError() == hipSuccess ? 0 : fail("launch failed");
}

}  // extern "C"
