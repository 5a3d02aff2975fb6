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
#include <type_traits>

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

// bit r of the graph's disconnect words: an OR of masked words (no selection by index -- a select
// chain over the words was rewritten into a dynamically indexed copy of them in LDS)
__device__ __forceinline__ uint32_t mbit(const MaskRegs M, int r) {
  const uint32_t q = (uint32_t)r >> 6;
  const uint64_t x = (M.w0 & (0ull - (uint64_t)(q == 0u))) | (M.w1 & (0ull - (uint64_t)(q == 1u))) |
                     (M.w2 & (0ull - (uint64_t)(q == 2u))) | (M.w3 & (0ull - (uint64_t)(q == 3u)));
  return (uint32_t)(x >> (r & 63)) & 1u;
}

// v, or +0.0 when row r or column c is disconnected (the reference assigns 0 to those entries,
// navigation_graph_safe.py:976-989): an AND with an all-ones / all-zeros word, branch-free
__device__ __forceinline__ float mask_val(float v, const MaskRegs M, int r, int c) {
  const uint32_t drop = mbit(M, r) | mbit(M, c);
  return __uint_as_float(__float_as_uint(v) & (drop - 1u));
}

__device__ __forceinline__ const float* graph_ptr(const AdjSrc& s, int64_t b) {
  const int64_t EE = (int64_t)s.E * s.E;
  return s.adj + (s.masks ? (b / s.N) : b) * EE;
}

// VEC = 4 (E even, so every graph and row pair is 16-B aligned): each lane takes 4 consecutive
// elements with one 16-B load; its nonzero count c in [0, 4] is spread over 3 ballots (bit k of c),
// so the exclusive prefix over lanes is sum_k 2^k * popcount(ballot_k below the lane).
// A graph is walked in batches of CH chunks of WAVE * VEC elements: every chunk's load of a batch is
// issued before the first is used, one memory round trip per batch rather than per chunk (E = 24:
// the whole 576-element graph in one). Addresses are clamped into the graph (a chunk past EE re-reads
// the graph's first elements, L2 hits) and values past EE zeroed by select.
constexpr int CH = 4;

template <int VEC, int NB>
__device__ __forceinline__ void load_batch(const float* g, int k0, int EE, float (&v)[CH][VEC]) {
  const int lane = lane_id();
  typedef float f32x1 __attribute__((ext_vector_type(1)));
  typedef typename std::conditional<VEC == 4, f32x4, f32x1>::type vec_t;
  vec_t q[CH];
#pragma unroll
  for (int h = 0; h < NB; ++h) {   // every load issued first: no use, no branch between them
    const int k = k0 + h * WAVE * VEC + VEC * lane;
    q[h] = __builtin_nontemporal_load((const vec_t*)(g + (k < EE ? k : 0)));
  }
#pragma unroll
  for (int h = 0; h < NB; ++h) {
    const bool in = k0 + h * WAVE * VEC + VEC * lane < EE;
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[h][i] = in ? q[h][i] : 0.0f;
  }
}

// the compact layout's disconnect masks applied (branch-free) to the lane's elements k .. k + VEC - 1
// of a chunk, then their nonzero count (NaN counts, -0.0 does not: torch's nonzero)
template <int VEC>
__device__ __forceinline__ int mask_count(const AdjSrc& s, const MaskRegs M, int k, float (&v)[VEC]) {
  if (M.on) {   // wave-uniform
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const int r = row_of(k + i, s.inv_e);
      v[i] = mask_val(v[i], M, r, k + i - r * s.E);
    }
  }
  int c = 0;
#pragma unroll
  for (int i = 0; i < VEC; ++i) c += v[i] != 0.0f;
  return c;
}

__device__ __forceinline__ uint32_t below(uint64_t bal) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

template <int VEC, int NB>
__global__ __launch_bounds__(256) void edge_count_kernel(AdjSrc s, int64_t* __restrict__ counts,
                                                         int64_t* __restrict__ offsets) {
  const int64_t b = (int64_t)blockIdx.x * GRAPHS_PER_BLOCK + (threadIdx.x >> 6);
  if (b >= s.B) return;   // whole wave exits together
  const float* g = graph_ptr(s, b);
  const MaskRegs M = load_masks(s.masks ? s.masks + b * s.W : nullptr, s.W);
  const int EE = s.E * s.E;
  int cnt = 0;
  for (int k0 = 0; k0 < EE; k0 += WAVE * VEC * NB) {
    float v[CH][VEC];
    load_batch<VEC, NB>(g, k0, EE, v);
#pragma unroll
    for (int h = 0; h < NB; ++h) {
      const int c = mask_count<VEC>(s, M, k0 + h * WAVE * VEC + VEC * lane_id(), v[h]);
      if (VEC == 1) {
        cnt += __popcll(__ballot(c != 0));
      } else {
        cnt += __popcll(__ballot(c & 1)) + 2 * __popcll(__ballot(c & 2)) + 4 * __popcll(__ballot(c & 4));
      }
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
template <int VEC, int NB>
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
  for (int kb = 0; kb < EE && (bad || pos < end); kb += WAVE * VEC * NB) {
  float vb[CH][VEC];
  load_batch<VEC, NB>(g, kb, EE, vb);
#pragma unroll
  for (int h = 0; h < NB; ++h) {
    const int k0 = kb + h * WAVE * VEC;
    if (k0 >= EE || !(bad || pos < end)) break;   // wave-uniform
    const int k = k0 + VEC * lane;
    float (&v)[VEC] = vb[h];
    const int c = mask_count<VEC>(s, M, k, v);
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

// chunks per memory round trip of the compact layout's kernels (the reference layout's: CH)
#ifndef LSM_EDGES_COMPACT_NB
#define LSM_EDGES_COMPACT_NB CH
#endif
template <int VEC>
void launch_count(const AdjSrc& s, int64_t blocks, int64_t* counts, int64_t* offsets, hipStream_t st) {
  if (s.masks) edge_count_kernel<VEC, LSM_EDGES_COMPACT_NB><<<dim3((unsigned)blocks), 256, 0, st>>>(s, counts, offsets);
  else edge_count_kernel<VEC, CH><<<dim3((unsigned)blocks), 256, 0, st>>>(s, counts, offsets);
}

template <int VEC>
void launch_emit(const AdjSrc& s, int64_t blocks, const int64_t* offsets, int64_t nnz, int64_t cap,
                 int64_t* edge_index, float* edge_attr, int64_t* bad, hipStream_t st) {
  if (s.masks)
    edge_emit_kernel<VEC, LSM_EDGES_COMPACT_NB><<<dim3((unsigned)blocks), 256, 0, st>>>(s, offsets, nnz, cap, edge_index,
                                                                                    edge_attr, bad);
  else
    edge_emit_kernel<VEC, CH><<<dim3((unsigned)blocks), 256, 0, st>>>(s, offsets, nnz, cap, edge_index, edge_attr, bad);
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
  if (E % 2 == 0) launch_count<4>(s, blocks, counts, offsets, st);
  else launch_count<1>(s, blocks, counts, offsets, st);
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
    launch_emit<4>(s, blocks, offsets, nnz, nnz, edge_index, edge_attr, nullptr, (hipStream_t)stream);
  else
    launch_emit<1>(s, blocks, offsets, nnz, nnz, edge_index, edge_attr, nullptr, (hipStream_t)stream);
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
    launch_emit<4>(s, blocks, offsets, -1, cap, edge_index, edge_attr, nullptr, (hipStream_t)stream);
  else
    launch_emit<1>(s, blocks, offsets, -1, cap, edge_index, edge_attr, nullptr, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? 0 : fail("launch failed");
}

// offsets[B], offsets[B + 1] -> host through a per-thread pinned staging pair: a D2H copy into
// pageable memory is staged by the runtime (a second synchronisation and a host copy) -- the one-pass
// call's host time (profiles/r06_s05_bench_edges.json: 34 us of 101 us per call)
static int read_pair(const int64_t* dev, int64_t* host, hipStream_t st) {
  static thread_local int64_t* pinned = nullptr;
  if (!pinned && hipHostMalloc((void**)&pinned, 2 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) {
    pinned = nullptr;
    return fail("pinned staging allocation failed");
  }
  if (hipMemcpyAsync(pinned, dev, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail("reading the edge count failed");
  host[0] = pinned[0];
  host[1] = pinned[1];
  return 0;
}

int lsm_edges_scan_emit(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                        const int64_t* counts, int64_t* offsets, void* workspace, size_t workspace_bytes, int64_t cap,
                        int64_t* edge_index, float* edge_attr, int64_t* host_nnz_bad, void* stream) {
  AdjSrc s;
  if (make_src(adj, masks, B, E, N, &s)) return 1;
  if (B > INT32_MAX) return fail("B exceeds the scan's int32 item count");
  if (!counts || !offsets) return fail("counts / offsets is null");
  if (cap < 0) return fail("cap < 0");
  if (cap > 0 && (!edge_index || !edge_attr)) return fail("edge_index / edge_attr is null");
  if (workspace_bytes < lsm_edges_workspace_bytes(B)) return fail("workspace too small");
  hipStream_t st = (hipStream_t)stream;
  offsets_init_kernel<<<1, 64, 0, st>>>(offsets, B);
  if (B == 0) {
    if (hipGetLastError() != hipSuccess) return fail("launch failed");
    return host_nnz_bad ? read_pair(offsets, host_nnz_bad, st) : 0;
  }
  const size_t cbytes = ((size_t)B * sizeof(int64_t) + 255) & ~(size_t)255;
  void* temp = (char*)workspace + cbytes;
  size_t tbytes = workspace_bytes - cbytes;
  if (hipcub::DeviceScan::InclusiveSum(temp, tbytes, counts, offsets + 1, (int)B, st) != hipSuccess)
    return fail("scan failed");
  if (cap > 0) {
    const int64_t blocks = (B + GRAPHS_PER_BLOCK - 1) / GRAPHS_PER_BLOCK;
    // the scan above rewrote offsets[B]; the error word offsets[B + 1] was cleared before it
    if (E % 2 == 0)
      launch_emit<4>(s, blocks, offsets, -1, cap, edge_index, edge_attr, offsets + B + 1, st);
    else
      launch_emit<1>(s, blocks, offsets, -1, cap, edge_index, edge_attr, offsets + B + 1, st);
  }
  if (hipGetLastError() != hipSuccess) return fail("launch failed");
  // the call's one synchronisation (torch.nonzero's): offsets[B], offsets[B + 1]
  return host_nnz_bad ? read_pair(offsets + B, host_nnz_bad, st) : 0;
}

}  // extern "C"
